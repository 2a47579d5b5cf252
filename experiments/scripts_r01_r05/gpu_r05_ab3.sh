# A/B (one box session): HEAD library (base), asm LDS-DMA in the Winograd kernel (asm), + kernel-11
# prefetch depth 2 (asmpd2), and the new default (asm DMA + no-NaN device flags: main), after the
# whole GPU suite on main
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
AB_NOTEST=1 AB="base:abx/lib_base.so asm:abx/lib_asm.so asmpd2:abx/lib_asmpd2.so main:main" AB_FILTER="wino|block_k3_c128|pair_k7_c32|block_k3_c32" bash scripts/ab_lib_env.sh
