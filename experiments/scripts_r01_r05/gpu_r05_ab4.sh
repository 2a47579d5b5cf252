# A/B (one box session): HEAD~ library (c40), the restructured Winograd epilogue without (pk0) and
# with packed fp32 math (main), and the transform jobs on the DMA waves (tg1), after the GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
AB_NOTEST=1 AB="c40:abx/lib_c40.so pk0:abx/lib_pk0.so main:main tg1:abx/lib_tg1.so" AB_FILTER="wino" bash scripts/ab_lib_env.sh
