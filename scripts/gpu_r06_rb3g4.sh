# Round 6: the bf16 128-channel kernel-3 whole block on 256-column tiles of 8 waves of 32 x 128
# (TTS_MI355X_RB3_GEO128=4) -- bf16 tests under it, then an A/B of the bf16 step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TTS_MI355X_RB3_GEO128=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_bf16_planes_gpu.py tests/test_hifigan_gpu.py -m gpu -k "bf16 or planes or block" -p no:cacheprovider > gpurun_out/rb3g4_pytest.log 2>&1 ||
  { tail -30 gpurun_out/rb3g4_pytest.log; exit 1; }
tail -1 gpurun_out/rb3g4_pytest.log
AB_NOTEST=1 AB_FILTER="block" AB_BENCH_ARGS="--math-mode bf16" \
  AB="main:main g4:main|TTS_MI355X_RB3_GEO128=4" bash scripts/ab_lib_env.sh
