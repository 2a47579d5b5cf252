# Round 6: the bf16 32-channel pairs as 2 waves of 32 x 128 (TTS_MI355X_PAIR32_GEO=9) -- bf16 tests
# under it, then an A/B of the bf16 step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TTS_MI355X_PAIR32_GEO=9 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_bf16_planes_gpu.py tests/test_hifigan_gpu.py -m gpu -k "bf16 or planes" -p no:cacheprovider > gpurun_out/p32g9_pytest.log 2>&1 ||
  { tail -30 gpurun_out/p32g9_pytest.log; exit 1; }
tail -1 gpurun_out/p32g9_pytest.log
AB_NOTEST=1 AB_FILTER="c32" AB_BENCH_ARGS="--math-mode bf16" \
  AB="main:main g9:main|TTS_MI355X_PAIR32_GEO=9" bash scripts/ab_lib_env.sh
