# Round 6: bf16 128 / 256-channel pairs on 8 waves of 32 rows x 128 columns (GEO 7 / 8: a weight
# fragment feeds 4 MFMAs) against the default GEO 5 / 6 -- bf16 tests under them, then an A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TTS_MI355X_PAIR128_GEO=7 TTS_MI355X_PAIR256_GEO=8 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_bf16_planes_gpu.py -m gpu -p no:cacheprovider > gpurun_out/pair78_pytest.log 2>&1 ||
  { tail -30 gpurun_out/pair78_pytest.log; exit 1; }
tail -1 gpurun_out/pair78_pytest.log
AB_NOTEST=1 AB_FILTER="c128|c256" AB_BENCH_ARGS="--math-mode bf16" \
  AB="main:main g7:main|TTS_MI355X_PAIR128_GEO=7 g8:main|TTS_MI355X_PAIR256_GEO=8" bash scripts/ab_lib_env.sh
