# Round 6: bf16 128 / 256-channel ResBlock1 pairs on 8 waves (two per SIMD; TTS_MI355X_PAIR128_GEO=5,
# TTS_MI355X_PAIR256_GEO=6) -- the bf16 GPU tests under both, then an interleaved A/B of the bf16 step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TTS_MI355X_PAIR128_GEO=5 TTS_MI355X_PAIR256_GEO=6 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_bf16_planes_gpu.py tests/test_hifigan_gpu.py -m gpu -k "bf16 or planes" -p no:cacheprovider > gpurun_out/pair8w_pytest.log 2>&1 ||
  { tail -30 gpurun_out/pair8w_pytest.log; exit 1; }
tail -1 gpurun_out/pair8w_pytest.log
AB_NOTEST=1 AB_FILTER=pair_k AB_BENCH_ARGS="--math-mode bf16" \
  AB="main:main g5:main|TTS_MI355X_PAIR128_GEO=5 g6:main|TTS_MI355X_PAIR256_GEO=6 g56:main|TTS_MI355X_PAIR128_GEO=5,TTS_MI355X_PAIR256_GEO=6" \
  bash scripts/ab_lib_env.sh
