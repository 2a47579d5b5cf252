# Round 6: bf16 256-channel kernel-11 ResBlock1 iterations as 8-wave pairs (TTS_MI355X_PAIR256_K11=1)
# against the Winograd per-conv launches -- the bf16 tests under it, then an interleaved A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TTS_MI355X_PAIR256_K11=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_bf16_planes_gpu.py tests/test_hifigan_gpu.py -m gpu -k "bf16 or planes" -p no:cacheprovider > gpurun_out/p256k11_pytest.log 2>&1 ||
  { tail -30 gpurun_out/p256k11_pytest.log; exit 1; }
tail -1 gpurun_out/p256k11_pytest.log
AB_NOTEST=1 AB_FILTER=c256 AB_BENCH_ARGS="--math-mode bf16" \
  AB="main:main k11p:main|TTS_MI355X_PAIR256_K11=1" bash scripts/ab_lib_env.sh
