# Glow WN layer at 12 waves (H = 192): the flow GPU tests on the new default,
# then an interleaved A/B of the decoder side line against the four-wave form (TTS_MI355X_WN_WAVES=4)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_glow_gpu.py tests/test_vits_gpu.py tests/test_glow_tts_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_wn12.log 2>&1 || { tail -30 gpurun_out/pytest_wn12.log; exit 1; }
tail -2 gpurun_out/pytest_wn12.log
for r in 1 2 3; do
  for v in 12 4; do
    echo -n "waves=$v round $r: "
    TTS_MI355X_WN_WAVES=$v timeout -k 10 120 python scripts/glow_ab.py f16x3 bf16 2>/dev/null | tr '\n' ' ' || exit 1
    echo
  done
done
