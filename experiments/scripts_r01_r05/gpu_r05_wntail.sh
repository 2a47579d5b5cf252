# The reverse flows' tail + next start conv inside the last WN layer's launch: the Glow / Glow-TTS /
# config GPU tests, then the decoder side line with and without it (TTS_MI355X_WN_TAIL)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_glow_gpu.py tests/test_glow_tts_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_wntail.log 2>&1 || { tail -40 gpurun_out/pytest_wntail.log; exit 1; }
tail -1 gpurun_out/pytest_wntail.log
for r in 1 2; do
  for v in 1 0; do
    TTS_MI355X_WN_TAIL=$v timeout -k 10 300 python scripts/glow_ab.py f16x3 bf16 > gpurun_out/wn_tail.json 2> gpurun_out/wn_tail.err || { tail -20 gpurun_out/wn_tail.err; exit 1; }
    echo "WN_TAIL=$v round $r: $(cat gpurun_out/wn_tail.json | tr '\n' ' ')"
  done
done
