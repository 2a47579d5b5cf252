# Glow decoder execution lanes: the Glow GPU tests (incl. lanes bitwise), then an interleaved A/B of
# the decoder side line at 1 / 2 / 3 / 4 lanes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_glow_gpu.py tests/test_glow_tts_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_glow.log 2>&1 || { tail -30 gpurun_out/pytest_glow.log; exit 1; }
tail -1 gpurun_out/pytest_glow.log
for r in 1 2; do
  for ln in 1 2 3 4; do
    TTS_MI355X_GLOW_LANES=$ln timeout -k 10 300 python scripts/glow_ab.py f16x3 bf16 > gpurun_out/glow_ab_${ln}_$r.json 2> gpurun_out/glow_ab_${ln}_$r.err || { tail -20 gpurun_out/glow_ab_${ln}_$r.err; exit 1; }
    echo "lanes=$ln round $r: $(cat gpurun_out/glow_ab_${ln}_$r.json | tr '\n' ' ')"
  done
done
