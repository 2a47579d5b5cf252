# One-launch WaveNet layer (kernels_glow_wn.hip): the Glow GPU tests (incl. the fused-vs-unfused
# and oracle tests), then an interleaved A/B of the Glow decoder side line with and without it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_glow_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_wnlayer.log 2>&1 || { tail -40 gpurun_out/pytest_wnlayer.log; exit 1; }
tail -1 gpurun_out/pytest_wnlayer.log
for r in 1 2; do
  for v in 1 0; do
    TTS_MI355X_WN_LAYER=$v timeout -k 10 300 python scripts/glow_ab.py f16x3 bf16 > gpurun_out/wn_ab.json 2> gpurun_out/wn_ab.err || { tail -20 gpurun_out/wn_ab.err; exit 1; }
    echo "WN_LAYER=$v round $r: $(cat gpurun_out/wn_ab.json | tr '\n' ' ')"
  done
done
