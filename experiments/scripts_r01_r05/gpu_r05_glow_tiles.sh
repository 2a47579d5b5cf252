# Glow decoder side line: tile sweep of the flow convs (TTS_MI355X_FLOW_TILE_K for the k5 in_layers,
# TTS_MI355X_FLOW_TILE_1X1 for start / res_skip / end), after the Glow GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_glow_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_glow.log 2>&1 || { tail -30 gpurun_out/pytest_glow.log; exit 1; }
tail -1 gpurun_out/pytest_glow.log
for v in ${GLOW_TILE_VARIANTS:-"-:-" "7:-" "10:-" "18:-" "8:-" "16:-" "17:-" "-:16" "-:18" "-:10" "-:-"}; do
  k=${v%%:*}; p=${v#*:}; [ "$k" = - ] && k=""; [ "$p" = - ] && p=""
  TTS_MI355X_FLOW_TILE_K=$k TTS_MI355X_FLOW_TILE_1X1=$p timeout -k 10 300 python scripts/glow_ab.py f16x3 bf16 > gpurun_out/glow_tile.json 2> gpurun_out/glow_tile.err || { tail -20 gpurun_out/glow_tile.err; exit 1; }
  echo "K=$k 1x1=$p: $(cat gpurun_out/glow_tile.json | tr '\n' ' ')"
done
