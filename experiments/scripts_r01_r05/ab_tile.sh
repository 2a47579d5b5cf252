# A/B of the Cout > 64 f16x3 conv tile: HiFiGAN f16x3 tests under each candidate tile first
# (correctness), then the interleaved bench A/B of scripts/ab_env.sh.
#   TILES="13 20 21" [TILEVAR=TTS_MI355X_TILE_SHORT] bash scripts/ab_tile.sh
# TILEVAR: TTS_MI355X_TILE_BIG (default; every Cout > 64 conv) or TTS_MI355X_TILE_SHORT (kernel <= 3
# and the ConvTranspose layers only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
V=${TILEVAR:-TTS_MI355X_TILE_BIG}
for t in ${TILES:-13 20 21}; do
  env $V=$t timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_hifigan_gpu.py -m gpu -p no:cacheprovider -k "f16x3" > gpurun_out/tile_${t}_pytest.log 2>&1 \
    || { echo "tile $t tests failed"; tail -30 gpurun_out/tile_${t}_pytest.log; exit 1; }
  echo "tile $t: $(tail -1 gpurun_out/tile_${t}_pytest.log)"
done
AB=""
for t in ${TILES:-13 20 21}; do AB="$AB t$t:$V=$t"; done
AB="$AB" AB_FILTER="${AB_FILTER:-c128|c256}" bash scripts/ab_env.sh
