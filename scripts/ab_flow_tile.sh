# A/B of the Glow / VITS flow conv tile (TTS_MI355X_FLOW_TILE): the flow GPU tests under each tile,
# then interleaved bench runs printing the Glow decoder and VITS waveform side lines.
#   TILES="-1 16 18" bash scripts/ab_flow_tile.sh      (-1 = the default selection)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for t in ${TILES:--1 16 18}; do
  TTS_MI355X_FLOW_TILE=$t timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_glow_gpu.py tests/test_vits_gpu.py -m gpu -p no:cacheprovider -k "f16x3 or bf16" \
    > gpurun_out/flow_tile_${t}_pytest.log 2>&1 || { echo "tile $t tests failed"; tail -30 gpurun_out/flow_tile_${t}_pytest.log; exit 1; }
  echo "tile $t: $(tail -1 gpurun_out/flow_tile_${t}_pytest.log)"
done
for r in 1 2; do
  for t in ${TILES:--1 16 18}; do
    TTS_MI355X_FLOW_TILE=$t timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt --no-xtts \
      > gpurun_out/flow_ab_${t}_$r.json 2> gpurun_out/flow_ab_${t}_$r.err || exit 1
    python3 -c "
import json;d=json.load(open('gpurun_out/flow_ab_${t}_$r.json'));g=d['glow_decoder'];v=d['vits_waveform']['variants'];e=d['glow_tts_e2e']['variants']
print('tile ${t} run $r glow', round(g['ms_per_step'],3), {k: g['breakdown_ms'][k] for k in ('glow_wn_in','glow_wn_res_skip','glow_start','glow_end')}, 'vits', {k: round(x['ms_per_step'],2) for k,x in v.items()}, 'e2e', {k: round(x['glow_tts_inference_ms'],2) for k,x in e.items()})"
  done
done
