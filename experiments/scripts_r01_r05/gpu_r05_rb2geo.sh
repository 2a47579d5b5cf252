# ResBlock2 at 64 channels: 128- vs 192-column whole-block tiles (TTS_MI355X_RB2_GEO64)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
for geo in 0 1; do
  TTS_MI355X_RB2_GEO64=$geo timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits --no-vits-tts > gpurun_out/rb2geo_$geo.json 2> gpurun_out/rb2geo_$geo.err || { tail -20 gpurun_out/rb2geo_$geo.err; exit 1; }
  python - $geo <<'PY'
import json, sys
r = json.loads(open(f"gpurun_out/rb2geo_{sys.argv[1]}.json").read().strip().splitlines()[-1])
for k, v in r["resblock2_decoder"]["variants"].items():
    if k.endswith("whole_block"):
        print("geo64", sys.argv[1], k, round(v["ms_per_step"], 2), {a: b for a, b in v["kernel_breakdown_ms"].items() if "c64" in a})
PY
done
done
