# bf16 (configs 3 / 5): Winograd vs the direct conv for the k7 / k11 MRF convs at >= 128 channels.
# The bf16 Winograd kernels run at 0.11-0.16 MFMA busy (profiles/mfma_busy_r05_bf16.csv): one MFMA
# product per MAC leaves the transform VALU exposed.  Two interleaved rounds, one box session.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bf16w
B="bench.py --math-mode bf16 --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits-tts --no-rb2"
for r in 1 2; do
  for v in wino direct; do
    envs=""; [ $v = direct ] && envs="TTS_MI355X_WINO=0"
    env $envs timeout -k 10 300 python $B > gpurun_out/bf16w/${v}_$r.json 2> gpurun_out/bf16w/${v}_$r.err || { tail -5 gpurun_out/bf16w/${v}_$r.err; exit 1; }
    python - gpurun_out/bf16w/${v}_$r.json $v $r <<'PY'
import json, re, sys
d = json.load(open(sys.argv[1])); b = d["kernel_breakdown_ms"]; vw = d.get("vits_waveform") or {}
print(sys.argv[2], sys.argv[3], "step", round(d["ms_per_step"], 2), "serial", round(sum(b.values()), 2),
      "vits_waveform", vw.get("ms_per_step"), {k: round(v, 2) for k, v in b.items() if re.search("wino|mrf_conv_k(7|11)", k)})
PY
  done
done
