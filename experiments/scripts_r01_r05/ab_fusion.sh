# A/B of the fused resblock iterations (default) against separate conv launches
# (TTS_MI355X_NO_PAIR_FUSION=1), interleaved in one GPU session.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
  for v in fused split; do
    if [ $v = split ]; then export TTS_MI355X_NO_PAIR_FUSION=1; else unset TTS_MI355X_NO_PAIR_FUSION; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow ${AB_ARGS} > gpurun_out/abf_${v}_$r.json 2>gpurun_out/abf_${v}_$r.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/abf_${v}_$r.json'));print('$v', round(d['ms_per_step'],2), {k: round(v,2) for k,v in list(d['kernel_breakdown_ms'].items())[:10]})"
  done
done
