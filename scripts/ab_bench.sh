# A/B the committed library (ab/lib_old.so) against the working tree (ab/lib_new.so) in ONE
# GPU session, interleaved, so device-to-device variation cancels out.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
  for v in old new; do
    TTS_MI355X_LIB=ab/lib_$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --math-mode fp32 > gpurun_out/ab_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_${v}_$r.json'));print('$v', 'fp32', round(d['ms_per_step'],2), {k: round(v,2) for k,v in list(d['kernel_breakdown_ms'].items())[:6]})"
  done
  TTS_MI355X_LIB=ab/lib_new.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --math-mode fp32x6 > gpurun_out/ab_x6_$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_x6_$r.json'));print('new', 'x6', round(d['ms_per_step'],2), {k: round(v,2) for k,v in list(d['kernel_breakdown_ms'].items())[:6]})"
done
