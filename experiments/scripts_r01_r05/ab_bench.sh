# A/B the committed library (ab/lib_old.so) against the working tree (ab/lib_new.so) in ONE
# GPU session, interleaved, so device-to-device variation cancels out.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MODES=${AB_MODES:-"fp32x6 fp32"}
for r in 1 2; do
  for m in $MODES; do
    for v in old new; do
      TTS_MI355X_LIB=ab/lib_$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --math-mode $m > gpurun_out/ab_${v}_${m}_$r.json 2>gpurun_out/ab_${v}_${m}_$r.err || exit 1
      python -c "import json;d=json.load(open('gpurun_out/ab_${v}_${m}_$r.json'));print('$v', '$m', round(d['ms_per_step'],2), {k: round(v,2) for k,v in list(d['kernel_breakdown_ms'].items())[:8]})"
    done
  done
done
