# Generic interleaved A/B of environment switches on the default bench (after the HiFiGAN GPU tests).
#   AB="on:TTS_MI355X_XCD_REMAP=1 off:TTS_MI355X_XCD_REMAP=0" bash scripts/ab_env.sh
# prints ms/step and the kernel families matching $AB_FILTER (regex, default: all) per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hifigan_gpu.py -m gpu -p no:cacheprovider > gpurun_out/ab_pytest.log 2>&1 || { tail -20 gpurun_out/ab_pytest.log; exit 1; }
tail -1 gpurun_out/ab_pytest.log
for r in 1 2; do
  for v in $AB; do
    name=${v%%:*}; envs=${v#*:}
    env ${envs//,/ } timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits > gpurun_out/ab_${name}_$r.json 2>gpurun_out/ab_${name}_$r.err || exit 1
    python -c "
import json,re;d=json.load(open('gpurun_out/ab_${name}_$r.json'));b=d['kernel_breakdown_ms']
print('${name}_$r', round(d['ms_per_step'],2), {k: round(v,2) for k,v in b.items() if re.search('${AB_FILTER:-.}', k)})"
  done
done
