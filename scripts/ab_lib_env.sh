# Interleaved A/B over (library, environment) variants on the default bench, after the HiFiGAN GPU tests:
#   AB="main:main|X=1 slp:abx/lib_slp.so|X=0" bash scripts/ab_lib_env.sh   (AB_BENCH_ARGS: extra bench flags)
# variant syntax name:LIB|ENV1,ENV2 (LIB "main" = the in-tree library); prints ms/step and the
# kernel families matching $AB_FILTER
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "$AB_NOTEST" ]; then
  timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hifigan_gpu.py -m gpu -p no:cacheprovider > gpurun_out/ab_pytest.log 2>&1 || { tail -20 gpurun_out/ab_pytest.log; exit 1; }
  tail -1 gpurun_out/ab_pytest.log
fi
for r in 1 2; do
  for v in $AB; do
    name=${v%%:*}; rest=${v#*:}; lib=${rest%%|*}; envs=${rest#*|}; [ "$envs" = "$rest" ] && envs=""
    [ "$lib" = main ] && lib=tts-3_amd/tts_amd/_lib/libtts_mi355x.so
    env TTS_MI355X_LIB=$lib ${envs//,/ } timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits --no-vits-tts --no-rb2 ${AB_BENCH_ARGS} > gpurun_out/ab_${name}_$r.json 2>gpurun_out/ab_${name}_$r.err || exit 1
    python -c "
import json,re;d=json.load(open('gpurun_out/ab_${name}_$r.json'));b=d['kernel_breakdown_ms']
print('${name}_$r', round(d['ms_per_step'],2), {k: round(v,2) for k,v in b.items() if re.search('${AB_FILTER:-.}', k)})"
  done
done
