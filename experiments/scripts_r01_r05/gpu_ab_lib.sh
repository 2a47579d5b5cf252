# A/B of library builds (ab/lib_<name>.so vs the product build), same box session:
# op timing of the bench shapes (tile 21 Winograd vs direct 13) and the default bench forward
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BENCH="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits"
for v in main $AB_LIBS main $AB_LIBS; do
  lib=tts-3_amd/tts_amd/_lib/libtts_mi355x.so; [ $v = main ] || lib=ab/lib_$v.so
  echo "== $v"
  if [ -n "$AB_SHAPES" ]; then
    TTS_MI355X_LIB=$lib TUNE_TILES=${AB_TILES:-21,13} timeout -k 10 200 python scripts/tune_conv.py f16x3 $AB_SHAPES 2>&1 | grep -v amdgpu.ids || exit 1
  fi
  [ -n "$AB_NOBENCH" ] && continue
  TTS_MI355X_LIB=$lib timeout -k 10 200 python $BENCH > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v',round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],2),'ms');print({k:v for k,v in d['kernel_breakdown_ms'].items()})"
done 2>&1 | tee gpurun_out/ab_lib.log
