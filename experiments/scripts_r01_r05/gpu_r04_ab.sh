# Round 4 kernel iteration in one box session: the HiFiGAN GPU tests on the in-tree library, an
# interleaved A/B of the bench forward against ab/lib_base.so (previous tree), then one PMC pass of
# LDS / wait counters per kernel family (both libraries)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$AB_SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_hifigan_gpu.py ${AB_TESTS} > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
  tail -1 gpurun_out/ab_pytest.log
fi
B="bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits"
VARS=${AB_VARIANTS:-base new}
for r in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in $VARS; do
    lib=tts-3_amd/tts_amd/_lib/libtts_mi355x.so; [ $v != new ] && lib=ab/lib_$v.so
    TTS_MI355X_LIB=$lib timeout -k 10 200 python $B > gpurun_out/ab_${v}_$r.json 2> gpurun_out/ab_${v}_$r.err || { tail -5 gpurun_out/ab_${v}_$r.err; exit 1; }
    python -c "
import json,re;d=json.load(open('gpurun_out/ab_${v}_$r.json'));b=d['kernel_breakdown_ms']
print('${v}_$r', round(d['ms_per_step'],2), {k: round(v,2) for k,v in b.items() if re.search('${AB_FILTER:-wino|block|pair|ups}', k)})"
  done
done
[ -n "$NO_PMC" ] && exit 0
P="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits"
for v in ${PMC_VARIANTS:-$VARS}; do
  lib=tts-3_amd/tts_amd/_lib/libtts_mi355x.so; [ $v != new ] && lib=ab/lib_$v.so
  OUT=gpurun_out/pmc_$v; mkdir -p $OUT
  export TTS_FORWARD_NAMES=$OUT/forward_names.json
  TTS_MI355X_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/p1 -o p1 --output-format csv -- python3 $P > $OUT/p1.log 2>&1 || { echo "pmc $v failed"; tail -5 $OUT/p1.log; exit 1; }
  python3 scripts/pmc_families.py $OUT p1 > $OUT/table.txt && grep -E "family|wino|block|pair|ups" $OUT/table.txt
done
