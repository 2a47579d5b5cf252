# rocprofv3 evidence for the bench workload (default math mode): kernel trace + stats, then
# separate PMC passes (HBM bytes: FETCH_SIZE and WRITE_SIZE in their own passes; SQ counters),
# then the per-family traffic table (scripts/traffic_from_pmc.py) and the MFMA-busy table
# (scripts/mfma_from_pmc.py).  ROUND names the output files (default r03).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof
MODE=${PROF_MODE:-f16x3}
ROUND=${ROUND:-r03}
mkdir -p $OUT
BENCH="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits --no-vits-tts --no-rb2 --math-mode $MODE"
export TTS_FORWARD_NAMES=$OUT/forward_names.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 $BENCH > $OUT/trace.log 2>&1 &&
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 $BENCH > $OUT/fetch.log 2>&1 &&
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 $BENCH > $OUT/write.log 2>&1 &&
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o sq --output-format csv -- python3 $BENCH > $OUT/sq.log 2>&1 &&
python3 scripts/traffic_from_pmc.py $OUT $MODE $OUT/traffic_hifigan_$ROUND.json &&
python3 scripts/mfma_from_pmc.py $OUT $MODE $OUT/mfma_busy_$ROUND.json
rc=$?
echo "profile rc=$rc"
find $OUT -name "*.csv" | head -20
exit $rc
