# rocprofv3 evidence for the bench workload: kernel trace + stats, then separate PMC passes
# (HBM bytes: FETCH_SIZE / WRITE_SIZE in their own passes; SQ occupancy/stall counters).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
BENCH="bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 $BENCH > $OUT/trace.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 $BENCH > $OUT/fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 $BENCH > $OUT/write.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o sq --output-format csv -- python3 $BENCH > $OUT/sq.log 2>&1
rc=$?
echo "profile rc=$rc"
find $OUT -name "*.csv" | head -20
exit $rc
