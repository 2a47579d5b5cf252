# PMC passes (separate, no tracing domains) on selected conv shapes via the tuning script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
ARGS="scripts/tune_conv.py fp32x6 c32_k3 c32_k11 c128_k11"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/p1 -o p1 --output-format csv -- python3 $ARGS > $OUT/p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_LEVEL_WAVES -d $OUT/p2 -o p2 --output-format csv -- python3 $ARGS > $OUT/p2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/p3 -o p3 --output-format csv -- python3 $ARGS > $OUT/p3.log 2>&1
echo "rc=$?"
