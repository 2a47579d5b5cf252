# SQ counters of the Winograd conv vs the direct tile on c128 k11 d3 (separate passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/wpmc
mkdir -p $OUT
for tile in 21 13; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $OUT/t$tile -o tr --output-format csv -- python3 scripts/wino_op.py $tile 128 11 3 0 3 > $OUT/t$tile.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $OUT/p$tile -o pm --output-format csv -- python3 scripts/wino_op.py $tile 128 11 3 0 3 > $OUT/p$tile.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES -d $OUT/q$tile -o pm --output-format csv -- python3 scripts/wino_op.py $tile 128 11 3 0 3 > $OUT/q$tile.log 2>&1 || exit 1
done
find $OUT -name "*.csv" | head -30
