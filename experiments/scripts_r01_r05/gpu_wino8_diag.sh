# 8-wave Winograd diagnostics: ablation builds (ab/lib_wa<N>.so) + SQ counters of the product build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/w8
AB_NOBENCH=1 AB_LIBS="${W8_LIBS:-wa2 wa8 wa16 wa18 wa24 wa32}" AB_TILES=21 AB_SHAPES="c128_k11 c128_k7" bash scripts/gpu_ab_lib.sh > gpurun_out/w8/ablate.log 2>&1 || exit 1
OUT=gpurun_out/w8
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $OUT/p -o pm --output-format csv -- python3 scripts/wino_op.py 21 128 11 3 0 3 > $OUT/p.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES -d $OUT/q -o pm --output-format csv -- python3 scripts/wino_op.py 21 128 11 3 0 3 > $OUT/q.log 2>&1
