# Round 4 profile evidence in one box session: rocprofv3 kernel trace + stats and the separate
# FETCH_SIZE / WRITE_SIZE / SQ passes of the bench workload (scripts/profile_round.sh, ROUND=r04),
# then the per-family counter table (scripts/gpu_pmc_families.sh: three passes within the
# per-block counter limits)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ROUND=r04 bash scripts/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -30 gpurun_out/profile_round.log; exit 1; }
tail -5 gpurun_out/profile_round.log
bash scripts/gpu_pmc_families.sh \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_COUNT GRBM_GUI_ACTIVE" \
  "SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" > gpurun_out/pmc_families.log 2>&1 || { tail -20 gpurun_out/pmc_families.log; exit 1; }
tail -25 gpurun_out/pmc_families.log
