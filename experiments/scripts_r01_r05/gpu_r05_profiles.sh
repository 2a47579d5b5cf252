# Round 5 profile evidence (one box session): rocprofv3 kernel trace + stats and the separate
# FETCH_SIZE / WRITE_SIZE / SQ passes of the bench workload (scripts/profile_round.sh, ROUND=r05)
# and the per-family counter table, all with the serial one-stream schedule (TTS_MI355X_SUBBATCH=1,
# TTS_MI355X_MRF_STREAMS=1: per-family launch times as in earlier rounds, the forward's dispatches
# in executor order); then the default bench line (concurrent lanes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_MI355X_SUBBATCH=1 TTS_MI355X_MRF_STREAMS=1
ROUND=r05 bash scripts/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -30 gpurun_out/profile_round.log; exit 1; }
tail -5 gpurun_out/profile_round.log
bash scripts/gpu_pmc_families.sh \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_COUNT GRBM_GUI_ACTIVE" \
  "SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" > gpurun_out/pmc_families.log 2>&1 || { tail -20 gpurun_out/pmc_families.log; exit 1; }
tail -25 gpurun_out/pmc_families.log
unset TTS_MI355X_SUBBATCH TTS_MI355X_MRF_STREAMS
timeout -k 10 600 python bench.py --traffic-json gpurun_out/prof/traffic_hifigan_r05.json --mfma-json gpurun_out/prof/mfma_busy_r05.json > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['ms_per_step'],d['value'],d['roofline']);print({k:(v or {}).get('variants', (v or {}).get('ms_per_step')) for k,v in d.items() if k in ('glow_decoder','xtts_decoder')})"
