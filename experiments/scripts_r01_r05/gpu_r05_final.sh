# Round-5 evidence on the current tree (one box session): the whole GPU suite (errors logged), the
# default bench line, then the per-family PMC counter table in the serial schedule
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['ms_per_step'],d['value'],d['roofline']['frac']);print({k:(v or {}).get('variants', (v or {}).get('ms_per_step')) for k,v in d.items() if k in ('glow_decoder','xtts_decoder','vits_waveform')})"
[ -n "$NO_PMC" ] && exit 0
TTS_MI355X_SUBBATCH=1 TTS_MI355X_MRF_STREAMS=1 bash scripts/gpu_pmc_families.sh \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_COUNT GRBM_GUI_ACTIVE" \
  "SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" > gpurun_out/pmc_families.log 2>&1 || { tail -20 gpurun_out/pmc_families.log; exit 1; }
tail -22 gpurun_out/pmc_families.log
