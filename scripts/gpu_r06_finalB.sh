# Round-6 final tree, part B: serial-schedule PMC tables for the f16x3 (headline) and the bf16 forwards
# (scripts/profile_round.sh: kernel trace + FETCH / WRITE / SQ passes -> traffic and MFMA-busy tables),
# then the default bench line under rocprofv3 --kernel-trace --stats with the fresh tables
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/prof
TTS_MI355X_SUBBATCH=1 TTS_MI355X_MRF_STREAMS=1 ROUND=r06 bash scripts/profile_round.sh > gpurun_out/profile_r06.log 2>&1 ||
  { tail -20 gpurun_out/profile_r06.log; exit 1; }
tail -1 gpurun_out/profile_r06.log
mkdir -p gpurun_out/prof16 && mv $P/trace gpurun_out/prof16/trace_f16x3 && rm -rf $P/fetch $P/write $P/sq
TTS_MI355X_SUBBATCH=1 TTS_MI355X_MRF_STREAMS=1 PROF_MODE=bf16 ROUND=r06_bf16 bash scripts/profile_round.sh > gpurun_out/profile_r06_bf16.log 2>&1 ||
  { tail -20 gpurun_out/profile_r06_bf16.log; exit 1; }
tail -1 gpurun_out/profile_r06_bf16.log
mv $P/trace gpurun_out/prof16/trace_bf16 && rm -rf $P/fetch $P/write $P/sq
J="--traffic-json $P/traffic_hifigan_r06.json --mfma-json $P/mfma_busy_r06.json"
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/benchprof -o bench --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 $J > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err ||
  { tail -20 gpurun_out/bench_prof.err; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/bench_prof.json').read().strip().splitlines()[-1])
print('bench under rocprofv3', d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('avg_launch_ms'), d['roofline'].get('traffic'))
"
find gpurun_out/benchprof -name "*kernel_stats.csv" | head -3
