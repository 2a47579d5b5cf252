# Round-6 final tree (third session), part B: the bf16 serial-schedule PMC tables (the bf16 pairs
# changed geometry) and the default bench line under rocprofv3 --kernel-trace --stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/prof
TTS_MI355X_SUBBATCH=1 TTS_MI355X_MRF_STREAMS=1 PROF_MODE=bf16 ROUND=r06_bf16 bash scripts/profile_round.sh > gpurun_out/profile_r06_bf16.log 2>&1 ||
  { tail -20 gpurun_out/profile_r06_bf16.log; exit 1; }
tail -1 gpurun_out/profile_r06_bf16.log
rm -rf $P/fetch $P/write $P/sq
J="--traffic-json profiles/traffic_hifigan_r06.json --mfma-json profiles/mfma_busy_r06.json"
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/benchprof -o bench --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 $J > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err ||
  { tail -20 gpurun_out/bench_prof.err; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/bench_prof.json').read().strip().splitlines()[-1])
print('bench under rocprofv3', d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('avg_launch_ms'), d['roofline'].get('traffic'))
"
find gpurun_out/benchprof -name "*kernel_stats.csv" | head -3
