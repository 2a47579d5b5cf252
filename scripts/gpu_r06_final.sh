# Round-6 measurement pass on the final tree (one box session):
#  1. the serial-schedule PMC tables (scripts/profile_round.sh: kernel trace + FETCH / WRITE / SQ passes,
#     per-family traffic and MFMA-busy tables) -> gpurun_out/prof/*_r06.json
#  2. the default bench line (driver arguments) under rocprofv3 --kernel-trace --stats, whose stats must
#     agree with the line's hipEvent average for the dominant kernel
#  3. the default bench line without the profiler (the number of record on this box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/prof
TTS_MI355X_SUBBATCH=1 TTS_MI355X_MRF_STREAMS=1 ROUND=r06 bash scripts/profile_round.sh > gpurun_out/profile_r06.log 2>&1 ||
  { tail -20 gpurun_out/profile_r06.log; exit 1; }
tail -3 gpurun_out/profile_r06.log
J="--traffic-json $P/traffic_hifigan_r06.json --mfma-json $P/mfma_busy_r06.json"
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/benchprof -o bench --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 $J > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err ||
  { tail -20 gpurun_out/bench_prof.err; exit 1; }
timeout -k 10 700 python3 bench.py --gpus 1 --steps 20 --warmup 5 $J > gpurun_out/bench.json 2> gpurun_out/bench.err ||
  { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "
import json
for f in ('gpurun_out/bench_prof.json', 'gpurun_out/bench.json'):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline'].get('avg_launch_ms'))
"
