# Round-end evidence in one box session: rocprofv3 trace + PMC passes of the bench workload
# (scripts/profile_round.sh), the traffic table into profiles/ (read by bench.py), then the GPU
# test suite and the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -20 gpurun_out/profile_round.log; exit 1; }
cp gpurun_out/prof/traffic_hifigan.json profiles/traffic_hifigan_r01.json
cp profiles/traffic_hifigan_r01.json gpurun_out/traffic_hifigan_r01.json
bash scripts/gpu_round.sh
