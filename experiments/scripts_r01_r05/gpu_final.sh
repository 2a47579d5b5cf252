# Round-end evidence in one box session: rocprofv3 trace + PMC passes of the bench workload
# (scripts/profile_round.sh), the traffic table into profiles/ (read by bench.py), then the GPU
# test suite and the default bench line (python bench.py, no flags: what the driver runs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -20 gpurun_out/profile_round.log; exit 1; }
cp gpurun_out/prof/traffic_hifigan.json profiles/traffic_hifigan_r02.json
cp profiles/traffic_hifigan_r02.json gpurun_out/traffic_hifigan_r02.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['ms_per_step'],d['value'],d['roofline'])"
