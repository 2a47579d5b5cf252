# A/B (one box session): lane 1 starting after lane 0's first n MRF branches (TTS_MI355X_LANE_OFFSET)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hifigan_gpu.py -k "concurrent" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_lanes.log 2>&1 || { tail -30 gpurun_out/pytest_lanes.log; exit 1; }
tail -1 gpurun_out/pytest_lanes.log
AB_NOTEST=1 AB="off0:main off1:main|TTS_MI355X_LANE_OFFSET=1 off2:main|TTS_MI355X_LANE_OFFSET=2 off3:main|TTS_MI355X_LANE_OFFSET=3 off5:main|TTS_MI355X_LANE_OFFSET=5" AB_FILTER="zzz" bash scripts/ab_lib_env.sh || exit 1
