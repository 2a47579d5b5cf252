# Execution lanes: the GPU suite (incl. the schedule-equivalence test), then an interleaved A/B of
# MRF branch streams x sub-batches on the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors.jsonl
timeout -k 10 300 python -u -m pytest tests/test_hifigan_gpu.py -k concurrent -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_lanes.log 2>&1 || { tail -30 gpurun_out/pytest_lanes.log; exit 1; }
tail -1 gpurun_out/pytest_lanes.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
AB_NOTEST=1 AB="s3b1:main s3b2:main|TTS_MI355X_SUBBATCH=2 s2b2:main|TTS_MI355X_SUBBATCH=2,TTS_MI355X_MRF_STREAMS=2 s1b2:main|TTS_MI355X_SUBBATCH=2,TTS_MI355X_MRF_STREAMS=1 s1b4:main|TTS_MI355X_SUBBATCH=4,TTS_MI355X_MRF_STREAMS=1" AB_FILTER="zzz" bash scripts/ab_lib_env.sh || exit 1
