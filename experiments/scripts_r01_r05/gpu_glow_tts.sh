set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_glow_tts_gpu.py -m gpu -p no:cacheprovider > gpurun_out/pytest_glow_tts.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_glow_tts.log
exit $rc
