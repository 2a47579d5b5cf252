# Round 6: the whole GPU suite (every measured error logged) + smoke, one box session
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors_r06.jsonl
rm -f $TTS_ERRLOG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_r06.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_r06.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu_r06.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r06.log 2>&1 || { tail -20 gpurun_out/smoke_r06.log; exit 1; }
tail -1 gpurun_out/smoke_r06.log
