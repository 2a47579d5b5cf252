# Round-5 closing evidence on the final tree (one box session): the whole GPU suite, then the
# profile set of scripts/gpu_r05_profiles.sh (kernel trace + stats, FETCH / WRITE / SQ passes,
# per-family counters, the default bench line with its traffic and MFMA-busy tables)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
unset TTS_ERRLOG
bash scripts/gpu_r05_profiles.sh
