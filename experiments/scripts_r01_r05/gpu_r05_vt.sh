# VITS text side GPU tests, then the bf16 profiling evidence (scripts/gpu_r05_bf16prof.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors_vt.jsonl
timeout -k 10 600 python -u -m pytest tests/test_vits_text_gpu.py tests/test_glow_tts_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_vt.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_vt.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r05_bf16prof.sh
