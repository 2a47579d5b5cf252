# Round 4: GPU suite on the in-tree library (fail fast), then the A/B against ab/lib_base.so and
# the LDS / wait counter pass (scripts/gpu_r04_ab.sh without its HiFiGAN test step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors.jsonl
rm -f $TTS_ERRLOG
timeout -k 10 900 python -u -m pytest -q --maxfail=10 --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR|Error:|assert " gpurun_out/pytest_gpu.log | head -40; exit $rc; }
unset TTS_ERRLOG
AB_SKIP_TESTS=1 bash scripts/gpu_r04_ab.sh
