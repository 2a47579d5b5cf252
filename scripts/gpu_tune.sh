set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 900 python scripts/tune_conv.py > gpurun_out/tune.log 2>&1
  echo "tune rc=$?"
  cat gpurun_out/tune.log
fi
