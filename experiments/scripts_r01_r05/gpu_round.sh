set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 8 > gpurun_out/bench.json 2> gpurun_out/bench.err
  echo "bench rc=$?" >> gpurun_out/bench.err
fi
tail -5 gpurun_out/pytest_gpu.log; cat gpurun_out/bench.json
