set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  for m in fp32 fp32x6; do
    timeout -k 10 600 python scripts/tune_conv.py $m > gpurun_out/tune_$m.log 2>&1; echo "tune $m rc=$?"; cat gpurun_out/tune_$m.log | grep -v amdgpu.ids
  done
  for m in fp32 fp32x6; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --math-mode $m > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err
    echo "bench $m rc=$?"
    python -c "import json;d=json.load(open('gpurun_out/bench_$m.json'));print(d['math_mode'], d['value'],d['ms_per_step']);print(d['roofline']);print(d['kernel_breakdown_ms'])"
  done
fi
