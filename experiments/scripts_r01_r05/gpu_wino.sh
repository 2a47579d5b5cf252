# Winograd F(4,4) conv: op + generator parity, then the default bench with and without it (A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hifigan_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "winograd or accuracy or c1 or c2 or golden" > gpurun_out/pytest_wino.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_wino.log
tail -15 gpurun_out/pytest_wino.log
[ $rc -le 1 ] || exit $rc
BENCH="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits"
timeout -k 10 300 python $BENCH > gpurun_out/bench_wino.json 2> gpurun_out/bench_wino.err &&
TTS_MI355X_WINO=0 timeout -k 10 300 python $BENCH > gpurun_out/bench_direct.json 2> gpurun_out/bench_direct.err
rc=$?
for f in bench_wino bench_direct; do
  python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f',d['value'],d['ms_per_step'],d['accuracy_vs_fp64_oracle'] if 'accuracy_vs_fp64_oracle' in d else '');print({k:v for k,v in d['kernel_breakdown_ms'].items() if 'c128' in k or 'c256' in k})"
done
exit $rc
