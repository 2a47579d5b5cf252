# Round 4 checkpoint in one box session: the GPU test suite (parity errors logged), then the
# driver's bench command (default: whole-batch CPU baseline included)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors.jsonl
rm -f $TTS_ERRLOG
timeout -k 10 1000 python -u -m pytest -q --maxfail=10 --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests ${TESTS_EXTRA} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR|Error:|assert " gpurun_out/pytest_gpu.log | head -30; exit $rc; }
unset TTS_ERRLOG
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['ms_per_step'],d['value'],d['build']);print(d['roofline']);print(d['cpu_baseline'])"
[ -n "$NO_REHEARSE" ] && exit 0
# config-4 / config-5 sharded legs over a one-rank RCCL group (the N > 1 code path on one GPU)
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --no-glow --no-e2e --no-xtts --rehearse-sharded > gpurun_out/bench_rehearse.json 2> gpurun_out/bench_rehearse.err || { tail -20 gpurun_out/bench_rehearse.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_rehearse.json'));print(d.get('sharded_rehearsal'));print(d.get('config5_sharded_rehearsal'))"
