# Round 3 evidence in one box session: GPU test suite (parity errors logged), the driver's bench
# command, then the rocprofv3 trace + PMC passes (traffic and MFMA-busy tables) of the bench workload
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors.jsonl
rm -f $TTS_ERRLOG
timeout -k 10 900 python -u -m pytest -q --maxfail=10 --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR|Error:|assert " gpurun_out/pytest_gpu.log | head -30; exit $rc; }
unset TTS_ERRLOG
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['ms_per_step'],d['value'],d['build']);print(d['roofline']);print(d['cpu_baseline'])"
[ -n "$NO_PROFILE" ] && exit 0
bash scripts/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -30 gpurun_out/profile_round.log; exit 1; }
tail -30 gpurun_out/profile_round.log
