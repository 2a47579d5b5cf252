# Round 3: the GPU test suite on the working tree (parity errors logged for gate calibration),
# then a short default-mode bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors.jsonl
rm -f $TTS_ERRLOG
timeout -k 10 900 python -u -m pytest -q --maxfail=10 --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  ${CHECK_TESTS:-tests} > gpurun_out/check_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/check_pytest.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR|Error:|assert " gpurun_out/check_pytest.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits \
  > gpurun_out/check_bench.json 2> gpurun_out/check_bench.err || { tail -20 gpurun_out/check_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/check_bench.json'));print(d['ms_per_step'],d['value'],d['build']);print(d['roofline']);print(d['kernel_breakdown_ms'])"
