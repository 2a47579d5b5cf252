# Round-5 check in one box session: the GPU test suite (errors logged), then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['ms_per_step'],d['value'],d['roofline']['frac'],d['roofline']['avg_launch_ms']);print(d['kernel_breakdown_ms']);print({k:(v or {}).get('variants', (v or {}).get('ms_per_step')) for k,v in d.items() if k in ('glow_decoder','glow_tts_e2e','xtts_decoder','vits_waveform')})"
