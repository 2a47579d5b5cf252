# Round-5 session: the whole GPU suite (new VITS text tests, fused conv_post, bf16 Winograd), the
# default bench line, then the bf16 profiling evidence (scripts/gpu_r05_bf16prof.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['ms_per_step'],d['value'],d['roofline']['frac'],d['roofline']['avg_launch_ms']);print(d['kernel_breakdown_ms']);print({k:(v or {}).get('variants', (v or {}).get('ms_per_step')) for k,v in d.items() if k in ('glow_decoder','glow_tts_e2e','xtts_decoder','vits_waveform')})"
[ -n "$NO_PROF" ] && exit $rc
bash scripts/gpu_r05_bf16prof.sh || exit 1
exit $rc
