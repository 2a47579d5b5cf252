# Round-6 final tree (third session), part A: the whole GPU suite (every measured error logged), smoke(), and the
# default bench line (driver arguments) without the profiler
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final2
export TTS_ERRLOG=gpurun_out/final2/parity_errors_r06_final.jsonl
rm -f $TTS_ERRLOG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/final2/pytest_gpu_r06_final.log 2>&1
rc=$?
tail -2 gpurun_out/final2/pytest_gpu_r06_final.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/final2/pytest_gpu_r06_final.log | head -30; exit $rc; }
unset TTS_ERRLOG
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2/smoke_r06_final.log 2>&1 || { tail -20 gpurun_out/final2/smoke_r06_final.log; exit 1; }
tail -1 gpurun_out/final2/smoke_r06_final.log
timeout -k 10 700 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final2/bench_r06_final.json 2> gpurun_out/final2/bench_r06_final.err || { tail -20 gpurun_out/final2/bench_r06_final.err; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/final2/bench_r06_final.json').read().strip().splitlines()[-1])
print('bench', round(d['ms_per_step'], 2), round(d['value'] / 1e6, 1), 'M samples/s frac', round(d['roofline']['frac'], 4))
print('side', {k: (v.get('ms_per_step') if isinstance(v, dict) else None) for k, v in d.items() if isinstance(v, dict) and 'ms_per_step' in v})
print('vits', {k: round(x['ms_per_step'], 2) for k, x in d['vits_waveform']['variants'].items()})
print('e2e', {k: round(x['ms_per_step'], 2) for k, x in d['glow_tts_e2e']['variants'].items()})
"
