# Concurrent MRF branches (three streams, default) vs one stream (TTS_MI355X_MRF_STREAMS=0): the GPU
# suite on the default, then an interleaved A/B of the headline, then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
AB_NOTEST=1 AB="streams:main one:main|TTS_MI355X_MRF_STREAMS=0" AB_FILTER="zzz" bash scripts/ab_lib_env.sh || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['ms_per_step'],d['value'],d['roofline']['frac']);print({k:(v or {}).get('variants', (v or {}).get('ms_per_step')) for k,v in d.items() if k in ('glow_decoder','glow_tts_e2e','xtts_decoder','vits_waveform')})"
