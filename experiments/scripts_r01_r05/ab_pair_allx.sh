# A/B of the resblock-pair input staging: all 16-channel groups at once (TTS_MI355X_PAIR_ALLX=1,
# default) vs double-buffered per group, after a parity pass of the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hifigan_gpu.py -m gpu -p no:cacheprovider > gpurun_out/aba_pytest.log 2>&1 || { tail -20 gpurun_out/aba_pytest.log; exit 1; }
tail -1 gpurun_out/aba_pytest.log
run() {
  name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts > gpurun_out/aba_$name.json 2>gpurun_out/aba_$name.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/aba_$name.json'));b=d['kernel_breakdown_ms'];print('$name', round(d['ms_per_step'],2), {k: round(v,2) for k,v in b.items() if 'pair' in k})"
}
for r in 1 2; do
  run allx_$r TTS_MI355X_PAIR_ALLX=1
  run dbuf_$r TTS_MI355X_PAIR_ALLX=0
done
