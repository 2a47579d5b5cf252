# A/B of the 64-channel resblock-pair geometry (TTS_MI355X_PAIR_GEO64) and of fusing every
# 64-channel iteration (TTS_MI355X_PAIR_FUSION=all), after a parity pass of the fused paths.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TTS_MI355X_PAIR_FUSION=all timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hifigan_gpu.py -m gpu -p no:cacheprovider -k "golden or oracle or reference" > gpurun_out/abg_pytest.log 2>&1 || { tail -20 gpurun_out/abg_pytest.log; exit 1; }
tail -2 gpurun_out/abg_pytest.log
run() {  # name, env...
  name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts > gpurun_out/abg_$name.json 2>gpurun_out/abg_$name.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abg_$name.json'));b=d['kernel_breakdown_ms'];print('$name', round(d['ms_per_step'],2), {k: round(v,2) for k,v in b.items() if 'c64' in k})"
}
for r in 1 2; do
  run geo1_$r TTS_MI355X_PAIR_GEO64=1
  run geo0_$r TTS_MI355X_PAIR_GEO64=0
  run geo1all_$r TTS_MI355X_PAIR_GEO64=1 TTS_MI355X_PAIR_FUSION=all
  run geo0all_$r TTS_MI355X_PAIR_GEO64=0 TTS_MI355X_PAIR_FUSION=all
done
