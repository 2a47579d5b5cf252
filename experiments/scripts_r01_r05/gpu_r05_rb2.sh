# ResBlock2 whole-block kernels: GPU tests (new + the whole-block / golden HiFiGAN tests), then the
# bench's ResBlock2 side line and the headline (RB1 kernels moved into resblock_block.hpp)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD/tts-3_amd:$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hifigan_gpu.py -k "resblock2 or whole_block or golden or config1 or post" > gpurun_out/rb2_tests.log 2>&1 || { tail -40 gpurun_out/rb2_tests.log; exit 1; }
tail -3 gpurun_out/rb2_tests.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits --no-vits-tts > gpurun_out/rb2_bench.json 2> gpurun_out/rb2_bench.err || { tail -20 gpurun_out/rb2_bench.err; exit 1; }
python - <<'PY'
import json
r = json.loads(open("gpurun_out/rb2_bench.json").read().strip().splitlines()[-1])
print("headline", round(r["ms_per_step"], 2), {k: v for k, v in list(r["kernel_breakdown_ms"].items())[:8]})
for k, v in r["resblock2_decoder"]["variants"].items():
    print(k, round(v["ms_per_step"], 2), list(v["kernel_breakdown_ms"].items())[:10])
PY
