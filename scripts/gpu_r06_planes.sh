# Round 6: bf16 activation planes (MATH_BF16).  (1) the new plane tests and every bf16 test of the
# HiFiGAN-executor paths (HiFiGAN, XTTS, VITS, configs); (2) A/B: planes on / off on the bf16
# HiFiGAN-v1 [32, 80, 1024] forward (bench main line in bf16) and the side lines, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/planes
export TTS_ERRLOG=gpurun_out/planes/parity_errors.jsonl
timeout -k 10 300 python -u -m pytest tests/test_bf16_planes_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/planes/pytest_planes.log 2>&1 || { tail -40 gpurun_out/planes/pytest_planes.log; exit 1; }
tail -2 gpurun_out/planes/pytest_planes.log
timeout -k 10 600 python -u -m pytest tests/test_hifigan_gpu.py tests/test_xtts_gpu.py tests/test_vits_gpu.py tests/test_configs_gpu.py tests/test_sharded_gpu.py -m gpu -k bf16 -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/planes/pytest_bf16.log 2>&1 || { tail -40 gpurun_out/planes/pytest_bf16.log; exit 1; }
tail -2 gpurun_out/planes/pytest_bf16.log
B="bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits --no-vits-tts --no-rb2 --math-mode bf16"
for r in 1 2; do
  for p in 1 0; do
    TTS_MI355X_BF16_PLANES=$p timeout -k 10 300 python $B > gpurun_out/planes/bf16_p${p}_$r.json 2> gpurun_out/planes/bf16_p${p}_$r.err || { tail -5 gpurun_out/planes/bf16_p${p}_$r.err; exit 1; }
    python - gpurun_out/planes/bf16_p${p}_$r.json $p $r <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); b = d["kernel_breakdown_ms"]
print("planes", sys.argv[2], "round", sys.argv[3], "step", round(d["ms_per_step"], 2), "serial", round(sum(b.values()), 2),
      {k: round(v, 2) for k, v in list(b.items())[:16]})
PY
  done
done
for r in 1 2; do
  for p in 1 0; do
    TTS_MI355X_BF16_PLANES=$p SIDE_VITS_TTS=1 timeout -k 10 300 python scripts/side_ab.py > gpurun_out/planes/side_p${p}_$r.json 2> gpurun_out/planes/side_p${p}_$r.err || { tail -5 gpurun_out/planes/side_p${p}_$r.err; exit 1; }
    echo "side planes=$p round $r: $(cat gpurun_out/planes/side_p${p}_$r.json)"
  done
done
