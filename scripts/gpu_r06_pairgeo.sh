# 64-channel ResBlock1 pair kernel: 128-column geometry at three workgroups per CU
# (TTS_MI355X_PAIR_GEO64=2) against the 192-column default; correctness first, then an interleaved A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pg
TTS_MI355X_PAIR_GEO64=2 timeout -k 10 600 python -u -m pytest tests/test_hifigan_gpu.py tests/test_vits_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pairgeo.log 2>&1 || { tail -30 gpurun_out/pytest_pairgeo.log; exit 1; }
tail -1 gpurun_out/pytest_pairgeo.log
B="bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits --no-vits-tts --no-rb2"
for r in 1 2 3; do
  for v in 1 2; do
    TTS_MI355X_PAIR_GEO64=$v timeout -k 10 300 python $B > gpurun_out/pg/g${v}_$r.json 2> gpurun_out/pg/g${v}_$r.err || { tail -5 gpurun_out/pg/g${v}_$r.err; exit 1; }
    python - gpurun_out/pg/g${v}_$r.json $v $r <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); b = d["kernel_breakdown_ms"]
print("geo", sys.argv[2], "round", sys.argv[3], "step", round(d["ms_per_step"], 2), "serial", round(sum(b.values()), 2),
      {k: round(v, 2) for k, v in b.items() if "c64" in k})
PY
  done
done
