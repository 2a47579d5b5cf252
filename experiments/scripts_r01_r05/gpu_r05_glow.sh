# Glow decoder lanes captured as a HIP graph: the Glow GPU tests (incl. lanes + graph bitwise), then
# an interleaved A/B of the decoder side line (1 lane direct, 2 lanes graph, 3 lanes graph)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_glow_gpu.py tests/test_glow_tts_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_glow.log 2>&1 || { tail -30 gpurun_out/pytest_glow.log; exit 1; }
tail -1 gpurun_out/pytest_glow.log
for r in 1 2; do
  for v in "1 0" "2 1" "3 1" "4 1"; do
    set -- $v
    TTS_MI355X_GLOW_LANES=$1 TTS_MI355X_GLOW_GRAPH=$2 timeout -k 10 300 python scripts/glow_ab.py f16x3 bf16 > gpurun_out/glow_ab_$1_$r.json 2> gpurun_out/glow_ab_$1_$r.err || { tail -20 gpurun_out/glow_ab_$1_$r.err; exit 1; }
    echo "lanes=$1 graph=$2 round $r: $(cat gpurun_out/glow_ab_$1_$r.json | tr '\n' ' ')"
  done
done
