# One-launch WaveNet layer in the VITS flows / posterior encoder: the VITS, Glow-TTS and config GPU
# tests, then the side lines with and without it (TTS_MI355X_WN_LAYER)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_vits_gpu.py tests/test_vits_text_gpu.py tests/test_glow_tts_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_wnlayer2.log 2>&1 || { tail -40 gpurun_out/pytest_wnlayer2.log; exit 1; }
tail -1 gpurun_out/pytest_wnlayer2.log
for r in 1 2; do
  for v in 1 0; do
    SIDE_VITS_TTS=1 TTS_MI355X_WN_LAYER=$v timeout -k 10 400 python scripts/side_ab.py > gpurun_out/side_wn$v.json 2> gpurun_out/side_wn$v.err || { tail -20 gpurun_out/side_wn$v.err; exit 1; }
    echo "WN_LAYER=$v round $r: $(cat gpurun_out/side_wn$v.json)"
  done
done
