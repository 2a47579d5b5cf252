# cond_layer GEMV kernel (cond_vec_kernel): the GPU tests of its users (VITS, XTTS, Glow cond,
# ResBlock2 / YourTTS, HiFiGAN goldens), then the side lines with the new kernel and the previous one
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_vits_gpu.py tests/test_configs_gpu.py tests/test_glow_gpu.py tests/test_hifigan_gpu.py tests/test_vits_text_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_condvec.log 2>&1 || { tail -40 gpurun_out/pytest_condvec.log; exit 1; }
tail -1 gpurun_out/pytest_condvec.log
for r in 1 2; do
  for v in main head; do
    lib=abx/lib_$v.so; [ $v = main ] && lib=tts-3_amd/tts_amd/_lib/libtts_mi355x.so
    TTS_MI355X_LIB=$lib timeout -k 10 400 python scripts/side_ab.py > gpurun_out/side_cv.json 2> gpurun_out/side_cv.err || { tail -20 gpurun_out/side_cv.err; exit 1; }
    echo "$v round $r: $(cat gpurun_out/side_cv.json)"
  done
done
