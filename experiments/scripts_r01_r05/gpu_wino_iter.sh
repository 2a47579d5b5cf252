# one iteration on the Winograd kernel: parity tests, op timing A/B over ab/ libs, stamps (ab/lib_stamps.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hifigan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "winograd" > gpurun_out/pytest_wino.log 2>&1 || { tail -20 gpurun_out/pytest_wino.log; exit 1; }
tail -2 gpurun_out/pytest_wino.log
for v in main $AB_LIBS; do
  lib=tts-3_amd/tts_amd/_lib/libtts_mi355x.so; [ $v = main ] || lib=ab/lib_$v.so
  echo "== $v"
  TTS_MI355X_LIB=$lib TUNE_TILES=21 timeout -k 10 200 python scripts/tune_conv.py f16x3 ${SHAPES:-c128_k11 c128_k7 c256_k11 c256_k7} 2>&1 | grep -v amdgpu.ids || exit 1
done
if [ -f ab/lib_stamps.so ]; then
  TTS_MI355X_LIB=ab/lib_stamps.so timeout -k 5 120 python scripts/wino_stamps.py 128 11 1 2>&1 | grep -v amdgpu.ids
fi
