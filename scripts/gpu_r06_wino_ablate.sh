# Winograd c128 ablations (timing only, wrong results): which resource bounds k7 / k11 c128.
# WINO_ABLATE bits (wino_kernel.hpp): 2 no transform jobs, 4 no A (weight) stream, 64 A loads all
# from step 0 (L1/L2 hits), 8 no MFMA, 16 no epilogue
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
for v in main a4 a64 a2 a6 a16 a22 a8; do
  lib=tts-3_amd/tts_amd/_lib/libtts_mi355x.so; [ $v = main ] || lib=abx/lib_$v.so
  echo "== $v round $r"
  TTS_MI355X_LIB=$lib TUNE_TILES=21 timeout -k 10 120 python scripts/tune_conv.py f16x3 c128_k11 c128_k7 c256_k11 2>&1 | grep -v amdgpu.ids || exit 1
done
done 2>&1 | tee gpurun_out/wino_ablate_r06.log
