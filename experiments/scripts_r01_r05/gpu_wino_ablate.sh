# Winograd kernel ablation builds (ab/lib_wab<N>.so, WINO_ABLATE bits: 1 no x loads, 2 no
# transform jobs, 4 no A stream; timing only) against the product build, op level, B=32 shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in main wab1 wab2 wab3 wab4 wab7; do
  echo "== $v"
  lib=tts-3_amd/tts_amd/_lib/libtts_mi355x.so; [ $v = main ] || lib=ab/lib_$v.so
  TTS_MI355X_LIB=$lib TUNE_TILES=21,13 timeout -k 10 120 python scripts/tune_conv.py f16x3 c128_k11 c128_k7 c256_k11 2>&1 | grep -v amdgpu.ids || exit 1
done 2>&1 | tee gpurun_out/wino_ablate.log
