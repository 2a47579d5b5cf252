# x6 kernel ablation: baseline vs builds with the staging refill (1), the A stream (2) or both (3)
# removed (results wrong, timing only), same session.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TUNE_TILES=${TUNE_TILES:-"7,3,10,1,2"}
for v in new abl1 abl2 abl3; do
  echo "== $v"
  TTS_MI355X_LIB=ab/lib_$v.so timeout -k 10 300 python scripts/tune_conv.py fp32x6 $ABL_ONLY > gpurun_out/abl_$v.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/abl_$v.log
done
