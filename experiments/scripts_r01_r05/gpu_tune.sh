# Tile sweep (both math modes) on the benchmark's conv shapes; logs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for m in ${TUNE_MODES:-fp32x6 fp32}; do
  timeout -k 10 400 python scripts/tune_conv.py $m $TUNE_ONLY > gpurun_out/tune_$m.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/tune_$m.log
done
