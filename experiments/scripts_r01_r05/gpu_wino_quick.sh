# Winograd conv: op parity tests + op timing (tile 21 vs direct tile 13) on the bench shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hifigan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "winograd" > gpurun_out/pytest_wino.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_wino.log
[ $rc -eq 0 ] || exit $rc
TUNE_TILES=21,13 timeout -k 10 200 python scripts/tune_conv.py f16x3 c128_k11 c128_k7 c256_k11 c256_k7 2>&1 | grep -v amdgpu.ids
