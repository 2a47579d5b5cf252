# One iteration on the GPU box: HiFiGAN/VITS/XTTS GPU tests on the working-tree library, then an
# interleaved A/B of ab/lib_<AB_LIBS>.so against it (scripts/gpu_ab_lib.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  ${ITER_TESTS:-tests/test_hifigan_gpu.py tests/test_vits_gpu.py tests/test_xtts_gpu.py} > gpurun_out/iter_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/iter_pytest.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/iter_pytest.log | head -20; exit $rc; }
[ -n "$AB_LIBS" ] && bash scripts/gpu_ab_lib.sh
