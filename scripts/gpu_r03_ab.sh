# Round 3 iteration: GPU tests on the working-tree library (CHECK_TESTS), then an interleaved A/B
# of ab/lib_<AB_LIBS>.so against it (scripts/gpu_ab_lib.sh: bench forward + kernel breakdown)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "$CHECK_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
    $CHECK_TESTS > gpurun_out/ab_pytest.log 2>&1
  rc=$?
  tail -3 gpurun_out/ab_pytest.log
  [ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR|Error:|assert " gpurun_out/ab_pytest.log | head -30; exit $rc; }
fi
[ -n "$AB_LIBS" ] && bash scripts/gpu_ab_lib.sh
