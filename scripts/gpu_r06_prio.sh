# Round 6: s_setprio on the Winograd kernel's point groups (WINO8_PRIO=1: the DMA waves 4-7,
# 2: the dense-transform waves 0-3) -- Winograd tests on both variants, then an A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in prio1 prio2; do
  TTS_MI355X_LIB=abx/lib_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_hifigan_gpu.py -m gpu -k "wino" -p no:cacheprovider > gpurun_out/${v}_pytest.log 2>&1 ||
    { tail -30 gpurun_out/${v}_pytest.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/${v}_pytest.log)"
done
AB_NOTEST=1 AB_FILTER=wino AB="main:main p1:abx/lib_prio1.so p2:abx/lib_prio2.so" bash scripts/ab_lib_env.sh
