# Round 6: Winograd epilogue L2 prefetch (WINO8_EPI_PF=1 variant, abx/lib_wpf.so) -- the Winograd
# GPU tests on the variant, then an interleaved A/B against the in-tree library on the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TTS_MI355X_LIB=abx/lib_wpf.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_hifigan_gpu.py -m gpu -k "wino or generator or golden" -p no:cacheprovider > gpurun_out/epipf_pytest.log 2>&1 ||
  { tail -30 gpurun_out/epipf_pytest.log; exit 1; }
tail -1 gpurun_out/epipf_pytest.log
AB_NOTEST=1 AB_FILTER=wino AB="main:main wpf:abx/lib_wpf.so" bash scripts/ab_lib_env.sh
