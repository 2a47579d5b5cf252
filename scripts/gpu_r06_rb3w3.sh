# 64-channel whole-block kernel-3 ResBlock at three waves per SIMD (RB3_W64=3, 168 VGPRs, small
# spill) against the two-wave default: correctness on the variant library, then an interleaved A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rb3
TTS_MI355X_LIB=abx/lib_rb3w3.so timeout -k 10 600 python -u -m pytest tests/test_hifigan_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "golden or config1 or whole_block or benchmark_size" > gpurun_out/pytest_rb3w3.log 2>&1 || { tail -30 gpurun_out/pytest_rb3w3.log; exit 1; }
tail -1 gpurun_out/pytest_rb3w3.log
AB_NOTEST=1 AB="main:main rb3w3:abx/lib_rb3w3.so" AB_FILTER="block" bash scripts/ab_lib_env.sh || exit 1
AB_NOTEST=1 AB="main:main rb3w3:abx/lib_rb3w3.so" AB_FILTER="block" bash scripts/ab_lib_env.sh || exit 1
