# A/B (one box session): kernel-11 Winograd without its spill (the dense group recomputes its
# transform unit from the lane id, WINO8_REMAT=1) against the default build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TTS_MI355X_LIB=abx/lib_remat.so timeout -k 10 600 python -u -m pytest tests/test_hifigan_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "wino or golden or config1" > gpurun_out/pytest_remat.log 2>&1 || { tail -30 gpurun_out/pytest_remat.log; exit 1; }
tail -1 gpurun_out/pytest_remat.log
AB_NOTEST=1 AB="main:main remat:abx/lib_remat.so" AB_FILTER="wino" bash scripts/ab_lib_env.sh || exit 1
AB_NOTEST=1 AB="main:main remat:abx/lib_remat.so" AB_FILTER="wino" bash scripts/ab_lib_env.sh || exit 1
