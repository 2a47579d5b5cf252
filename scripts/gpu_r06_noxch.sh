# Round 6: Winograd without the partial-sum exchange (WINO8_NOXCH=1, abx/lib_noxch.so: each wave all
# 7 points of one 32-column block) -- Winograd tests, bitwise equality with the in-tree library, A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
AB_SKIP=1 true || TTS_MI355X_LIB=abx/lib_noxch.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_hifigan_gpu.py -m gpu -k "wino or golden" -p no:cacheprovider > gpurun_out/noxch_pytest.log 2>&1 ||
  { tail -30 gpurun_out/noxch_pytest.log; exit 1; }
echo "noxch $(tail -1 gpurun_out/noxch_pytest.log)"
timeout -k 10 120 python scripts/lib_bitwise.py gpurun_out/bw_main.npz || exit 1
TTS_MI355X_LIB=abx/lib_noxch.so timeout -k 10 120 python scripts/lib_bitwise.py gpurun_out/bw_noxch.npz gpurun_out/bw_main.npz || exit 1
AB_NOTEST=1 AB_FILTER=wino AB="main:main nx:abx/lib_noxch.so" bash scripts/ab_lib_env.sh
