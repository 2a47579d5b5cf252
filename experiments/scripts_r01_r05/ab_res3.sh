# Parity of the whole-block kernel-3 ResBlock fusion (TTS_MI355X_RESBLOCK3 = 32 / all) then an
# interleaved A/B against the per-iteration pair kernels (0) and of the 64-channel geometries.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TTS_MI355X_RESBLOCK3=all timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hifigan_gpu.py tests/test_vits_gpu.py tests/test_xtts_gpu.py -m gpu -p no:cacheprovider > gpurun_out/r3_pytest.log 2>&1 || { tail -30 gpurun_out/r3_pytest.log; exit 1; }
echo "policy all: $(tail -1 gpurun_out/r3_pytest.log)"
AB="${AB:-c32:TTS_MI355X_RESBLOCK3=32 all128:TTS_MI355X_RESBLOCK3=all all192:TTS_MI355X_RESBLOCK3=all,TTS_MI355X_RES3_GEO64=1}" AB_FILTER="k3_c|block" bash scripts/ab_env.sh
