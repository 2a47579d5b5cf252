# One-launch WN layer tuning A/B (abx/ variant libraries of kernels_glow_wn.hip): the Glow GPU tests
# on the default build, then the Glow decoder side line per variant, two interleaved rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_glow_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "wn_layer or reference" > gpurun_out/pytest_wntune.log 2>&1 || { tail -40 gpurun_out/pytest_wntune.log; exit 1; }
tail -1 gpurun_out/pytest_wntune.log
for r in 1 2; do
  for v in ${WN_VARIANTS:-main old pd3 pd4 noepi}; do
    lib=abx/lib_$v.so; [ $v = main ] && lib=tts-3_amd/tts_amd/_lib/libtts_mi355x.so
    TTS_MI355X_LIB=$lib timeout -k 10 300 python scripts/glow_ab.py f16x3 bf16 > gpurun_out/wn_tune.json 2> gpurun_out/wn_tune.err || { tail -20 gpurun_out/wn_tune.err; exit 1; }
    echo "$v round $r: $(cat gpurun_out/wn_tune.json | tr '\n' ' ')"
  done
done
