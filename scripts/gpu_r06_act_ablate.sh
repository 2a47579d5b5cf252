# (1) the flow tests on the 8 / 12-wave WN layers (H 128 / 192 / 256); (2) the activation-traffic
# ablation (ACT_ABLATE=1, conv_device.hpp: every activation-plane descriptor cut to 64 KiB, timing
# only) against the product library, HiFiGAN-v1 [32, 80, 1024] in f16x3 and bf16 (VERDICT r5 item 3:
# is the bf16 forward bound by its fp32 activation planes?)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/act
timeout -k 10 600 python -u -m pytest tests/test_glow_gpu.py tests/test_vits_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_wn8.log 2>&1 || { tail -30 gpurun_out/pytest_wn8.log; exit 1; }
tail -1 gpurun_out/pytest_wn8.log
B="bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits --no-vits-tts --no-rb2"
for r in 1 2; do
  for mode in f16x3 bf16; do
    for v in main act; do
      lib=tts-3_amd/tts_amd/_lib/libtts_mi355x.so; [ $v = act ] && lib=abx/lib_act.so
      TTS_MI355X_LIB=$lib timeout -k 10 300 python $B --math-mode $mode > gpurun_out/act/${mode}_${v}_$r.json 2> gpurun_out/act/${mode}_${v}_$r.err || { tail -5 gpurun_out/act/${mode}_${v}_$r.err; exit 1; }
      python - gpurun_out/act/${mode}_${v}_$r.json $mode $v $r <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); b = d["kernel_breakdown_ms"]
print(sys.argv[2], sys.argv[3], sys.argv[4], "step", round(d["ms_per_step"], 2), "serial", round(sum(b.values()), 2),
      {k: round(v, 2) for k, v in list(b.items())[:14]})
PY
    done
  done
done
