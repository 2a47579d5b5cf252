# Session: flow / text / config GPU tests (WN-update fusion), the Winograd s_setprio A/B, and a
# kernel trace of the Glow decoder side line (inter-kernel gaps).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_glow_gpu.py tests/test_vits_gpu.py tests/test_glow_tts_gpu.py tests/test_configs_gpu.py tests/test_vits_text_gpu.py tests/test_xtts_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s3.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_s3.log
[ $rc -eq 0 ] || exit $rc
AB_NOTEST=1 AB="main:main p1:abx/lib_prio1.so p2:abx/lib_prio2.so" AB_FILTER="wino" bash scripts/ab_lib_env.sh || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_glow -o glow --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-alt --no-e2e --no-xtts --no-vits > gpurun_out/prof_glow.log 2>&1 || { tail -5 gpurun_out/prof_glow.log; exit 1; }
for wn in 1 0; do
  TTS_MI355X_WN_FUSION=$wn timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt --no-e2e --no-xtts --no-vits > gpurun_out/glow_wn$wn.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/glow_wn$wn.json'));g=d['glow_decoder'];print('wn$wn', round(g['ms_per_step'],3), g['launches_per_step'], g['breakdown_ms']); v=d.get('vits_tts_e2e'); print(v and {k:(round(x['ms_per_step'],2), x['mel_frames']) for k,x in v['variants'].items()})"
done
