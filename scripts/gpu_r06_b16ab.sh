# Round 6: bf16 scheme A/B of environment switches on HiFiGAN-v1 [32, 80, 1024] bf16 (bench main line
# in bf16, two rounds):  VARS="main: nowino:TTS_MI355X_WINO_BF16=0 ..." (name:ENV1,ENV2);
# SUITE=1 then runs the whole GPU suite on this tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/b16ab
B="bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits --no-vits-tts --no-rb2 --math-mode ${MODE:-bf16}"
for r in 1 2; do
  for v in ${VARS:-main:}; do
    name=${v%%:*}; envs=${v#*:}
    env ${envs//,/ } timeout -k 10 300 python $B > gpurun_out/b16ab/${name}_$r.json 2> gpurun_out/b16ab/${name}_$r.err || { tail -5 gpurun_out/b16ab/${name}_$r.err; exit 1; }
    python - gpurun_out/b16ab/${name}_$r.json $name $r <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); b = d["kernel_breakdown_ms"]
print(sys.argv[2], sys.argv[3], "step", round(d["ms_per_step"], 2), "serial", round(sum(b.values()), 2),
      {k: round(v, 2) for k, v in list(b.items())[:12]})
PY
  done
done
if [ -n "$SUITE" ]; then
  export TTS_ERRLOG=gpurun_out/parity_errors_r06b.jsonl
  rm -f $TTS_ERRLOG
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_r06b.log 2>&1
  rc=$?
  tail -3 gpurun_out/pytest_gpu_r06b.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu_r06b.log | head -30; exit $rc; }
fi
