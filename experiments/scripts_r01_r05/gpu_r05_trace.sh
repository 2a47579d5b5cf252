# Kernel trace of the default (concurrent) schedule: how much of the step is covered by kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ctrace
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/ctrace -o ct --output-format csv -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits --no-vits-tts --no-rb2 > gpurun_out/ctrace/bench.json 2> gpurun_out/ctrace/bench.err || { tail -20 gpurun_out/ctrace/bench.err; exit 1; }
f=$(find gpurun_out/ctrace -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_coverage.py "$f"
