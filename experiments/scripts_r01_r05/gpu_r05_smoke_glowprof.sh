# smoke() on the final tree, then a rocprofv3 kernel trace + stats of the Glow decoder side line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/glowprof
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/glowprof -o glow --output-format csv -- python3 scripts/glow_ab.py f16x3 bf16 > gpurun_out/glowprof/run.log 2>&1 || { tail -20 gpurun_out/glowprof/run.log; exit 1; }
cat gpurun_out/glowprof/run.log | tail -2
find gpurun_out/glowprof -name "*kernel_stats.csv"
