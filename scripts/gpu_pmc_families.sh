# Extra PMC passes over the bench forward (one rocprofv3 run per counter group), per kernel family
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmcf
mkdir -p $OUT
BENCH="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits --no-vits-tts --no-rb2"
export TTS_FORWARD_NAMES=$OUT/forward_names.json
timeout -s KILL 120 rocprofv3 --list-avail > $OUT/counters_avail.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -s KILL 240 rocprofv3 --pmc $grp -d $OUT/p$i -o p$i --output-format csv -- python3 $BENCH > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/pmc_families.py $OUT $(seq -f "p%g" 1 $i)
