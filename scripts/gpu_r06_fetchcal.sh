# FETCH_SIZE calibration for the staging pattern: a 1.08 GB plane read once
# with three access patterns (scripts/probe_fetch.hip), FETCH_SIZE and the request-size split
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/fetchcal
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/scripts/probe_fetch
timeout -k 10 60 $P 2 > $OUT/probe_plain.log 2>&1 || { cat $OUT/probe_plain.log; exit 1; }
cat $OUT/probe_plain.log
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- $P 2 > $OUT/fetch.log 2>&1 || { tail -5 $OUT/fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $OUT/req -o r --output-format csv -- $P 2 > $OUT/req.log 2>&1 || { tail -5 $OUT/req.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d $OUT/hit -o h --output-format csv -- $P 2 > $OUT/hit.log 2>&1 || { tail -5 $OUT/hit.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $OUT/trace -o t --output-format csv -- $P 3 > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
python3 - <<'PY'
import csv, glob, os, collections
out = os.environ.get("GRAFT_REPO_ROOT") + "/gpurun_out/fetchcal"
for sub in ("fetch", "req", "hit"):
    f = glob.glob(f"{out}/{sub}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(sub, k, {c: sum(v) / len(v) for c, v in d.items()})
PY
