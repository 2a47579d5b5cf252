"""Average PMC counters per dispatch of the kernels whose name matches a pattern, over one or more
rocprofv3 counter_collection.csv files: python kernel_pmc_avg.py PATTERN file.csv [...]"""
import collections
import csv
import re
import sys

pat = re.compile(sys.argv[1])
tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for path in sys.argv[2:]:
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if not pat.search(name):
                continue
            key = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))[-90:]
            tot[(key, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[(key, r["Counter_Name"])].add((path, r["Dispatch_Id"]))
for (k, c), v in sorted(tot.items()):
    n = len(disp[(k, c)])
    print(f"{k:90s} {c:28s} n={n:5d} avg={v / n:.4g}")
