#!/usr/bin/env python3
"""Per-family averages of arbitrary rocprofv3 PMC counters over the bench forward.

usage: pmc_families.py <root> <pass-subdir> [<pass-subdir> ...]
Every pass directory holds one rocprofv3 --pmc run of `bench.py` (counter_collection.csv); the
library's dispatches are cut into forwards by <root>/forward_names.json (the launch sequence bench.py
dumps with TTS_FORWARD_NAMES) exactly like scripts/mfma_from_pmc.py.  Prints one row per family
with every counter's per-launch average; writes <root>/pmc_families.json.
"""
import csv
import json
import os
import sys
from collections import defaultdict


def find(root, suffix):
    for dp, _, fs in os.walk(root):
        for f in fs:
            if f.endswith(suffix):
                return os.path.join(dp, f)
    raise FileNotFoundError(f"{suffix} under {root}")


def main():
    root = sys.argv[1]
    names = json.load(open(os.path.join(root, "forward_names.json")))
    fam = defaultdict(lambda: defaultdict(list))
    for sub in sys.argv[2:]:
        rows = defaultdict(dict)
        kern = {}
        for r in csv.DictReader(open(find(os.path.join(root, sub), "counter_collection.csv"))):
            d = int(r["Dispatch_Id"])
            kern[d] = r["Kernel_Name"]
            rows[d][r["Counter_Name"]] = rows[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        seq = [rows[d] for d in sorted(rows) if "tts::" in kern[d]]
        if len(seq) % len(names):
            print(f"{sub}: {len(seq)} dispatches not a multiple of {len(names)}; skipped")
            continue
        for f in range(len(seq) // len(names)):
            for i, nm in enumerate(names):
                for k, v in seq[f * len(names) + i].items():
                    fam[nm][k].append(v)
    out = {nm: {k: sum(v) / len(v) for k, v in c.items()} for nm, c in fam.items()}
    json.dump(out, open(os.path.join(root, "pmc_families.json"), "w"), indent=1)
    keys = sorted({k for c in out.values() for k in c})
    print("family".ljust(22) + "".join(k[:18].rjust(19) for k in keys))
    for nm in sorted(out, key=names.index):
        print(nm.ljust(22) + "".join(f"{out[nm].get(k, 0):19.4g}" for k in keys))


if __name__ == "__main__":
    main()
