#!/usr/bin/env python3
"""Per-family averages of arbitrary PMC counters over the HiFiGAN forward of a bench run.

usage: pmc_family_counters.py <pmc dir> <forward_names.json> COUNTER [COUNTER ...]
The library's dispatches are cut into forwards and named by position (the profiled forward's
names, bench.py TTS_FORWARD_NAMES), as scripts/traffic_from_pmc.py does; prints one line per
family with the per-launch average of every counter (raw counter units).
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
    root, names_path, counters = sys.argv[1], sys.argv[2], sys.argv[3:]
    names = json.load(open(names_path))
    path = find(root, "counter_collection.csv")
    per = defaultdict(lambda: defaultdict(float))
    kname = {}
    for r in csv.DictReader(open(path)):
        if "tts::" not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        kname[d] = r["Kernel_Name"]
    ds = sorted(per)
    if len(ds) % len(names):
        raise SystemExit(f"{len(ds)} library dispatches is not a multiple of {len(names)}")
    fam = defaultdict(lambda: defaultdict(list))
    for i, d in enumerate(ds):
        nm = names[i % len(names)]
        for c in counters:
            fam[nm][c].append(per[d].get(c, 0.0))
    out = {}
    for nm in dict.fromkeys(names):
        out[nm] = {c: sum(v) / len(v) for c, v in fam[nm].items()}
        print(nm, " ".join(f"{c}={out[nm][c]:.4g}" for c in counters))
    json.dump(out, open(os.path.join(root, "family_counters.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
