#!/usr/bin/env python3
"""HBM traffic per launch family of the HiFiGAN-v1 forward, from rocprofv3 PMC passes.

Input: the directory written by scripts/profile_round.sh (a kernel trace, a FETCH_SIZE pass and
a WRITE_SIZE pass over `bench.py --steps S --warmup W --no-alt --no-glow --no-cpu-baseline`).
Every forward enqueues the same launch sequence (HifiganGenerator executor order), so the
library's dispatches are cut into forwards and named by position; the names come from the
profiled forward bench.py dumps (TTS_FORWARD_NAMES=<root>/forward_names.json).

Counter handling (MI355X_MICROARCH.md, HBM / rocprofv3 section): FETCH_SIZE and WRITE_SIZE are
KiB counters, collected in separate passes.  The gfx950 FETCH_SIZE undercount is documented for
16-B/lane streaming reads only; our activations stream with 4-B/lane buffer loads, so the FETCH
scale is calibrated in-run on `amax_mel`, which reads exactly B*80*T fp32 once (f16x3 mode).
Output: JSON with per_launch_bytes["<mode>:<family>"] and the per-forward total, used by
bench.py for roofline.traffic and the step-level HBM fraction.
"""
import csv
import json
import os
import sys
from collections import defaultdict

V1 = dict(C0=512, ups=[8, 8, 2, 2], kernels=[3, 7, 11])


def forward_names(mode):
    names = []
    if mode == "f16x3":
        names.append("amax_mel")
    names.append("conv_pre_k7_c512")
    C = V1["C0"]
    for u in V1["ups"]:
        C //= 2
        names.append(f"ups_u{u}_c{C}")
        for k in V1["kernels"]:
            fam = "mrf_wino" if (mode == "f16x3" and C >= 128 and k in (7, 11)) else "mrf_conv"
            names += [f"{fam}_k{k}_c{C}"] * 6
    names.append("conv_post")
    return names


def read_pmc(path, counter):
    rows = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        rows[d] = (r["Kernel_Name"], rows.get(d, (None, 0.0))[1] + float(r["Counter_Value"]))
    return [rows[d] for d in sorted(rows)]


def ours(name):
    return "tts::" in name


def find(root, suffix):
    for dp, _, fs in os.walk(root):
        for f in fs:
            if f.endswith(suffix):
                return os.path.join(dp, f)
    raise FileNotFoundError(f"{suffix} under {root}")


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
    mode = sys.argv[2] if len(sys.argv) > 2 else "f16x3"
    B, T = 32, 1024
    out_path = sys.argv[3] if len(sys.argv) > 3 else "profiles/traffic_hifigan_r01.json"
    fn = os.path.join(root, "forward_names.json")
    names = json.load(open(fn)) if os.path.exists(fn) else forward_names(mode)
    per = {}
    for counter, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        seq = [(n, v) for n, v in read_pmc(find(os.path.join(root, sub), "counter_collection.csv"), counter) if ours(n)]
        if len(seq) % len(names):
            raise SystemExit(f"{counter}: {len(seq)} library dispatches is not a multiple of {len(names)}")
        nfw = len(seq) // len(names)
        acc = defaultdict(list)
        for f in range(nfw):
            for i, nm in enumerate(names):
                kname, v = seq[f * len(names) + i]
                acc[nm].append(v * 1024.0)  # KiB -> bytes
        per[counter] = {k: sum(v) / len(v) for k, v in acc.items()}
        per[counter + "_kernel"] = {nm: seq[i][0] for i, nm in enumerate(names)}
    fetch_scale = 1.0
    calib = None
    if "amax_mel" in per["FETCH_SIZE"]:
        algo = 4.0 * B * 80 * T
        calib = {"kernel": "amax_mel", "algorithmic_read_bytes": algo, "raw_fetch_bytes": per["FETCH_SIZE"]["amax_mel"]}
        fetch_scale = algo / per["FETCH_SIZE"]["amax_mel"]
    else:
        # no amax_mel launch (bf16 mode): the probe calibration of the same staging lane map
        # (profiles/fetch_calibration_r06.txt: a 1,084,227,584-byte plane read once counts
        # 529,419.5 KiB of FETCH_SIZE, exactly half)
        fetch_scale = 1084227584.0 / (529419.5 * 1024.0)
        calib = {"probe": "profiles/fetch_calibration_r06.txt (scripts/probe_fetch.hip, staging lane map)",
                 "algorithmic_read_bytes": 1084227584.0, "raw_fetch_bytes": 529419.5 * 1024.0}
    fams = sorted(set(names), key=names.index)
    counts = {f: names.count(f) for f in fams}
    per_launch = {}
    table = []
    total = 0.0
    for f in fams:
        rd = per["FETCH_SIZE"][f] * fetch_scale
        wr = per["WRITE_SIZE"][f]
        per_launch[f"{mode}:{f}"] = rd + wr
        total += (rd + wr) * counts[f]
        table.append({"family": f, "launches_per_forward": counts[f], "kernel": per["FETCH_SIZE_kernel"][f],
                      "fetch_bytes_raw": per["FETCH_SIZE"][f], "fetch_bytes": rd, "write_bytes": wr})
    per_launch[f"{mode}:__forward__"] = total
    # per-family kernel durations from the kernel trace (rocprof's own stats aggregate by kernel
    # symbol, and families of equal tile share one symbol)
    trace = [r for r in csv.DictReader(open(find(os.path.join(root, "trace"), "kernel_trace.csv"))) if ours(r["Kernel_Name"])]
    trace.sort(key=lambda r: int(r["Dispatch_Id"]))
    durs = defaultdict(list)
    if len(trace) % len(names) == 0:
        for f in range(len(trace) // len(names)):
            for i, nm in enumerate(names):
                r = trace[f * len(names) + i]
                durs[nm].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    for row in table:
        d = durs.get(row["family"], [])
        row["trace_avg_ms"] = sum(d) / len(d) if d else None
        row["trace_launches"] = len(d)
    doc = {
        "source": f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) over bench.py, math_mode {mode}, "
                  f"B={B}, T={T}; scripts/profile_round.sh + scripts/traffic_from_pmc.py",
        "note": "bytes = FETCH_SIZE*1024*fetch_scale + WRITE_SIZE*1024 per launch, averaged over the profiled "
                "forwards; fetch_scale calibrated in-run on amax_mel (exact read size, same 4-B/lane buffer-load "
                "pattern as the activation staging), or from the staging-pattern probe where no amax_mel runs "
                "(bf16). FETCH counts L2->fabric requests, i.e. HBM plus "
                "Infinity-Cache hits.",
        "fetch_scale": fetch_scale,
        "fetch_calibration": calib,
        "per_launch_bytes": per_launch,
        "families": table,
    }
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    json.dump(doc, open(out_path, "w"), indent=1)
    print(f"fetch_scale {fetch_scale:.3f}; per-forward bytes {total / 1e9:.2f} GB")
    with open(os.path.join(os.path.dirname(out_path) or ".", "family_stats.csv"), "w") as fh:
        fh.write("family,launches_per_forward,trace_launches,trace_avg_ms,fetch_bytes,write_bytes,kernel\n")
        for r in table:
            fh.write(f"{r['family']},{r['launches_per_forward']},{r['trace_launches']},{r['trace_avg_ms']},"
                     f"{r['fetch_bytes']:.0f},{r['write_bytes']:.0f},\"{r['kernel']}\"\n")
    for r in table:
        print(f"{r['family']:22s} x{r['launches_per_forward']:2d}  read {r['fetch_bytes'] / 1e6:9.1f} MB  "
              f"write {r['write_bytes'] / 1e6:9.1f} MB  avg {r['trace_avg_ms'] or 0:7.3f} ms")


if __name__ == "__main__":
    main()
