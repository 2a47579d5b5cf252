#!/usr/bin/env python3
"""MFMA-busy fraction per launch family of the HiFiGAN-v1 forward, from a rocprofv3 SQ pass.

Input: the directory written by scripts/profile_round.sh: a kernel trace (durations) and the
`sq` PMC pass (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE, SQ_BUSY_CYCLES, ...) over
`bench.py --steps S --warmup W`, plus forward_names.json (the launch sequence of one forward).

Counter handling (MI355X_MICROARCH.md): SQ_VALU_MFMA_BUSY_CYCLES counts MFMA pipe cycles summed
over every SIMD (32 per v_mfma_f32_32x32x16_{f16,bf16}); GRBM_GUI_ACTIVE is summed over the 8 XCDs,
so GRBM_GUI_ACTIVE / 8 is the dispatch's cycle count and (GRBM_GUI_ACTIVE / 8) / duration its
effective clock (DVFS).  With 256 CUs x 4 SIMDs:

  mfma_busy_frac_at_clock = MFMA_BUSY / (1024 * GRBM_GUI_ACTIVE / 8)    (busy share of the cycles run)
  mfma_busy_frac          = MFMA_BUSY / (1024 * 2.4 GHz * duration)     (share of the nominal peak)

Durations come from the kernel-trace pass (the PMC pass serialises dispatches).  Output JSON:
families["<mode>:<family>"] -> fractions, clock, counters per launch; read by bench.py
(roofline.mfma_busy_frac) and committed under profiles/.
"""
import csv
import json
import os
import sys
from collections import defaultdict

N_SIMD = 256 * 4
NOMINAL_GHZ = 2.4


def find(root, suffix):
    for dp, _, fs in os.walk(root):
        for f in fs:
            if f.endswith(suffix):
                return os.path.join(dp, f)
    raise FileNotFoundError(f"{suffix} under {root}")


def ours(name):
    return "tts::" in name


def read_counters(path):
    rows = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        names[d] = r["Kernel_Name"]
        rows[d][r["Counter_Name"]] = rows[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [(names[d], rows[d]) for d in sorted(rows)]


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
    mode = sys.argv[2] if len(sys.argv) > 2 else "f16x3"
    out_path = sys.argv[3] if len(sys.argv) > 3 else "profiles/mfma_busy_r03.json"
    names = json.load(open(os.path.join(root, "forward_names.json")))
    seq = [(n, c) for n, c in read_counters(find(os.path.join(root, "sq"), "counter_collection.csv")) if ours(n)]
    if len(seq) % len(names):
        raise SystemExit(f"{len(seq)} library dispatches in the SQ pass is not a multiple of {len(names)}")
    trace = [r for r in csv.DictReader(open(find(os.path.join(root, "trace"), "kernel_trace.csv")))
             if ours(r["Kernel_Name"])]
    trace.sort(key=lambda r: int(r["Dispatch_Id"]))
    if len(trace) % len(names):
        raise SystemExit(f"{len(trace)} traced dispatches is not a multiple of {len(names)}")
    dur = defaultdict(list)
    for f in range(len(trace) // len(names)):
        for i, nm in enumerate(names):
            r = trace[f * len(names) + i]
            dur[nm].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    acc = defaultdict(lambda: defaultdict(list))
    for f in range(len(seq) // len(names)):
        for i, nm in enumerate(names):
            for k, v in seq[f * len(names) + i][1].items():
                acc[nm][k].append(v)
    fams = {}
    for nm in sorted(set(names), key=names.index):
        c = {k: sum(v) / len(v) for k, v in acc[nm].items()}
        d = sum(dur[nm]) / len(dur[nm])
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        cycles = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        fams[f"{mode}:{nm}"] = {
            "launches_per_forward": names.count(nm),
            "trace_avg_ms": d * 1e3,
            "clock_ghz": cycles / d / 1e9 if d > 0 else None,
            "mfma_busy_frac_at_clock": busy / (N_SIMD * cycles) if cycles else None,
            "mfma_busy_frac": busy / (N_SIMD * NOMINAL_GHZ * 1e9 * d) if d > 0 else None,
            "counters_per_launch": c,
        }
    doc = {
        "source": f"rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES "
                  f"GRBM_GUI_ACTIVE over bench.py (math_mode {mode}, B=32, T=1024) + a --kernel-trace pass for "
                  f"durations; scripts/profile_round.sh + scripts/mfma_from_pmc.py",
        "formula": {"mfma_busy_frac": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * 2.4 GHz * trace duration)",
                    "mfma_busy_frac_at_clock": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 * GRBM_GUI_ACTIVE / 8)",
                    "clock_ghz": "GRBM_GUI_ACTIVE / 8 / trace duration"},
        "families": fams,
    }
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    json.dump(doc, open(out_path, "w"), indent=1)
    with open(os.path.splitext(out_path)[0] + ".csv", "w") as fh:
        fh.write("family,launches_per_forward,trace_avg_ms,clock_ghz,mfma_busy_frac,mfma_busy_frac_at_clock,"
                 "SQ_VALU_MFMA_BUSY_CYCLES,GRBM_GUI_ACTIVE,SQ_BUSY_CYCLES\n")
        for k, r in fams.items():
            c = r["counters_per_launch"]
            fh.write(f"{k.split(':', 1)[1]},{r['launches_per_forward']},{r['trace_avg_ms']:.4f},{r['clock_ghz']:.3f},"
                     f"{r['mfma_busy_frac']:.4f},{r['mfma_busy_frac_at_clock']:.4f},"
                     f"{c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0):.0f},{c.get('GRBM_GUI_ACTIVE', 0):.0f},"
                     f"{c.get('SQ_BUSY_CYCLES', 0):.0f}\n")
    for k, r in sorted(fams.items(), key=lambda kv: -kv[1]["trace_avg_ms"] * kv[1]["launches_per_forward"]):
        print(f"{k:28s} x{r['launches_per_forward']:2d} {r['trace_avg_ms']:7.3f} ms  clk {r['clock_ghz']:.2f} GHz  "
              f"mfma busy {r['mfma_busy_frac']:.3f} (at clock {r['mfma_busy_frac_at_clock']:.3f})")


if __name__ == "__main__":
    main()
