#!/usr/bin/env python3
"""Busy coverage of a rocprofv3 kernel trace: cut the library's dispatches into the bench's timed
steps (gaps > 1 ms between them), and for each step report wall time, the union of kernel
intervals (time with at least one kernel running), and the time with two or more running."""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    if "tts::" not in r["Kernel_Name"]:
        continue
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
steps, cur = [], [rows[0]]
for a in rows[1:]:
    if a[0] - max(e for _, e, _ in cur) > 1_000_000:  # 1 ms idle: a new step / phase
        steps.append(cur)
        cur = []
    cur.append(a)
steps.append(cur)
for i, st in enumerate(steps):
    t0, t1 = st[0][0], max(e for _, e, _ in st)
    ev = sorted([(s, 1) for s, _, _ in st] + [(e, -1) for _, e, _ in st])
    busy = multi = 0
    depth, last = 0, ev[0][0]
    for t, d in ev:
        if depth >= 1:
            busy += t - last
        if depth >= 2:
            multi += t - last
        depth += d
        last = t
    print(f"phase {i}: {len(st)} dispatches, wall {(t1 - t0) / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms "
          f"({busy / (t1 - t0):.3f}), >=2 kernels {multi / 1e6:.2f} ms")
