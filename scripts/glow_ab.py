"""Glow decoder side line alone (bench.glow_bench, no CPU baseline), for A/B runs: prints ms/step."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tts-3_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
for mode in sys.argv[1:] or ["f16x3"]:
    r = bench.glow_bench(dev, mode, steps=30, warmup=5, cpu=False)
    print(json.dumps({"mode": mode, "ms_per_step": round(r["ms_per_step"], 4), "launches": r["launches_per_step"],
                      "kernel_sum_ms": round(r["kernel_sum_ms"], 3),
                      "top": dict(list(r["breakdown_ms"].items())[:4])}))
