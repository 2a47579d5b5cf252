"""Side lines alone (bench.vits_bench, bench.xtts_decoder_bench, bench.glow_tts_e2e_bench), for
A/B runs of environment switches: prints ms/step per variant."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tts-3_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
out = {}
v = bench.vits_bench(dev)
out["vits"] = {k: round(x["ms_per_step"], 3) for k, x in v["variants"].items()}
out["xtts"] = round(bench.xtts_decoder_bench(dev, "f16x3")["ms_per_step"], 3)
e = bench.glow_tts_e2e_bench(dev, {"fp32_faithful": ("f16x3", "f16x3"), "bf16": ("bf16", "bf16")})
out["e2e"] = {k: round(x["ms_per_step"], 3) for k, x in e["variants"].items()}
if os.environ.get("SIDE_VITS_TTS"):
    t = bench.vits_tts_bench(dev)
    out["vits_tts"] = {k: round(x["ms_per_step"], 3) for k, x in t["variants"].items()}
print(json.dumps(out))
