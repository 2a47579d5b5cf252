"""Per-launch breakdown of the Glow-TTS encoder at config 3 (B=16 x 128 tokens)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tts-3_amd"))
import torch  # noqa: E402

from tts_amd import synthetic  # noqa: E402
from tts_amd.config import GLOW_TTS_ENCODER as E  # noqa: E402
from tts_amd.tts import Encoder  # noqa: E402

dev = torch.device("cuda", 0)
B, T = int(sys.argv[1]) if len(sys.argv) > 1 else 16, int(sys.argv[2]) if len(sys.argv) > 2 else 128
cfg = dict(E, num_chars=64)
e = Encoder(64, cfg["out_channels"], cfg["hidden_channels"], cfg["hidden_channels_dp"], cfg["encoder_type"],
            cfg["encoder_params"], mean_only=True, use_prenet=True)
e.load_state_dict(synthetic.glow_encoder_state_dict(**cfg, seed=1))
e = e.to(dev)
tok = synthetic.tokens(B, T, 64, seed=1).to(dev)
lens = torch.full((B,), T, dtype=torch.int64, device=dev)
for _ in range(3):
    e(tok, lens)
fam = {}
for _ in range(5):
    _, rows = e.profile(tok, lens)
    for r in rows:
        f = fam.setdefault(r["name"], [0.0, 0, 0.0])
        f[0] += r["ms"] / 5
        f[1] += 1
        f[2] += r["flops"] / 5
tot = sum(v[0] for v in fam.values())
print(json.dumps({k: {"ms": round(v[0], 4), "launches": v[1] // 5, "tflops": round(v[2] / max(v[0], 1e-9) / 1e9, 2)}
                  for k, v in sorted(fam.items(), key=lambda kv: -kv[1][0])}, indent=1))
print("total ms", tot)
