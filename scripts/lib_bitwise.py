"""Forward outputs of the library named by TTS_MI355X_LIB (or the in-tree one) for a fixed input,
saved to an .npz: run once per library, then compare the files (variant A/Bs that must be bitwise
equal to the in-tree kernels).  usage: python scripts/lib_bitwise.py OUT.npz [compare.npz]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tts-3_amd"))
from tts_amd import synthetic  # noqa: E402
from tts_amd.config import HIFIGAN_V1  # noqa: E402
from tts_amd.vocoder import HifiganGenerator  # noqa: E402

dev = torch.device("cuda", 0)
cfg = dict(in_channels=80, out_channels=1, **HIFIGAN_V1)
sd = synthetic.hifigan_state_dict(**cfg, seed=1234, weight_norm=True)
mel = synthetic.mel(4, 150, seed=3).to(dev)
outs = {}
for mode in ("f16x3", "bf16", "fp32x6"):
    g = HifiganGenerator(**cfg, math_mode=mode)
    g.load_state_dict(sd)
    g.eval()
    g.remove_weight_norm()
    g = g.to(dev)
    outs[mode] = g.inference(mel).cpu().numpy()
np.savez(sys.argv[1], **outs)
if len(sys.argv) > 2:
    ref = np.load(sys.argv[2])
    for k, v in outs.items():
        eq = np.array_equal(v, ref[k])
        print(k, "bitwise equal" if eq else f"DIFFERS max|d|={np.abs(v - ref[k]).max():.3e}")
