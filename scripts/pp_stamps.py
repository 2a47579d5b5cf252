#!/usr/bin/env python3
"""Phase timing of the ping-pong ResBlock pair kernel from a PP_STAMPS=1 build:
TTS_MI355X_LIB=ab/lib_ppst.so python scripts/pp_stamps.py
Runs one bench-shape HiFiGAN-v1 forward (f16x3, B=32 x 1024) and prints the median cycles of each
phase of periods 8..23 of workgroups 0..7 of the last C=64, K=11 pair launch without MRF gathers."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tts-3_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tts_amd import _native as N  # noqa: E402
from tts_amd import synthetic  # noqa: E402
from tts_amd.config import HIFIGAN_V1  # noqa: E402
from tts_amd.vocoder import HifiganGenerator  # noqa: E402

dev = torch.device("cuda", 0)
cfg = dict(in_channels=80, out_channels=1, **HIFIGAN_V1)
g = HifiganGenerator(**cfg, math_mode="f16x3")
g.load_state_dict(synthetic.hifigan_state_dict(**cfg, seed=1234, weight_norm=True))
g.eval()
g.remove_weight_norm()
g = g.to(dev)
mel = synthetic.mel(32, 1024, seed=0).to(dev)
for _ in range(2):
    g.inference(mel)
torch.cuda.synchronize()
buf = np.zeros((8, 16, 8, 8), np.uint64)
lib = N.lib()
assert lib.tts_debug_pp_stamps(buf.ctypes.data_as(ctypes.c_void_p)) == 0
st = buf.astype(np.int64)


def q(a):
    a = np.asarray(a, np.float64).ravel()
    return f"med {np.median(a):7.0f}  p10 {np.percentile(a, 10):7.0f}  p90 {np.percentile(a, 90):7.0f}"


names = {0: "A (convs1)", 1: "B (convs2)"}
for grp in (0, 1):
    s = st[:, :, 4 * grp:4 * grp + 4, :]
    print(f"-- {names[grp]}")
    if grp == 0:
        print(" phase 1: convs1 loop   ", q(s[..., 1] - s[..., 0]))
        print(" phase 1: lrelu/max     ", q(s[..., 2] - s[..., 1]))
    else:
        print(" phase 1: epilogue      ", q(s[..., 2] - s[..., 0]))
    print(" B1 wait                ", q(s[..., 3] - s[..., 2]))
    if grp == 0:
        print(" phase 2: xt split/store", q(s[..., 4] - s[..., 3]))
        print(" phase 2: window store  ", q(s[..., 5] - s[..., 4]))
        print(" phase 2: -> B2 arrive  ", q(s[..., 6] - s[..., 5]))
    else:
        print(" phase 2: convs2 loop   ", q(s[..., 6] - s[..., 3]))
    print(" B2 wait                ", q(s[..., 7] - s[..., 6]))
    print(" period                 ", q(s[..., 7] - s[..., 0]))
