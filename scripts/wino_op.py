#!/usr/bin/env python3
"""Time one conv1d shape through tts_op_conv1d_bench (for rocprofv3 counter passes):
python scripts/wino_op.py <tile> <C> <K> <dil> <res 0/1> [reps] [Cin]  (B=32, T of the C-channel stage)"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tts-3_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tts_amd import _native as N  # noqa: E402

tile, C, K, dil, use_res = (int(v) for v in sys.argv[1:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
Cin = int(sys.argv[7]) if len(sys.argv) > 7 else C
B, T = 32, {256: 8 * 1034, 128: 64 * 1034, 64: 128 * 1034, 32: 256 * 1034}[C]
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
x = torch.randn(B, Cin, T, generator=g).to(dev)
w = (torch.randn(C, Cin, K, generator=g) / np.sqrt(Cin * K)).numpy()
bias = (torch.randn(C, generator=g) * 0.1).numpy()
res = torch.randn(B, C, T, generator=g).to(dev) if use_res else None
y = torch.empty(B, C, T, device=dev)
d = N.TtsConv1dDesc(B, Cin, C, T, K, dil, 0, 0.1, 1.0 if use_res else 0.1, 0, 1.0, N.MATH_MODES["f16x3"])
ms = ctypes.c_float(0)
N.call("tts_op_conv1d_bench", ctypes.byref(d), N.ptr(x), N.ptr(w), N.ptr(bias), N.ptr(res), N.ptr(y), None, tile, reps,
       ctypes.byref(ms), N.stream_ptr(dev))
print(f"tile {tile} C{C} Cin{Cin} K{K} d{dil} res{use_res}: {ms.value:.3f} ms, {2.0 * B * C * Cin * K * T / ms.value / 1e9:.1f} TF")
