#!/usr/bin/env python3
"""Phase timing of the 8-wave Winograd conv from a WINO_STAMPS=1 build (ab/lib_stamps.so):
python scripts/wino_stamps.py <C> <K> <dil>   (B=32 bench shapes, zmode 0)"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tts-3_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tts_amd import _native as N  # noqa: E402

C, K, dil = (int(v) for v in sys.argv[1:4])
B, T = 32, {256: 8 * 1034, 128: 64 * 1034}[C]
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
x = torch.randn(B, C, T, generator=g).to(dev)
w = (torch.randn(C, C, K, generator=g) / np.sqrt(C * K)).numpy()
bias = (torch.randn(C, generator=g) * 0.1).numpy()
y = torch.empty(B, C, T, device=dev)
D = dil
J = 64 // D
TW = 4 * D * J
nwg = -(-T // TW) * (C // 128) * B
z = torch.zeros(nwg * 8 * 32 * 2, dtype=torch.float32, device=dev)
d = N.TtsConv1dDesc(B, C, C, T, K, dil, 0, 0.1, 0.1, 0, 1.0, N.MATH_MODES["f16x3"])
ms = ctypes.c_float(0)
N.call("tts_op_conv1d_bench", ctypes.byref(d), N.ptr(x), N.ptr(w), N.ptr(bias), None, N.ptr(y), N.ptr(z), 21, 1,
       ctypes.byref(ms), N.stream_ptr(dev))
st = z.cpu().numpy().view(np.uint64).reshape(nwg, 8, 32).astype(np.int64)
nc = C // 16
print(f"C{C} K{K} d{dil}: {ms.value:.3f} ms, {nwg} workgroups, {nc} chunks")
t0 = st[:, :, 0]
def q(a):
    a = np.asarray(a, np.float64).ravel()
    return f"med {np.median(a):8.0f}  p10 {np.percentile(a, 10):8.0f}  p90 {np.percentile(a, 90):8.0f}"
for grp in (0, 1):
    s = st[:, 4 * grp:4 * grp + 4, :]
    print(f"-- waves {4 * grp}-{4 * grp + 3}")
    print(" prologue dma wait ", q(s[:, :, 1] - s[:, :, 0]) if grp == 1 else "")
    print(" prologue total    ", q(s[:, :, 2] - s[:, :, 0]))
    for k in range(min(nc, 8)):
        body = s[:, :, 4 + 2 * k] - s[:, :, 3 + 2 * k]
        print(f" chunk {k} body      ", q(body))
        if k + 1 < min(nc, 8):
            print(f" chunk {k} barrier   ", q(s[:, :, 3 + 2 * (k + 1)] - s[:, :, 4 + 2 * k]))
    print(" loop->partials    ", q(s[:, :, 20] - s[:, :, 4 + 2 * (min(nc, 8) - 1)]))
    print(" exchange          ", q(s[:, :, 21] - s[:, :, 20]))
    print(" finish (stores)   ", q(s[:, :, 22] - s[:, :, 21]))
    print(" total             ", q(s[:, :, 22] - s[:, :, 0]))
# dispatch: workgroup start times sorted
start = np.sort(t0.min(axis=1))
end = np.sort(st[:, :, 22].max(axis=1))
span = end.max() - start.min()
print("kernel span (cycles)", span, "sum of wg lifetimes / 256 CUs", (st[:, :, 22].max(axis=1) - t0.min(axis=1)).sum() / 256)
