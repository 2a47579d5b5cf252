#!/usr/bin/env python3
"""Sweep the conv1d tile configurations compiled into libtts_mi355x.so over the conv shapes of
the benchmark workload (HiFiGAN-v1, B=32, T=1024 -> T'=1034) and print time / TFLOP/s per tile.
Every tile's output is checked against the default tile's (max |diff| must be fp32-small)."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tts-3_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tts_amd import _native as N  # noqa: E402

B, TP = 32, 1034
SHAPES = []  # (name, Cin, Cout, T, K, dil, res)
for C, L in ((256, 8 * TP), (128, 64 * TP), (64, 128 * TP), (32, 256 * TP)):
    for K in (3, 7, 11):
        SHAPES.append((f"c{C}_k{K}_d3", C, C, L, K, 3, False))
        SHAPES.append((f"c{C}_k{K}_d1res", C, C, L, K, 1, True))


def main():
    args = sys.argv[1:]
    mode = "fp32"
    if args and args[0] in N.MATH_MODES:
        mode, args = args[0], args[1:]
    only = args or None
    dev = torch.device("cuda", 0)
    ntiles = N.lib().tts_op_conv1d_num_tiles(N.MATH_MODES[mode])
    reps = 5
    out = {}
    for name, Cin, Cout, T, K, dil, use_res in SHAPES:
        if only and not any(o in name for o in only):
            continue
        g = torch.Generator().manual_seed(0)
        x = torch.randn(B, Cin, T, generator=g).to(dev)
        w = (torch.randn(Cout, Cin, K, generator=g) / np.sqrt(Cin * K)).numpy()
        bias = (torch.randn(Cout, generator=g) * 0.1).numpy()
        res = torch.randn(B, Cout, T, generator=g).to(dev) if use_res else None
        flops = 2.0 * B * Cout * Cin * K * T
        d = N.TtsConv1dDesc(B, Cin, Cout, T, K, dil, 0, 0.1, 1.0 if use_res else 0.1, 0, 1.0, N.MATH_MODES[mode])
        ref = None
        rows = []
        tiles = [int(t) for t in os.environ["TUNE_TILES"].split(",")] if os.environ.get("TUNE_TILES") else range(ntiles)
        for tile in tiles:
            y = torch.empty(B, Cout, T, device=dev)
            ms = ctypes.c_float(0)
            st = N.lib().tts_op_conv1d_bench(ctypes.byref(d), N.ptr(x), N.ptr(w), N.ptr(bias), N.ptr(res), N.ptr(y),
                                             None, tile, reps, ctypes.byref(ms), N.stream_ptr(dev))
            if st != 0:
                rows.append((tile, None, N.lib().tts_last_error().decode()[:60]))
                continue
            if ref is None:
                ref = y.clone()
                err = 0.0
            else:
                err = (y - ref).abs().max().item()
            if tile == 0 and mode != "fp32":  # compare the first tile against exact fp32
                d32 = N.TtsConv1dDesc(B, Cin, Cout, T, K, dil, 0, 0.1, 1.0 if use_res else 0.1, 0, 1.0, 0)
                y32 = torch.empty_like(y)
                N.call("tts_op_conv1d", ctypes.byref(d32), N.ptr(x), N.ptr(w), N.ptr(bias), N.ptr(res), N.ptr(y32),
                       None, N.stream_ptr(dev))
                err = (y - y32).abs().max().item()
            rows.append((tile, ms.value, err))
        best = min((r for r in rows if r[1] is not None), key=lambda r: r[1])
        print(f"{name:18s} " + " ".join(
            f"t{t}:{ms:6.2f}" + ("!" if isinstance(e, float) and e > 1e-4 else "") if ms is not None else f"t{t}:  --  "
            for t, ms, e in rows) + f"  best t{best[0]} {flops / best[1] / 1e9:6.1f} TF", flush=True)
        out[name] = {"flops": flops, "tiles": {t: ms for t, ms, _ in rows}, "errors": {t: e for t, _, e in rows}}
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(REPO, "gpurun_out", f"tune_conv_{mode}.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
