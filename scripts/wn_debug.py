"""Fused vs unfused WN layer: max |diff| and differing count per (mode, L) on one flow block."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tts-3_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402
from test_glow_gpu import build  # noqa: E402

dev = torch.device("cuda", 0)
for mode in ["fp32x6", "bf16", "f16x3"]:
    for L in [1, 2, 4]:
        for T, lens in [(64, [64]), (301, [301, 150, 9])]:
            cfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=1,
                       num_coupling_layers=L, num_splits=4, num_squeeze=2)
            gen = torch.Generator().manual_seed(31)
            B = len(lens)
            x = torch.randn(B, 80, T, generator=gen).to(dev)
            m = (torch.arange(T)[None] < torch.tensor(lens)[:, None]).float().unsqueeze(1).to(dev)
            outs = []
            for on in ("1", "0"):
                os.environ["TTS_MI355X_WN_LAYER"] = on
                outs.append(build(cfg, 23, dev, mode)(x, m, reverse=True)[0])
            d = (outs[0] - outs[1]).abs()
            idx = torch.nonzero(d)
            print(mode, "L", L, "T", T, "max", d.max().item(), "ndiff", idx.shape[0], "of", d.numel(),
                  "first", idx[:4].tolist(), flush=True)
