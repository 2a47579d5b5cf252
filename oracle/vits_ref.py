"""ORACLE — test infrastructure only.  Never imported by the product path (tts-3_amd/).

CPU restatement of the VITS flow (both directions) and the posterior encoder in
``torch.nn.functional``, fp32 or fp64.  Follows Coqui TTS 0.22.0:

* ``TTS/tts/layers/vits/networks.py:217-232``  ResidualCouplingBlocks.forward(reverse=True):
  for flow in reversed(flows): x = flip(x, [1]); x = flow(x, mask, g, reverse=True)
* ``:144-166``  ResidualCouplingBlock.forward (mean_only=True, the VITS setting :213):
  x0, x1 = split halves; h = pre(x0) * mask; h = WN(h, mask, g); m = post(h) * mask;
  x1 = (x1 - m) * exp(-0) * mask; cat(x0, x1)
* ``:225-228``  forward(reverse=False): for flow in flows: x = flow(x); x = flip(x, [1])
* ``:235-288``  PosteriorEncoder: pre -> WN -> proj -> split -> (m + eps * exp(logs)) * mask
* ``TTS/tts/layers/generic/wavenet.py:94-115``  WN with the optional cond_layer (:98-99,
  g_l = cond[:, 2H*i : 2H*(i+1)], :103-107) and the fused gate (:6-13)

VITS keeps its weight-norm parametrizations at inference (no remove_weight_norm anywhere in
vits.py), so weights are evaluated in the run dtype.  Pinned against golden vectors of the
reference module (tests/golden/make_goldens.py).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn.functional as F

from .hifigan_ref import fold_weight_norm


def _wn(w, h, mask, g, pre, L, H, kernel_size, dilation_rate):
    output = torch.zeros_like(h)
    cond = None
    if g is not None:
        cond = F.conv1d(g, w[f"{pre}.cond_layer.weight"], w[f"{pre}.cond_layer.bias"])
    for i in range(L):
        d = dilation_rate**i
        x_in = F.conv1d(h, w[f"{pre}.in_layers.{i}.weight"], w[f"{pre}.in_layers.{i}.bias"],
                        dilation=d, padding=int((kernel_size * d - d) / 2))
        g_l = cond[:, i * 2 * H : (i + 1) * 2 * H] if cond is not None else torch.zeros_like(x_in)
        in_act = x_in + g_l
        acts = torch.tanh(in_act[:, :H]) * torch.sigmoid(in_act[:, H:])
        rs = F.conv1d(acts, w[f"{pre}.res_skip_layers.{i}.weight"], w[f"{pre}.res_skip_layers.{i}.bias"])
        if i < L - 1:
            h = (h + rs[:, :H]) * mask
            output = output + rs[:, H:]
        else:
            output = output + rs
    return output * mask


def vits_flow_reverse(
    sd: Dict[str, torch.Tensor],
    x: torch.Tensor,
    x_mask: torch.Tensor,
    g: Optional[torch.Tensor] = None,
    channels: int = 192,
    hidden_channels: int = 192,
    kernel_size: int = 5,
    dilation_rate: int = 1,
    num_layers: int = 4,
    num_flows: int = 4,
    dtype=torch.float64,
    **_unused,
):
    w = fold_weight_norm(sd, dtype, dtype)
    x = x.to(dtype)
    x_mask = x_mask.to(dtype)
    g = g.to(dtype) if g is not None else None
    half = channels // 2
    for f in reversed(range(num_flows)):
        pre = f"flows.{f}"
        x = torch.flip(x, [1])
        x0, x1 = x[:, :half], x[:, half:]
        h = F.conv1d(x0, w[f"{pre}.pre.weight"], w[f"{pre}.pre.bias"]) * x_mask
        h = _wn(w, h, x_mask, g, f"{pre}.enc", num_layers, hidden_channels, kernel_size, dilation_rate)
        m = F.conv1d(h, w[f"{pre}.post.weight"], w[f"{pre}.post.bias"]) * x_mask
        x1 = (x1 - m) * torch.exp(-torch.zeros_like(m)) * x_mask
        x = torch.cat([x0, x1], 1)
    return x


def vits_flow_forward(
    sd: Dict[str, torch.Tensor],
    x: torch.Tensor,
    x_mask: torch.Tensor,
    g: Optional[torch.Tensor] = None,
    channels: int = 192,
    hidden_channels: int = 192,
    kernel_size: int = 5,
    dilation_rate: int = 1,
    num_layers: int = 4,
    num_flows: int = 4,
    dtype=torch.float64,
    **_unused,
):
    """ResidualCouplingBlocks.forward(reverse=False) (networks.py:225-228): for flow in flows:
    x = flow(x) (:154-160: x1 = m + x1 * exp(0) * mask); x = flip(x, [1])."""
    w = fold_weight_norm(sd, dtype, dtype)
    x = x.to(dtype)
    x_mask = x_mask.to(dtype)
    g = g.to(dtype) if g is not None else None
    half = channels // 2
    for f in range(num_flows):
        pre = f"flows.{f}"
        x0, x1 = x[:, :half], x[:, half:]
        h = F.conv1d(x0, w[f"{pre}.pre.weight"], w[f"{pre}.pre.bias"]) * x_mask
        h = _wn(w, h, x_mask, g, f"{pre}.enc", num_layers, hidden_channels, kernel_size, dilation_rate)
        m = F.conv1d(h, w[f"{pre}.post.weight"], w[f"{pre}.post.bias"]) * x_mask
        x1 = m + x1 * torch.exp(torch.zeros_like(m)) * x_mask
        x = torch.flip(torch.cat([x0, x1], 1), [1])
    return x


def vits_posterior(
    sd: Dict[str, torch.Tensor],
    x: torch.Tensor,
    x_mask: torch.Tensor,
    eps: Optional[torch.Tensor] = None,
    g: Optional[torch.Tensor] = None,
    num_layers: int = 16,
    hidden_channels: int = 192,
    out_channels: int = 192,
    kernel_size: int = 5,
    dilation_rate: int = 1,
    dtype=torch.float64,
    **_unused,
):
    """PosteriorEncoder.forward (networks.py:275-288) with the noise given: h = pre(x) * mask;
    h = WN(h, mask, g); stats = proj(h) * mask; m, logs = split; z = (m + eps * exp(logs)) * mask.
    Returns (z, m, logs)."""
    w = fold_weight_norm(sd, dtype, dtype)
    x = x.to(dtype)
    x_mask = x_mask.to(dtype)
    g = g.to(dtype) if g is not None else None
    h = F.conv1d(x, w["pre.weight"], w["pre.bias"]) * x_mask
    h = _wn(w, h, x_mask, g, "enc", num_layers, hidden_channels, kernel_size, dilation_rate)
    stats = F.conv1d(h, w["proj.weight"], w["proj.bias"]) * x_mask
    m, logs = torch.split(stats, out_channels, dim=1)
    e = eps.to(dtype) if eps is not None else torch.zeros_like(m)
    return (m + e * torch.exp(logs)) * x_mask, m, logs
