"""ORACLE — test infrastructure only.  Never imported by the product path (tts-3_amd/).

CPU restatement of the Glow-TTS decoder flow (reverse direction, the inference path) in
``torch.nn.functional``, fp32 or fp64.  Follows Coqui TTS 0.22.0:

* ``TTS/tts/layers/glow_tts/decoder.py:8-28``   squeeze (odd-index mask, x * mask)
* ``:31-47``    unsqueeze (mask repeated, x * mask)
* ``:113-137``  forward(reverse=True): squeeze -> reversed(flows) -> unsqueeze
* ``TTS/tts/layers/generic/normalization.py:96-98``  ActNorm reverse: (x - bias) * exp(-logs) * mask
* ``TTS/tts/layers/glow_tts/glow.py:102-137``  InvConvNear: channel regroup view(b,2,c/S,S/2,t)
  .permute(0,1,3,2,4), 1x1 conv2d with W^-1 (torch.inverse, :123/:140), regroup back, * mask
* ``glow.py:201-230``  CouplingBlock reverse: h = start(x0)*mask; WN; out = end(h);
  t = out[:C/2], s = out[C/2:]; z1 = (x1 - t) * exp(-s) * mask; cat(x0, z1)
* ``TTS/tts/layers/generic/wavenet.py:94-115`` (+ the fused gate :6-13): g_l = rows
  [2Hl, 2H(l+1)) of cond_layer(g) (:98-107, weight norm folded by store_inverse :117-123), or 0

Pinned against golden vectors of the reference module (tests/golden/make_goldens.py).
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

from .hifigan_ref import fold_weight_norm


def squeeze(x, x_mask, num_sqz=2):
    b, c, t = x.size()
    t = (t // num_sqz) * num_sqz
    x = x[:, :, :t]
    x_sqz = x.view(b, c, t // num_sqz, num_sqz).permute(0, 3, 1, 2).contiguous().view(b, c * num_sqz, t // num_sqz)
    x_mask = x_mask[:, :, num_sqz - 1 :: num_sqz]
    return x_sqz * x_mask, x_mask


def unsqueeze(x, x_mask, num_sqz=2):
    b, c, t = x.size()
    x_unsqz = x.view(b, num_sqz, c // num_sqz, t).permute(0, 2, 3, 1).contiguous().view(b, c // num_sqz, t * num_sqz)
    x_mask = x_mask.unsqueeze(-1).repeat(1, 1, 1, num_sqz).view(b, 1, t * num_sqz)
    return x_unsqz * x_mask, x_mask


def _wn(w, h, mask, L, H, kernel_size, dilation_rate, pre, g=None):
    output = torch.zeros_like(h)
    if g is not None:
        g = F.conv1d(g, w[f"{pre}.wn.cond_layer.weight"], w[f"{pre}.wn.cond_layer.bias"])
    for i in range(L):
        d = dilation_rate**i
        x_in = F.conv1d(h, w[f"{pre}.wn.in_layers.{i}.weight"], w[f"{pre}.wn.in_layers.{i}.bias"],
                        dilation=d, padding=int((kernel_size * d - d) / 2))
        if g is not None:
            x_in = x_in + g[:, i * 2 * H:(i + 1) * 2 * H, :]
        acts = torch.tanh(x_in[:, :H]) * torch.sigmoid(x_in[:, H:])
        rs = F.conv1d(acts, w[f"{pre}.wn.res_skip_layers.{i}.weight"], w[f"{pre}.wn.res_skip_layers.{i}.bias"])
        if i < L - 1:
            h = (h + rs[:, :H]) * mask
            output = output + rs[:, H:]
        else:
            output = output + rs
    return output * mask


def glow_decoder_reverse(
    sd: Dict[str, torch.Tensor],
    x: torch.Tensor,
    x_mask: torch.Tensor,
    in_channels: int = 80,
    hidden_channels: int = 192,
    kernel_size: int = 5,
    dilation_rate: int = 1,
    num_flow_blocks: int = 12,
    num_coupling_layers: int = 4,
    num_splits: int = 4,
    num_squeeze: int = 2,
    sigmoid_scale: bool = False,
    dtype=torch.float64,
    fold_dtype=torch.float32,
    g: torch.Tensor = None,
    **_unused,
):
    """Decoder.forward(x, x_mask, g, reverse=True)[0]; g: speaker vector [B, c_in, 1] or None."""
    # store_inverse (glow.py:232-233) folds the WN layers' weight norm at load (fp32), but
    # CouplingBlock.start keeps its parametrization, so it is evaluated in the run dtype.
    w = fold_weight_norm({k: v for k, v in sd.items() if ".start." not in k}, dtype, fold_dtype)
    w.update(fold_weight_norm({k: v for k, v in sd.items() if ".start." in k}, dtype, dtype))
    x = x.to(dtype)
    x_mask = x_mask.to(dtype)
    if g is not None:
        g = g.to(dtype)
    if num_squeeze > 1:
        x, x_mask = squeeze(x, x_mask, num_squeeze)
    C2 = x.size(1)
    S = num_splits
    H = hidden_channels
    for f in reversed(range(num_flow_blocks)):
        a, c, cb = 3 * f, 3 * f + 1, 3 * f + 2
        pre = f"flows.{cb}"
        # CouplingBlock reverse (glow.py:210-230)
        x0, x1 = x[:, : C2 // 2], x[:, C2 // 2 :]
        h = F.conv1d(x0, w[f"{pre}.start.weight"], w[f"{pre}.start.bias"]) * x_mask
        h = _wn(w, h, x_mask, num_coupling_layers, H, kernel_size, dilation_rate, pre, g)
        out = F.conv1d(h, w[f"{pre}.end.weight"], w[f"{pre}.end.bias"])
        t, s = out[:, : C2 // 2], out[:, C2 // 2 :]
        if sigmoid_scale:
            s = torch.log(1e-6 + torch.sigmoid(s + 2))
        z1 = (x1 - t) * torch.exp(-s) * x_mask
        x = torch.cat([x0, z1], 1)
        # InvConvNear reverse (glow.py:108-137)
        b, cc, tt = x.size()
        winv = w.get(f"flows.{c}.weight_inv")
        if winv is None:
            # store_inverse (glow.py:139-141): fp32 inverse of the parameter, which is
            # column-major in the reference (born from torch.linalg.qr, :96; load_state_dict
            # keeps the layout), so LAPACK is handed the Fortran-ordered matrix.
            wf = w[f"flows.{c}.weight"].float()
            winv = torch.inverse(wf.t().contiguous().t()).to(dtype)
        xg = x.view(b, 2, cc // S, S // 2, tt).permute(0, 1, 3, 2, 4).contiguous().view(b, S, cc // S, tt)
        z = F.conv2d(xg, winv.view(S, S, 1, 1))
        x = z.view(b, 2, S // 2, cc // S, tt).permute(0, 1, 3, 2, 4).contiguous().view(b, cc, tt) * x_mask
        # ActNorm reverse (normalization.py:96-98)
        x = (x - w[f"flows.{a}.bias"]) * torch.exp(-w[f"flows.{a}.logs"]) * x_mask
    if num_squeeze > 1:
        x, x_mask = unsqueeze(x, x_mask, num_squeeze)
    return x


def glow_decoder_forward(
    sd: Dict[str, torch.Tensor],
    x: torch.Tensor,
    x_mask: torch.Tensor,
    in_channels: int = 80,
    hidden_channels: int = 192,
    kernel_size: int = 5,
    dilation_rate: int = 1,
    num_flow_blocks: int = 12,
    num_coupling_layers: int = 4,
    num_splits: int = 4,
    num_squeeze: int = 2,
    sigmoid_scale: bool = False,
    dtype=torch.float64,
    fold_dtype=torch.float32,
    g: torch.Tensor = None,
    **_unused,
):
    """Decoder.forward(x, x_mask, g, reverse=False) -> (z, logdet [B]) (decoder.py:119-133):
    squeeze, then per block in order ActNorm (normalization.py:99-101: z = (bias + exp(logs) * x) *
    mask, logdet = sum(logs) * x_len), InvConvNear (glow.py:126-135: conv2d with W itself,
    logdet = logdet(W) * (C / S) * x_len), CouplingBlock (glow.py:225-227: z1 = (t + exp(s) * x1) *
    mask, logdet = sum(s * mask)); unsqueeze."""
    w = fold_weight_norm({k: v for k, v in sd.items() if ".start." not in k}, dtype, fold_dtype)
    w.update(fold_weight_norm({k: v for k, v in sd.items() if ".start." in k}, dtype, dtype))
    x = x.to(dtype)
    x_mask = x_mask.to(dtype)
    if g is not None:
        g = g.to(dtype)
    if num_squeeze > 1:
        x, x_mask = squeeze(x, x_mask, num_squeeze)
    C2 = x.size(1)
    S = num_splits
    H = hidden_channels
    x_len = torch.sum(x_mask, [1, 2])
    logdet = torch.zeros(x.size(0), dtype=dtype)
    for f in range(num_flow_blocks):
        a, c, cb = 3 * f, 3 * f + 1, 3 * f + 2
        # ActNorm forward
        x = (w[f"flows.{a}.bias"] + torch.exp(w[f"flows.{a}.logs"]) * x) * x_mask
        logdet = logdet + torch.sum(w[f"flows.{a}.logs"]) * x_len
        # InvConvNear forward
        b, cc, tt = x.size()
        wf = w[f"flows.{c}.weight"]
        xg = x.view(b, 2, cc // S, S // 2, tt).permute(0, 1, 3, 2, 4).contiguous().view(b, S, cc // S, tt)
        z = F.conv2d(xg, wf.view(S, S, 1, 1))
        x = z.view(b, 2, S // 2, cc // S, tt).permute(0, 1, 3, 2, 4).contiguous().view(b, cc, tt) * x_mask
        logdet = logdet + torch.logdet(wf) * (cc / S) * x_len
        # CouplingBlock forward
        pre = f"flows.{cb}"
        x0, x1 = x[:, : C2 // 2], x[:, C2 // 2 :]
        h = F.conv1d(x0, w[f"{pre}.start.weight"], w[f"{pre}.start.bias"]) * x_mask
        h = _wn(w, h, x_mask, num_coupling_layers, H, kernel_size, dilation_rate, pre, g)
        out = F.conv1d(h, w[f"{pre}.end.weight"], w[f"{pre}.end.bias"])
        t, s = out[:, : C2 // 2], out[:, C2 // 2 :]
        if sigmoid_scale:
            s = torch.log(1e-6 + torch.sigmoid(s + 2))
        z1 = (t + torch.exp(s) * x1) * x_mask
        logdet = logdet + torch.sum(s * x_mask, [1, 2])
        x = torch.cat([x0, z1], 1)
    if num_squeeze > 1:
        x, x_mask = unsqueeze(x, x_mask, num_squeeze)
    return x, logdet
