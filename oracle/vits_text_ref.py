"""ORACLE — test infrastructure only.  Never imported by the product path (tts-3_amd/).

CPU restatement of the VITS text side of ``Vits.inference`` in ``torch.nn.functional`` (fp32 or
fp64).  Follows Coqui TTS 0.22.0:

* ``TTS/tts/layers/vits/networks.py:29-100``  TextEncoder: emb * sqrt(H), transpose, sequence_mask,
  RelativePositionTransformer(layer_norm_type "2", rel_attn_window_size 4) on x * x_mask,
  stats = proj(x) * x_mask, (m, logs) = split(stats)
* ``TTS/tts/layers/vits/stochastic_duration_predictor.py:11-63``  DilatedDepthSeparableConv:
  x (+ g); per layer y = sep_conv_i(x * mask) (depthwise, k, dilation k^i), LayerNorm2, gelu,
  1x1, LayerNorm2, gelu; x = x + y; return x * mask
* ``:66-83``  ElementwiseAffine reverse: (x - t) * exp(-log_scale) * mask
* ``:86-148``  ConvFlow reverse: h = pre(x0); h = DDS(h, mask, g); h = proj(h) * mask; the
  rational-quadratic spline (``TTS/tts/layers/vits/transforms.py:12-198``, tails "linear",
  inverse) on x1; cat * mask
* ``:150-282``  StochasticDurationPredictor(reverse=True): x = proj(DDS(pre(x) + cond(g))) * mask;
  flows = reversed(flows) without the first ConvFlow (:275-276); z = noise * noise_scale; per flow
  z = flip(z); z = flow(z, mask, g=x, reverse=True); logw = z[:, :1]
* ``TTS/tts/models/vits.py:1137-1152``  durations w = exp(logw) * x_mask * length_scale,
  w_ceil = ceil(w), y_lengths = clamp_min(sum(w_ceil), 1); generate_path
  (``TTS/tts/utils/helpers.py:154-169``); m_p / logs_p = attn^T m_p / logs_p;
  z_p = m_p + noise * exp(logs_p) * noise_scale (no y_mask)
* language embeddings (YourTTS): the text encoder's cat(emb * sqrt(H), lang_emb.expand(T))
  (networks.py:86-91) and the SDP's cond_lang (stochastic_duration_predictor.py:253-254)
* ``TTS/tts/layers/glow_tts/duration_predictor.py:49-68``  the deterministic predictor VITS builds
  with use_sdp=False (vits.py:694-702): x + cond(g) + cond_lang(lang), 2 x (conv -> relu ->
  LayerNorm), proj, * mask
* ``TTS/tts/models/vits.py:944-959``  upsampling_z: F.interpolate(z, scale_factor=[f], "linear"),
  sequence_mask(y_lengths * f)

Pinned against golden vectors of the reference modules (tests/golden/make_goldens.py vits_text).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

from .glow_tts_ref import rel_transformer, sequence_mask

MIN_BIN_WIDTH = 1e-3   # transforms.py:7-9
MIN_BIN_HEIGHT = 1e-3
MIN_DERIVATIVE = 1e-3


def _w(sd, dtype):
    return {k: v.to(dtype) if v.is_floating_point() else v for k, v in sd.items()}


def text_encoder(sd: Dict[str, torch.Tensor], tokens: torch.Tensor, lengths: torch.Tensor, hidden_channels: int = 192,
                 out_channels: int = 192, hidden_channels_ffn: int = 768, num_heads: int = 2, num_layers: int = 6,
                 kernel_size: int = 3, dtype=torch.float64, lang_emb: Optional[torch.Tensor] = None, **_unused):
    """TextEncoder.forward (networks.py:83-100) -> (x, m, logs, x_mask); lang_emb [B, L, 1] is
    concatenated to every token's embedding (:90-91), the transformer then runs at H + L."""
    w = _w(sd, dtype)
    H = hidden_channels
    x = F.embedding(tokens, w["emb.weight"]) * math.sqrt(H)
    if lang_emb is not None:
        x = torch.cat((x, lang_emb.to(dtype).transpose(2, 1).expand(x.size(0), x.size(1), -1)), dim=-1)
    x = x.transpose(1, -1)
    x_mask = sequence_mask(lengths, x.size(2)).unsqueeze(1).to(dtype)
    ep = dict(kernel_size=kernel_size, num_layers=num_layers, num_heads=num_heads, hidden_channels_ffn=hidden_channels_ffn,
              layer_norm_type="2")
    x = rel_transformer(w, x * x_mask, x_mask, ep) * x_mask
    stats = F.conv1d(x, w["proj.weight"], w["proj.bias"]) * x_mask
    m, logs = torch.split(stats, out_channels, dim=1)
    return x, m, logs, x_mask


def _ln2(x, gamma, beta):
    """LayerNorm2 (normalization.py:50-53): F.layer_norm over the channel axis, eps 1e-5."""
    return F.layer_norm(x.transpose(1, -1), (x.size(1),), gamma, beta, 1e-5).transpose(1, -1)


def dds_conv(w, pre: str, x, x_mask, num_layers: int, kernel_size: int, g=None):
    """DilatedDepthSeparableConv.forward (stochastic_duration_predictor.py:46-63)."""
    if g is not None:
        x = x + g
    C = x.size(1)
    for i in range(num_layers):
        d = kernel_size**i
        pad = (kernel_size * d - d) // 2
        y = F.conv1d(x * x_mask, w[f"{pre}.convs_sep.{i}.weight"], w[f"{pre}.convs_sep.{i}.bias"], groups=C,
                     dilation=d, padding=pad)
        y = F.gelu(_ln2(y, w[f"{pre}.norms_1.{i}.gamma"], w[f"{pre}.norms_1.{i}.beta"]))
        y = F.conv1d(y, w[f"{pre}.convs_1x1.{i}.weight"], w[f"{pre}.convs_1x1.{i}.bias"])
        y = F.gelu(_ln2(y, w[f"{pre}.norms_2.{i}.gamma"], w[f"{pre}.norms_2.{i}.beta"]))
        x = x + y
    return x * x_mask


def rq_spline(inputs, uw, uh, ud, inverse: bool, tail_bound: float):
    """unconstrained_rational_quadratic_spline (transforms.py:50-94) with tails "linear":
    inputs [...], uw / uh [..., nb], ud [..., nb - 1] -> (outputs, logabsdet)."""
    inside = (inputs >= -tail_bound) & (inputs <= tail_bound)
    out = inputs.clone()
    lad = torch.zeros_like(inputs)
    ud = F.pad(ud, (1, 1))
    const = float(np.log(np.exp(1 - MIN_DERIVATIVE) - 1))
    ud[..., 0] = const
    ud[..., -1] = const
    if inside.any():
        o, l = _rq_inside(inputs[inside], uw[inside], uh[inside], ud[inside], inverse, -tail_bound, tail_bound)
        out[inside] = o
        lad[inside] = l
    return out, lad


def _rq_inside(x, uw, uh, ud, inverse, left, right):
    """rational_quadratic_spline (transforms.py:97-198) with bottom = left, top = right."""
    nb = uw.shape[-1]
    widths = F.softmax(uw, dim=-1)
    widths = MIN_BIN_WIDTH + (1 - MIN_BIN_WIDTH * nb) * widths
    cumw = F.pad(torch.cumsum(widths, dim=-1), (1, 0), value=0.0)
    cumw = (right - left) * cumw + left
    cumw[..., 0] = left
    cumw[..., -1] = right
    widths = cumw[..., 1:] - cumw[..., :-1]
    der = MIN_DERIVATIVE + F.softplus(ud)
    heights = F.softmax(uh, dim=-1)
    heights = MIN_BIN_HEIGHT + (1 - MIN_BIN_HEIGHT * nb) * heights
    cumh = F.pad(torch.cumsum(heights, dim=-1), (1, 0), value=0.0)
    cumh = (right - left) * cumh + left
    cumh[..., 0] = left
    cumh[..., -1] = right
    heights = cumh[..., 1:] - cumh[..., :-1]
    loc = (cumh if inverse else cumw).clone()
    loc[..., -1] += 1e-6  # searchsorted's eps on the last edge (transforms.py:45-47)
    idx = (torch.sum(x[..., None] >= loc, dim=-1) - 1)[..., None]
    icw = cumw.gather(-1, idx)[..., 0]
    ibw = widths.gather(-1, idx)[..., 0]
    ich = cumh.gather(-1, idx)[..., 0]
    delta = heights / widths
    idl = delta.gather(-1, idx)[..., 0]
    id0 = der.gather(-1, idx)[..., 0]
    id1 = der[..., 1:].gather(-1, idx)[..., 0]
    ih = heights.gather(-1, idx)[..., 0]
    if inverse:
        a = (x - ich) * (id0 + id1 - 2 * idl) + ih * (idl - id0)
        b = ih * id0 - (x - ich) * (id0 + id1 - 2 * idl)
        c = -idl * (x - ich)
        disc = b.pow(2) - 4 * a * c
        root = (2 * c) / (-b - torch.sqrt(disc))
        out = root * ibw + icw
        t1t = root * (1 - root)
        den = idl + (id0 + id1 - 2 * idl) * t1t
        num = idl.pow(2) * (id1 * root.pow(2) + 2 * idl * t1t + id0 * (1 - root).pow(2))
        return out, -(torch.log(num) - 2 * torch.log(den))
    theta = (x - icw) / ibw
    t1t = theta * (1 - theta)
    num = ih * (idl * theta.pow(2) + id0 * t1t)
    den = idl + (id0 + id1 - 2 * idl) * t1t
    out = ich + num / den
    dnum = idl.pow(2) * (id1 * theta.pow(2) + 2 * idl * t1t + id0 * (1 - theta).pow(2))
    return out, torch.log(dnum) - 2 * torch.log(den)


def conv_flow_reverse(w, pre: str, z, x_mask, g, hidden_channels: int, kernel_size: int, num_bins: int = 10,
                      tail_bound: float = 5.0):
    """ConvFlow.forward(reverse=True) (stochastic_duration_predictor.py:122-148) for in_channels 2."""
    x0, x1 = z[:, :1], z[:, 1:]
    h = F.conv1d(x0, w[f"{pre}.pre.weight"], w[f"{pre}.pre.bias"])
    h = dds_conv(w, f"{pre}.convs", h, x_mask, 3, kernel_size, g=g)
    h = F.conv1d(h, w[f"{pre}.proj.weight"], w[f"{pre}.proj.bias"]) * x_mask
    b, c, t = x0.shape
    h = h.reshape(b, c, -1, t).permute(0, 1, 3, 2)
    s = math.sqrt(hidden_channels)
    x1, _ = rq_spline(x1, h[..., :num_bins] / s, h[..., num_bins:2 * num_bins] / s, h[..., 2 * num_bins:],
                      True, tail_bound)
    return torch.cat([x0, x1], 1) * x_mask


def sdp_reverse(sd: Dict[str, torch.Tensor], x: torch.Tensor, x_mask: torch.Tensor, noise: torch.Tensor,
                g: Optional[torch.Tensor] = None, noise_scale: float = 1.0, hidden_channels: int = 192,
                kernel_size: int = 3, num_flows: int = 4, dtype=torch.float64,
                lang_emb: Optional[torch.Tensor] = None, **_unused):
    """StochasticDurationPredictor.forward(x, x_mask, g=g, reverse=True, noise_scale) with the noise
    torch.randn(B, 2, T) the reference draws at :277 given -> logw [B, 1, T]."""
    w = _w(sd, dtype)
    x = x.to(dtype)
    x_mask = x_mask.to(dtype)
    x = F.conv1d(x, w["pre.weight"], w["pre.bias"])
    if g is not None:
        x = x + F.conv1d(g.to(dtype), w["cond.weight"], w["cond.bias"])
    if lang_emb is not None:  # :253-254
        x = x + F.conv1d(lang_emb.to(dtype), w["cond_lang.weight"], w["cond_lang.bias"])
    x = dds_conv(w, "convs", x, x_mask, 3, kernel_size)
    x = F.conv1d(x, w["proj.weight"], w["proj.bias"]) * x_mask
    z = noise.to(dtype) * noise_scale
    for f in [*range(num_flows, 1, -1), 0]:  # reversed(flows)[:-2] + [flows[0]] (:275-276)
        z = torch.flip(z, [1])
        if f == 0:  # ElementwiseAffine reverse (:81-83)
            z = (z - w["flows.0.translation"]) * torch.exp(-w["flows.0.log_scale"]) * x_mask
        else:
            z = conv_flow_reverse(w, f"flows.{f}", z, x_mask, x, hidden_channels, kernel_size)
    return z[:, :1]


def vits_durations(logw: torch.Tensor, x_mask: torch.Tensor, length_scale: float = 1.0):
    """vits.py:1137-1149 -> (w_ceil [B,1,T_x], y_lengths [B] int64)."""
    w = torch.exp(logw) * x_mask * length_scale
    w_ceil = torch.ceil(w)
    y_lengths = torch.clamp_min(torch.sum(w_ceil, [1, 2]), 1).long()
    return w_ceil, y_lengths


def vits_expand(w_ceil, x_mask, y_lengths, m_p, logs_p, noise=None, noise_scale: float = 0.667):
    """vits.py:1150-1155 (+ helpers.generate_path) -> (z_p, y_mask, m_p', logs_p', attn [B,T_x,T_y])."""
    y_mask = sequence_mask(y_lengths, None).unsqueeze(1).to(x_mask.dtype)
    attn_mask = x_mask * y_mask.transpose(1, 2)  # [B, T_y, T_x]
    t_y = y_mask.size(2)
    cum = torch.cumsum(w_ceil.squeeze(1), 1)
    path = (torch.arange(t_y, dtype=cum.dtype)[None, None, :] < cum[:, :, None]).to(x_mask.dtype)
    path = path - F.pad(path, [0, 0, 1, 0])[:, :-1]
    attn = path * attn_mask.transpose(1, 2)
    mp = torch.matmul(attn.transpose(1, 2), m_p.transpose(1, 2)).transpose(1, 2)
    lp = torch.matmul(attn.transpose(1, 2), logs_p.transpose(1, 2)).transpose(1, 2)
    if noise is None:
        noise = torch.zeros_like(mp)
    z_p = mp + noise.to(mp.dtype) * torch.exp(lp) * noise_scale
    return z_p, y_mask, mp, lp, attn


def dp_forward(sd: Dict[str, torch.Tensor], x: torch.Tensor, x_mask: torch.Tensor, g: Optional[torch.Tensor] = None,
               lang_emb: Optional[torch.Tensor] = None, kernel_size: int = 3, dtype=torch.float64, **_unused):
    """DurationPredictor.forward (glow_tts/duration_predictor.py:49-68; dropout is identity at eval)
    -> logw [B, 1, T]."""
    from .glow_tts_ref import layer_norm

    w = _w(sd, dtype)
    x = x.to(dtype)
    x_mask = x_mask.to(dtype)
    if g is not None:
        x = x + F.conv1d(g.to(dtype), w["cond.weight"], w["cond.bias"])
    if lang_emb is not None:
        x = x + F.conv1d(lang_emb.to(dtype), w["cond_lang.weight"], w["cond_lang.bias"])
    x = F.conv1d(x * x_mask, w["conv_1.weight"], w["conv_1.bias"], padding=kernel_size // 2)
    x = layer_norm(torch.relu(x), w["norm_1.gamma"], w["norm_1.beta"])
    x = F.conv1d(x * x_mask, w["conv_2.weight"], w["conv_2.bias"], padding=kernel_size // 2)
    x = layer_norm(torch.relu(x), w["norm_2.gamma"], w["norm_2.beta"])
    x = F.conv1d(x * x_mask, w["proj.weight"], w["proj.bias"])
    return x * x_mask


def upsample_z(z: torch.Tensor, y_lengths: torch.Tensor, factor: float):
    """Vits.upsampling_z (vits.py:944-959) with encoder_sample_rate and interpolate_z:
    (F.interpolate(z, scale_factor=[factor], mode="linear"), sequence_mask(y_lengths * factor))."""
    z2 = F.interpolate(z, scale_factor=[factor], mode="linear")
    lens = y_lengths * factor  # long * python float -> float32 lengths
    seq = torch.arange(lens.max(), dtype=lens.dtype)  # helpers.sequence_mask: arange of a float max
    y_mask = (seq[None, :] < lens[:, None]).to(z.dtype).unsqueeze(1)
    return z2, y_mask
