"""ORACLE — test infrastructure only.  Never imported by the product path (tts-3_amd/).

CPU restatement of the Glow-TTS text side of inference in ``torch.nn.functional`` (fp32 or
fp64): the rel_pos_transformer ``Encoder`` and the duration / alignment glue of
``GlowTTS.inference``.  Follows Coqui TTS 0.22.0:

* ``TTS/tts/layers/glow_tts/encoder.py:143-179``  Encoder.forward: emb * sqrt(H), transpose,
  sequence_mask, prenet, transformer, proj_m (proj_s or zeros), duration predictor on x
* ``TTS/tts/layers/glow_tts/glow.py:55-67``  ResidualConv1dLayerNormBlock (prenet)
* ``TTS/tts/layers/glow_tts/transformer.py:117-201``  RelativePositionMultiHeadAttention
  (scores / sqrt(d_k), relative-key logits, masked_fill(-1e4), softmax, relative values;
  ``_get_relative_embeddings`` :233-245, ``_relative_position_to_absolute_position`` :247-266,
  ``_absolute_position_to_relative_position`` :268-283)
* ``transformer.py:319-341``  FeedForwardNetwork (same padding), ``:415-432`` the layer loop
* ``TTS/tts/layers/glow_tts/duration_predictor.py:47-73``  DurationPredictor
* ``TTS/tts/layers/generic/normalization.py:23-28``  LayerNorm (channel axis, eps 1e-4)
* ``TTS/tts/models/glow_tts.py:349-361``  durations, y_mask, generate_path, compute_outputs
  (:138-148), z; ``TTS/tts/utils/helpers.py:43-57`` sequence_mask, ``:154-169`` generate_path
* the other encoder types (encoder.py:112-127): ``generic/gated_conv.py:27-36`` (conv on o * mask,
  LayerNorm, GLU, residual), ``generic/res_conv_bn.py:39-44, :80-83, :119-127`` (unpadded conv,
  zero pad (d(k-1)//2, rest), relu, BatchNorm; residual + mask per block; postnet conv1x1 ->
  BatchNorm, * mask), ``generic/time_depth_sep_conv.py:44-56, :82-84`` (x * mask, conv1x1, BN,
  GLU, depthwise conv, BN, swish, conv1x1, BN, residual)

The relative-position terms are computed here directly from their definition (key j of query i
uses embedding j - i + W when |j - i| <= W) instead of the reference's pad/reshape skew; the
golden fixtures pin the two against each other (tests/test_oracle_golden.py).
Pinned against golden vectors of the reference modules (tests/golden/make_goldens.py glow_tts).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F


def sequence_mask(lengths: torch.Tensor, max_len: Optional[int] = None) -> torch.Tensor:
    if max_len is None:
        max_len = int(lengths.max())
    return torch.arange(max_len, dtype=lengths.dtype)[None, :] < lengths[:, None]


def layer_norm(x, gamma, beta, eps=1e-4):
    mean = torch.mean(x, 1, keepdim=True)
    var = torch.mean((x - mean) ** 2, 1, keepdim=True)
    return (x - mean) * torch.rsqrt(var + eps) * gamma + beta


def rel_attention(q, k, v, mask, num_heads, emb_rel_k=None, emb_rel_v=None, input_length=None):
    """q, k, v [B, C, T], mask [B, 1, T] -> [B, C, T] (transformer.py:142-180); input_length: the
    block mask of :148-150 (scores outside |i - j| <= input_length are -1e4)."""
    b, c, t = q.shape
    dk = c // num_heads
    qh = q.view(b, num_heads, dk, t).transpose(2, 3)
    kh = k.view(b, num_heads, dk, t).transpose(2, 3)
    vh = v.view(b, num_heads, dk, t).transpose(2, 3)
    scores = torch.matmul(qh, kh.transpose(-2, -1)) / math.sqrt(dk)
    if emb_rel_k is not None:
        W = (emb_rel_k.size(1) - 1) // 2
        rel = torch.matmul(qh, emb_rel_k[0].t())  # [b, h, t, 2W+1]
        i = torch.arange(t)[:, None]
        j = torch.arange(t)[None, :]
        r = j - i + W
        ok = (r >= 0) & (r <= 2 * W)
        loc = torch.gather(rel, 3, r.clamp(0, 2 * W).expand(b, num_heads, t, t)) * ok
        scores = scores + loc / math.sqrt(dk)
    am = mask.unsqueeze(2) * mask.unsqueeze(-1)  # transformer.py:419
    scores = scores.masked_fill(am == 0, -1e4)
    if input_length is not None:
        band = (torch.arange(t)[None, :] - torch.arange(t)[:, None]).abs() <= input_length
        scores = scores.masked_fill(~band, -1e4)
    p = F.softmax(scores, dim=-1)
    out = torch.matmul(p, vh)
    if emb_rel_v is not None:
        W = (emb_rel_v.size(1) - 1) // 2
        i = torch.arange(t)[:, None]
        j = torch.arange(t)[None, :]
        r = j - i + W
        ok = ((r >= 0) & (r <= 2 * W)).to(p.dtype)
        # relative weights pr[i, r] = p[i, i + r - W]
        pr = torch.zeros(b, num_heads, t, 2 * W + 1, dtype=p.dtype)
        pr.scatter_add_(3, r.clamp(0, 2 * W).expand(b, num_heads, t, t), p * ok)
        out = out + torch.matmul(pr, emb_rel_v[0])
    return out.transpose(2, 3).contiguous().view(b, c, t)


def rel_transformer(w, x, x_mask, ep, prefix="encoder"):
    """RelativePositionTransformer.forward (transformer.py:410-432) with in = out = hidden: per layer
    x = LN1(x*mask + attn(x*mask)); x = LN2(x + FFN(x, mask)); LayerNorm2 (layer_norm_type "2",
    normalization.py:42-53) is F.layer_norm over channels with eps 1e-5, LayerNorm ("1") eps 1e-4."""
    K = ep.get("kernel_size", 1)
    pl, pr = (K - 1) // 2, K // 2
    eps_tf = 1e-5 if ep.get("layer_norm_type", "1") == "2" else 1e-4
    for i in range(ep["num_layers"]):  # transformer.py:420-431
        pre = f"{prefix}.attn_layers.{i}"
        x = x * x_mask
        q = F.conv1d(x, w[f"{pre}.conv_q.weight"], w[f"{pre}.conv_q.bias"])
        k = F.conv1d(x, w[f"{pre}.conv_k.weight"], w[f"{pre}.conv_k.bias"])
        v = F.conv1d(x, w[f"{pre}.conv_v.weight"], w[f"{pre}.conv_v.bias"])
        a = rel_attention(q, k, v, x_mask, ep["num_heads"], w.get(f"{pre}.emb_rel_k"), w.get(f"{pre}.emb_rel_v"),
                          ep.get("input_length"))
        y = F.conv1d(a, w[f"{pre}.conv_o.weight"], w[f"{pre}.conv_o.bias"])
        x = layer_norm(x + y, w[f"{prefix}.norm_layers_1.{i}.gamma"].reshape(1, -1, 1),
                       w[f"{prefix}.norm_layers_1.{i}.beta"].reshape(1, -1, 1), eps_tf)
        f = f"{prefix}.ffn_layers.{i}"
        y = F.conv1d(F.pad(x * x_mask, [pl, pr]), w[f"{f}.conv_1.weight"], w[f"{f}.conv_1.bias"])
        y = torch.relu(y)
        y = F.conv1d(F.pad(y * x_mask, [pl, pr]), w[f"{f}.conv_2.weight"], w[f"{f}.conv_2.bias"]) * x_mask
        x = layer_norm(x + y, w[f"{prefix}.norm_layers_2.{i}.gamma"].reshape(1, -1, 1),
                       w[f"{prefix}.norm_layers_2.{i}.beta"].reshape(1, -1, 1), eps_tf)
    return x


def _bn(x, w, pre, eps=1e-5):
    """nn.BatchNorm1d in eval mode (running statistics)."""
    return F.batch_norm(x, w[f"{pre}.running_mean"], w[f"{pre}.running_var"], w[f"{pre}.weight"], w[f"{pre}.bias"],
                        False, 0.0, eps)


def encoder_forward(sd: Dict[str, torch.Tensor], tokens: torch.Tensor, lengths: torch.Tensor,
                    hidden_channels: int = 192, encoder_params: Optional[dict] = None, mean_only: bool = True,
                    use_prenet: bool = True, dtype=torch.float64, g: Optional[torch.Tensor] = None,
                    encoder_type: str = "rel_pos_transformer", **_unused):
    """Encoder.forward(x, x_lengths, g) -> (x_m, x_logs, logw, x_mask) (encoder.py:143-179); g [B, c_in, 1]
    is expanded over time and concatenated to the duration predictor's input (:166-168)."""
    et = encoder_type.lower()
    ep = encoder_params or {"kernel_size": 3, "num_layers": 6, "num_heads": 2, "hidden_channels_ffn": 768}
    w = {k: v.to(dtype) if v.is_floating_point() else v for k, v in sd.items()}
    H = hidden_channels
    x = F.embedding(tokens, w["emb.weight"]) * math.sqrt(H)
    x = x.transpose(1, -1)
    x_mask = sequence_mask(lengths, x.size(2)).unsqueeze(1).to(dtype)
    if et == "residual_conv_bn" and use_prenet:
        raise TypeError("Sequential.forward() takes 2 positional arguments but 3 were given")  # encoder.py:158
    if use_prenet and et in ("rel_pos_transformer", "time_depth_separable"):  # glow.py:61-67
        x_res = x
        for i in range(3):
            x = F.conv1d(x * x_mask, w[f"prenet.conv_layers.{i}.weight"], w[f"prenet.conv_layers.{i}.bias"], padding=2)
            x = layer_norm(x * x_mask, w[f"prenet.norm_layers.{i}.gamma"], w[f"prenet.norm_layers.{i}.beta"])
            x = F.relu(x)
        x = x_res + F.conv1d(x, w["prenet.proj.weight"], w["prenet.proj.bias"])
        x = x * x_mask
    K = ep.get("kernel_size", 1)
    pl, pr = (K - 1) // 2, K // 2
    if et == "gated_conv":  # gated_conv.py:27-36 (dropout: identity at inference)
        o = res = x
        for i in range(ep["num_layers"]):
            o = F.conv1d(o * x_mask, w[f"encoder.conv_layers.{i}.weight"], w[f"encoder.conv_layers.{i}.bias"],
                         padding=K // 2)
            o = layer_norm(o, w[f"encoder.norm_layers.{i}.gamma"], w[f"encoder.norm_layers.{i}.beta"])
            o = res + F.glu(o, dim=1)
            res = o
        x = o
    elif et == "residual_conv_bn":  # res_conv_bn.py:119-127, :80-83, :39-44; postnet encoder.py:161-162
        o = x * x_mask
        for i, d in enumerate(ep["dilations"]):
            res = o
            for j in range(ep.get("num_conv_blocks", 2)):
                pre = f"encoder.res_blocks.{i}.conv_bn_blocks.{j}"
                o = F.conv1d(o, w[f"{pre}.conv1d.weight"], w[f"{pre}.conv1d.bias"], dilation=d)
                ptot = d * (K - 1)
                o = F.pad(o, [ptot // 2, ptot - ptot // 2])
                o = _bn(F.relu(o), w, f"{pre}.norm")
            o = (o + res) * x_mask
        x = _bn(F.conv1d(o, w["postnet.0.weight"], w["postnet.0.bias"]), w, "postnet.1") * x_mask
    elif et == "time_depth_separable":  # time_depth_sep_conv.py:44-56, :82-84
        for i in range(ep["num_layers"]):
            pre = f"encoder.layers.{i}"
            x = x * x_mask
            h = _bn(F.conv1d(x, w[f"{pre}.time_conv.weight"], w[f"{pre}.time_conv.bias"]), w, f"{pre}.norm1")
            h = F.glu(h, dim=1)
            h = F.conv1d(h, w[f"{pre}.depth_conv.weight"], w[f"{pre}.depth_conv.bias"], padding=(K - 1) // 2,
                         groups=H)
            h = _bn(h, w, f"{pre}.norm2")
            h = h * torch.sigmoid(h)
            h = _bn(F.conv1d(h, w[f"{pre}.time_conv2.weight"], w[f"{pre}.time_conv2.bias"]), w, f"{pre}.norm3")
            x = x + h
    if et == "rel_pos_transformer":
        x = rel_transformer(w, x, x_mask, ep)
    x = x * x_mask
    x_m = F.conv1d(x, w["proj_m.weight"], w["proj_m.bias"]) * x_mask
    if mean_only:
        x_logs = torch.zeros_like(x_m)
    else:
        x_logs = F.conv1d(x, w["proj_s.weight"], w["proj_s.bias"]) * x_mask
    d = "duration_predictor"  # duration_predictor.py:63-73
    x_dp = x if g is None else torch.cat([x, g.to(dtype).expand(-1, -1, x.size(-1))], 1)
    h = F.conv1d(x_dp * x_mask, w[f"{d}.conv_1.weight"], w[f"{d}.conv_1.bias"], padding=1)
    h = layer_norm(torch.relu(h), w[f"{d}.norm_1.gamma"], w[f"{d}.norm_1.beta"])
    h = F.conv1d(h * x_mask, w[f"{d}.conv_2.weight"], w[f"{d}.conv_2.bias"], padding=1)
    h = layer_norm(torch.relu(h), w[f"{d}.norm_2.gamma"], w[f"{d}.norm_2.beta"])
    logw = F.conv1d(h * x_mask, w[f"{d}.proj.weight"], w[f"{d}.proj.bias"]) * x_mask
    return x_m, x_logs, logw, x_mask


def durations(logw: torch.Tensor, x_mask: torch.Tensor, length_scale: float = 1.0):
    """glow_tts.py:350-352 -> (w_ceil [B,1,T_x], y_lengths [B] int64)."""
    w = (torch.exp(logw) - 1) * x_mask * length_scale
    w_ceil = torch.clamp_min(torch.ceil(w), 1)
    y_lengths = torch.clamp_min(torch.sum(w_ceil, [1, 2]), 1).long()
    return w_ceil, y_lengths


def expand(w_ceil, x_mask, y_lengths, o_mean, o_log_scale, noise=None, noise_scale: float = 0.0):
    """glow_tts.py:354-361 (+ helpers.generate_path, compute_outputs) ->
    (z, y_mask, y_mean, y_log_scale, attn [B,T_x,T_y], o_attn_dur)."""
    y_mask = sequence_mask(y_lengths, None).unsqueeze(1).to(x_mask.dtype)
    attn_mask = x_mask.unsqueeze(-1) * y_mask.unsqueeze(2)  # [B,1,T_x,T_y]
    b, _, t_x, t_y = attn_mask.shape
    cum = torch.cumsum(w_ceil.squeeze(1), 1)  # generate_path (helpers.py:161-169)
    path = (torch.arange(t_y, dtype=cum.dtype)[None, None, :] < cum[:, :, None]).to(x_mask.dtype)
    path = path - F.pad(path, [0, 0, 1, 0])[:, :-1]
    attn = path * attn_mask.squeeze(1)
    y_mean = torch.matmul(attn.transpose(1, 2), o_mean.transpose(1, 2)).transpose(1, 2)
    y_log_scale = torch.matmul(attn.transpose(1, 2), o_log_scale.transpose(1, 2)).transpose(1, 2)
    o_attn_dur = torch.log(1 + torch.sum(attn.unsqueeze(1), -1)) * x_mask
    if noise is None:
        noise = torch.zeros_like(y_mean)
    z = (y_mean + torch.exp(y_log_scale) * noise.to(y_mean.dtype) * noise_scale) * y_mask
    return z, y_mask, y_mean, y_log_scale, attn, o_attn_dur
