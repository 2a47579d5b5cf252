"""Deterministic synthetic checkpoints with the reference's state_dict keys.

There are no pretrained HiFiGAN / Glow-TTS checkpoints offline, and PyTorch's default init
makes HiFiGAN's output nearly constant (std ~0.002), which is a weak parity test.  These
generators draw variance-preserving weights from ``numpy.random.default_rng(seed)`` in a fixed
key order:

* Conv1d weight  ~ N(0,1) * s / sqrt(Cin*k), s = 0.5 on the C->C MRF convs, 1 elsewhere
* ConvTranspose1d weight ~ N(0,1) / sqrt(Cin*k/u)
* biases ~ N(0, 0.01^2)
* weight norm: v = the weight above, g = ||v|| * exp(0.1*N(0,1)) per output channel (dim 0),
  so folding g*v/||v|| is exercised with non-trivial g.

Keys match ``TTS/vocoder/models/hifigan_generator.py`` (torch.nn.utils.parametrizations
.weight_norm naming: ``<conv>.parametrizations.weight.original0`` = g,
``original1`` = v) and ``TTS/tts/layers/glow_tts/decoder.py``.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Sequence

import numpy as np
import torch

from .config import HIFIGAN_V1, GLOW_TTS_DECODER, GLOW_TTS_ENCODER, VITS_FLOW, VITS_SDP, VITS_TEXT_ENCODER


def _wn_pair(rng, v: np.ndarray):
    dims = tuple(range(1, v.ndim))
    norm = np.sqrt((v.astype(np.float64) ** 2).sum(axis=dims, keepdims=True))
    g = norm * np.exp(0.1 * rng.standard_normal(norm.shape))
    return g.astype(np.float32), v.astype(np.float32)


def hifigan_state_dict(
    in_channels: int = 80,
    out_channels: int = 1,
    resblock_type: str = "1",
    resblock_dilation_sizes: Sequence[Sequence[int]] = HIFIGAN_V1["resblock_dilation_sizes"],
    resblock_kernel_sizes: Sequence[int] = HIFIGAN_V1["resblock_kernel_sizes"],
    upsample_kernel_sizes: Sequence[int] = HIFIGAN_V1["upsample_kernel_sizes"],
    upsample_initial_channel: int = HIFIGAN_V1["upsample_initial_channel"],
    upsample_factors: Sequence[int] = HIFIGAN_V1["upsample_factors"],
    cond_channels: int = 0,
    conv_pre_weight_norm: bool = True,
    conv_post_weight_norm: bool = True,
    conv_post_bias: bool = True,
    seed: int = 1234,
    weight_norm: bool = True,
    cond_in_each_up_layer: bool = False,
    **_unused,
) -> "OrderedDict[str, torch.Tensor]":
    """State dict of a HifiganGenerator (hifigan_generator.py:163-234) with synthetic weights
    (``cond_in_each_up_layer``: the XTTS generator's ``conds.i``, xtts/hifigan_decoder.py:240-244).

    ``weight_norm=True`` gives the training-time parametrized keys; ``False`` gives the keys
    after ``remove_weight_norm`` (plain ``.weight``).
    """
    rng = np.random.default_rng(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    C0 = upsample_initial_channel

    def conv(name: str, cout: int, cin: int, k: int, scale: float, wn: bool, bias: bool = True,
             fan: float = None):
        fan = cin * k if fan is None else fan
        w = rng.standard_normal((cout, cin, k)) * (scale / np.sqrt(fan))
        b = rng.standard_normal((cout,)) * 0.01 if bias else None
        if b is not None:
            sd[f"{name}.bias"] = torch.from_numpy(b.astype(np.float32))
        if wn and weight_norm:
            g, v = _wn_pair(rng, w)
            sd[f"{name}.parametrizations.weight.original0"] = torch.from_numpy(g)
            sd[f"{name}.parametrizations.weight.original1"] = torch.from_numpy(v)
        else:
            if wn:  # consume the same random stream as the parametrized variant
                g, v = _wn_pair(rng, w)
                w = (g / np.sqrt((v.astype(np.float64) ** 2).sum(axis=(1, 2), keepdims=True))) * v
            sd[f"{name}.weight"] = torch.from_numpy(np.ascontiguousarray(w, dtype=np.float32))

    def convT(name: str, cin: int, cout: int, k: int, u: int):
        w = rng.standard_normal((cin, cout, k)) / np.sqrt(cin * k / u)
        b = rng.standard_normal((cout,)) * 0.01
        sd[f"{name}.bias"] = torch.from_numpy(b.astype(np.float32))
        g, v = _wn_pair(rng, w)
        if weight_norm:
            sd[f"{name}.parametrizations.weight.original0"] = torch.from_numpy(g)
            sd[f"{name}.parametrizations.weight.original1"] = torch.from_numpy(v)
        else:
            wf = (g / np.sqrt((v.astype(np.float64) ** 2).sum(axis=(1, 2), keepdims=True))) * v
            sd[f"{name}.weight"] = torch.from_numpy(wf.astype(np.float32))

    conv("conv_pre", C0, in_channels, 7, 1.0, conv_pre_weight_norm)
    for i, (u, k) in enumerate(zip(upsample_factors, upsample_kernel_sizes)):
        convT(f"ups.{i}", C0 >> i, C0 >> (i + 1), k, u)
    r = 0
    for i in range(len(upsample_factors)):
        ch = C0 >> (i + 1)
        for k, dil in zip(resblock_kernel_sizes, resblock_dilation_sizes):
            if resblock_type == "1":
                for m in range(3):
                    conv(f"resblocks.{r}.convs1.{m}", ch, ch, k, 0.5, True)
                for m in range(3):
                    conv(f"resblocks.{r}.convs2.{m}", ch, ch, k, 0.5, True)
            else:
                for m in range(2):
                    conv(f"resblocks.{r}.convs.{m}", ch, ch, k, 0.5, True)
            r += 1
    ch = C0 >> len(upsample_factors)
    conv("conv_post", out_channels, ch, 7, 1.0, conv_post_weight_norm, bias=conv_post_bias)
    if cond_channels > 0:
        w = rng.standard_normal((C0, cond_channels, 1)) / np.sqrt(cond_channels)
        sd["cond_layer.weight"] = torch.from_numpy(w.astype(np.float32))
        sd["cond_layer.bias"] = torch.from_numpy((rng.standard_normal((C0,)) * 0.01).astype(np.float32))
    if cond_in_each_up_layer:
        for i in range(len(upsample_factors)):
            ci = C0 >> (i + 1)
            w = rng.standard_normal((ci, cond_channels, 1)) * (0.3 / np.sqrt(cond_channels))
            sd[f"conds.{i}.weight"] = torch.from_numpy(w.astype(np.float32))
            sd[f"conds.{i}.bias"] = torch.from_numpy((rng.standard_normal((ci,)) * 0.01).astype(np.float32))
    # canonical module order: conv_pre, ups, resblocks, conv_post, cond_layer, conds
    return sd


def glow_decoder_state_dict(
    in_channels: int = GLOW_TTS_DECODER["in_channels"],
    hidden_channels: int = GLOW_TTS_DECODER["hidden_channels"],
    kernel_size: int = GLOW_TTS_DECODER["kernel_size"],
    dilation_rate: int = GLOW_TTS_DECODER["dilation_rate"],
    num_flow_blocks: int = GLOW_TTS_DECODER["num_flow_blocks"],
    num_coupling_layers: int = GLOW_TTS_DECODER["num_coupling_layers"],
    num_splits: int = GLOW_TTS_DECODER["num_splits"],
    num_squeeze: int = GLOW_TTS_DECODER["num_squeeze"],
    seed: int = 4321,
    c_in_channels: int = 0,
    **_unused,
) -> "OrderedDict[str, torch.Tensor]":
    """State dict of a Glow-TTS ``Decoder`` (decoder.py:68-111) with synthetic weights.

    ``end`` (zero-initialised in the reference, glow.py:194-196) and ActNorm are randomised too,
    otherwise the reverse flow is an identity map and parity says nothing.  ``c_in_channels > 0``
    adds every WN's ``cond_layer`` (wavenet.py:64-66), drawn after the flow's other weights so the
    unconditioned stream (and every existing fixture) is unchanged.
    """
    rng = np.random.default_rng(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    C2 = in_channels * num_squeeze
    H = hidden_channels
    S = num_splits

    def wn_conv(name: str, cout: int, cin: int, k: int, scale: float):
        w = rng.standard_normal((cout, cin, k)) * (scale / np.sqrt(cin * k))
        b = rng.standard_normal((cout,)) * 0.02
        sd[f"{name}.bias"] = torch.from_numpy(b.astype(np.float32))
        g, v = _wn_pair(rng, w)
        sd[f"{name}.parametrizations.weight.original0"] = torch.from_numpy(g)
        sd[f"{name}.parametrizations.weight.original1"] = torch.from_numpy(v)

    for f in range(num_flow_blocks):
        a, c, cb = 3 * f, 3 * f + 1, 3 * f + 2
        sd[f"flows.{a}.logs"] = torch.from_numpy((rng.standard_normal((1, C2, 1)) * 0.1).astype(np.float32))
        sd[f"flows.{a}.bias"] = torch.from_numpy((rng.standard_normal((1, C2, 1)) * 0.1).astype(np.float32))
        q, _ = np.linalg.qr(rng.standard_normal((S, S)))
        if np.linalg.det(q) < 0:
            q[:, 0] = -q[:, 0]
        sd[f"flows.{c}.weight"] = torch.from_numpy(np.ascontiguousarray(q, dtype=np.float32))
        wn_conv(f"flows.{cb}.start", H, C2 // 2, 1, 1.0)
        w_end = rng.standard_normal((C2, H, 1)) * (0.1 / np.sqrt(H))
        sd[f"flows.{cb}.end.weight"] = torch.from_numpy(w_end.astype(np.float32))
        sd[f"flows.{cb}.end.bias"] = torch.from_numpy((rng.standard_normal((C2,)) * 0.02).astype(np.float32))
        for l in range(num_coupling_layers):
            wn_conv(f"flows.{cb}.wn.in_layers.{l}", 2 * H, H, kernel_size, 1.0)
        for l in range(num_coupling_layers):
            rsc = 2 * H if l < num_coupling_layers - 1 else H
            wn_conv(f"flows.{cb}.wn.res_skip_layers.{l}", rsc, H, 1, 1.0)
        if c_in_channels > 0:
            wn_conv(f"flows.{cb}.wn.cond_layer", 2 * H * num_coupling_layers, c_in_channels, 1, 1.0)
    return sd


def vits_posterior_state_dict(
    in_channels: int = 513,
    out_channels: int = 192,
    hidden_channels: int = 192,
    kernel_size: int = 5,
    dilation_rate: int = 1,
    num_layers: int = 16,
    cond_channels: int = 0,
    seed: int = 1357,
    **_unused,
) -> "OrderedDict[str, torch.Tensor]":
    """State dict of a VITS ``PosteriorEncoder`` (TTS/tts/layers/vits/networks.py:235-288) with
    synthetic variance-preserving weights, in the reference's key order (pre, enc = WN with weight
    norm, proj).  proj is scaled down so that exp(log_scale) stays O(1)."""
    rng = np.random.default_rng(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    H = hidden_channels

    def conv(name: str, cout: int, cin: int, k: int, scale: float):
        w = rng.standard_normal((cout, cin, k)) * (scale / np.sqrt(cin * k))
        sd[f"{name}.weight"] = torch.from_numpy(w.astype(np.float32))
        sd[f"{name}.bias"] = torch.from_numpy((rng.standard_normal((cout,)) * 0.02).astype(np.float32))

    def wn_conv(name: str, cout: int, cin: int, k: int, scale: float):
        w = rng.standard_normal((cout, cin, k)) * (scale / np.sqrt(cin * k))
        sd[f"{name}.bias"] = torch.from_numpy((rng.standard_normal((cout,)) * 0.02).astype(np.float32))
        g, v = _wn_pair(rng, w)
        sd[f"{name}.parametrizations.weight.original0"] = torch.from_numpy(g)
        sd[f"{name}.parametrizations.weight.original1"] = torch.from_numpy(v)

    conv("pre", H, in_channels, 1, 1.0)
    for l in range(num_layers):
        wn_conv(f"enc.in_layers.{l}", 2 * H, H, kernel_size, 1.0)
    for l in range(num_layers):
        wn_conv(f"enc.res_skip_layers.{l}", 2 * H if l < num_layers - 1 else H, H, 1, 1.0)
    if cond_channels > 0:
        wn_conv("enc.cond_layer", 2 * H * num_layers, cond_channels, 1, 0.5)
    conv("proj", 2 * out_channels, H, 1, 0.3)
    return sd


def vits_flow_state_dict(
    channels: int = VITS_FLOW["channels"],
    hidden_channels: int = VITS_FLOW["hidden_channels"],
    kernel_size: int = VITS_FLOW["kernel_size"],
    dilation_rate: int = VITS_FLOW["dilation_rate"],
    num_layers: int = VITS_FLOW["num_layers"],
    num_flows: int = VITS_FLOW["num_flows"],
    cond_channels: int = 0,
    seed: int = 2468,
    **_unused,
) -> "OrderedDict[str, torch.Tensor]":
    """State dict of a VITS ``ResidualCouplingBlocks`` flow (TTS/tts/layers/vits/networks.py:169-232,
    mean-only blocks :103-166) with synthetic weights, in the reference's key order.

    ``post`` (zero-initialised in the reference, :135-136) is randomised too, otherwise every
    block is an identity map and parity says nothing.
    """
    rng = np.random.default_rng(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    half = channels // 2
    H = hidden_channels

    def conv(name: str, cout: int, cin: int, k: int, scale: float):
        w = rng.standard_normal((cout, cin, k)) * (scale / np.sqrt(cin * k))
        sd[f"{name}.weight"] = torch.from_numpy(w.astype(np.float32))
        sd[f"{name}.bias"] = torch.from_numpy((rng.standard_normal((cout,)) * 0.02).astype(np.float32))

    def wn_conv(name: str, cout: int, cin: int, k: int, scale: float):
        w = rng.standard_normal((cout, cin, k)) * (scale / np.sqrt(cin * k))
        sd[f"{name}.bias"] = torch.from_numpy((rng.standard_normal((cout,)) * 0.02).astype(np.float32))
        g, v = _wn_pair(rng, w)
        sd[f"{name}.parametrizations.weight.original0"] = torch.from_numpy(g)
        sd[f"{name}.parametrizations.weight.original1"] = torch.from_numpy(v)

    for f in range(num_flows):
        pre = f"flows.{f}"
        conv(f"{pre}.pre", H, half, 1, 1.0)
        for l in range(num_layers):
            wn_conv(f"{pre}.enc.in_layers.{l}", 2 * H, H, kernel_size, 1.0)
        for l in range(num_layers):
            rsc = 2 * H if l < num_layers - 1 else H
            wn_conv(f"{pre}.enc.res_skip_layers.{l}", rsc, H, 1, 1.0)
        if cond_channels > 0:
            wn_conv(f"{pre}.enc.cond_layer", 2 * H * num_layers, cond_channels, 1, 0.5)
        conv(f"{pre}.post", half, H, 1, 0.3)
    return sd


def glow_encoder_state_dict(
    num_chars: int = 64,
    out_channels: int = GLOW_TTS_ENCODER["out_channels"],
    hidden_channels: int = GLOW_TTS_ENCODER["hidden_channels"],
    hidden_channels_dp: int = GLOW_TTS_ENCODER["hidden_channels_dp"],
    encoder_params: Dict = None,
    mean_only: bool = GLOW_TTS_ENCODER["mean_only"],
    use_prenet: bool = GLOW_TTS_ENCODER["use_prenet"],
    c_in_channels: int = 0,
    seed: int = 8642,
    log_duration: float = 1.6,
    encoder_type: str = "rel_pos_transformer",
    **_unused,
) -> "OrderedDict[str, torch.Tensor]":
    """State dict of a Glow-TTS ``Encoder`` (TTS/tts/layers/glow_tts/encoder.py:83-152, any
    ``encoder_type``) with synthetic weights, in the reference's key order.

    * embedding ~ N(0, H^-0.5) as the reference (:102), so emb * sqrt(H) has unit variance
    * convs variance-preserving (1x1 q/k/v/o, FFN k3, duration predictor k3); the prenet's
      zero-initialised ``proj`` (glow.py:51-53) is randomised, otherwise the prenet is identity
    * LayerNorm gamma ~ 1 + 0.1 N, beta ~ 0.1 N (reference init 0.1 / 0: a weak test)
    * duration ``proj`` bias = ``log_duration`` with small weights, so exp(logw) - 1 is a few
      frames per token (a random-init predictor clamps every duration to 1)
    * BatchNorms (gated / residual / time-depth-separable encoders): weight ~ 1 + 0.1 N, bias and
      running mean ~ 0.1 N, running var ~ exp(0.2 N) (the reference's init, 1 / 0 / 0 / 1, is the
      identity)
    """
    et = encoder_type.lower()
    if encoder_params is None:
        ep = dict(GLOW_TTS_ENCODER["encoder_params"]) if et == "rel_pos_transformer" else {}
    else:
        ep = dict(encoder_params)
    rng = np.random.default_rng(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    H = hidden_channels
    K = ep.get("kernel_size", 1)

    def t(a):
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))

    def conv(name: str, cout: int, cin: int, k: int, scale: float = 1.0, bias_std: float = 0.02, groups: int = 1):
        w = rng.standard_normal((cout, cin // groups, k)) * (scale / np.sqrt(cin // groups * k))
        sd[f"{name}.weight"] = t(w)
        sd[f"{name}.bias"] = t(rng.standard_normal((cout,)) * bias_std)

    def norm(name: str, c: int):
        sd[f"{name}.gamma"] = t(1.0 + 0.1 * rng.standard_normal((1, c, 1)))
        sd[f"{name}.beta"] = t(0.1 * rng.standard_normal((1, c, 1)))

    def bnorm(name: str, c: int):  # BatchNorm1d (eval): random affine and running statistics
        sd[f"{name}.weight"] = t(1.0 + 0.1 * rng.standard_normal((c,)))
        sd[f"{name}.bias"] = t(0.1 * rng.standard_normal((c,)))
        sd[f"{name}.running_mean"] = t(0.1 * rng.standard_normal((c,)))
        sd[f"{name}.running_var"] = t(np.exp(0.2 * rng.standard_normal((c,))))
        sd[f"{name}.num_batches_tracked"] = torch.tensor(0)

    def prenet_rcln():
        for l in range(3):
            conv(f"prenet.conv_layers.{l}", H, H, 5)
        for l in range(3):
            norm(f"prenet.norm_layers.{l}", H)
        conv("prenet.proj", H, H, 1, 0.5)

    sd["emb.weight"] = t(rng.standard_normal((num_chars, H)) * H**-0.5)
    if et != "rel_pos_transformer":
        if et == "gated_conv":  # generic/gated_conv.py:21-24 (no prenet, encoder.py:112-113)
            for l in range(ep["num_layers"]):
                conv(f"encoder.conv_layers.{l}", 2 * H, H, K, 0.7)
            for l in range(ep["num_layers"]):
                norm(f"encoder.norm_layers.{l}", 2 * H)
        elif et == "residual_conv_bn":  # generic/res_conv_bn.py; encoder.py:114-120
            if use_prenet:
                conv("prenet.0", H, H, 1)
            for i in range(len(ep["dilations"])):
                for j in range(ep.get("num_conv_blocks", 2)):
                    pre = f"encoder.res_blocks.{i}.conv_bn_blocks.{j}"
                    conv(f"{pre}.conv1d", H, H, K, 0.6)
                    bnorm(f"{pre}.norm", H)
            conv("postnet.0", H, H, 1)
            bnorm("postnet.1", H)
        elif et == "time_depth_separable":  # generic/time_depth_sep_conv.py; encoder.py:121-127
            if use_prenet:
                prenet_rcln()
            for l in range(ep["num_layers"]):
                pre = f"encoder.layers.{l}"
                conv(f"{pre}.time_conv", 2 * H, H, 1)
                bnorm(f"{pre}.norm1", 2 * H)
                conv(f"{pre}.depth_conv", H, H, K, 1.0, groups=H)
                bnorm(f"{pre}.norm2", H)
                conv(f"{pre}.time_conv2", H, H, 1, 0.5)
                bnorm(f"{pre}.norm3", H)
        else:
            raise ValueError(f"unknown encoder_type {encoder_type}")
        _glow_encoder_heads(sd, conv, norm, t, H, out_channels, hidden_channels_dp, mean_only, c_in_channels,
                            log_duration)
        return sd
    F_ = ep["hidden_channels_ffn"]
    nh = ep["num_heads"]
    W = ep.get("rel_attn_window_size")

    def tnorm(name: str, c: int):  # the transformer's LayerNorm ("1", [1, C, 1]) or LayerNorm2 ("2", [C])
        norm(name, c)
        if ep.get("layer_norm_type", "1") == "2":
            for k in ("gamma", "beta"):
                sd[f"{name}.{k}"] = sd[f"{name}.{k}"].reshape(-1)
    if use_prenet:
        prenet_rcln()
    for l in range(ep["num_layers"]):
        pre = f"encoder.attn_layers.{l}"
        for n in ("q", "k", "v", "o"):
            conv(f"{pre}.conv_{n}", H, H, 1)
        if W is not None:
            kc = H // nh
            sd[f"{pre}.emb_rel_k"] = t(rng.standard_normal((1, 2 * W + 1, kc)) * kc**-0.5)
            sd[f"{pre}.emb_rel_v"] = t(rng.standard_normal((1, 2 * W + 1, kc)) * kc**-0.5)
    for l in range(ep["num_layers"]):
        tnorm(f"encoder.norm_layers_1.{l}", H)
    for l in range(ep["num_layers"]):
        conv(f"encoder.ffn_layers.{l}.conv_1", F_, H, K, 1.4)  # relu halves the variance
        conv(f"encoder.ffn_layers.{l}.conv_2", H, F_, K)
    for l in range(ep["num_layers"]):
        tnorm(f"encoder.norm_layers_2.{l}", H)
    _glow_encoder_heads(sd, conv, norm, t, H, out_channels, hidden_channels_dp, mean_only, c_in_channels,
                        log_duration)
    return sd


def _glow_encoder_heads(sd, conv, norm, t, H, out_channels, hidden_channels_dp, mean_only, c_in_channels,
                        log_duration):
    """proj_m / proj_s and the duration predictor (encoder.py:128-141), shared by every encoder type."""
    conv("proj_m", out_channels, H, 1)
    if not mean_only:
        conv("proj_s", out_channels, H, 1, 0.3)
    conv("duration_predictor.conv_1", hidden_channels_dp, H + c_in_channels, 3, 1.4)  # [x; g] (encoder.py:140)
    norm("duration_predictor.norm_1", hidden_channels_dp)
    conv("duration_predictor.conv_2", hidden_channels_dp, hidden_channels_dp, 3, 1.4)
    norm("duration_predictor.norm_2", hidden_channels_dp)
    conv("duration_predictor.proj", 1, hidden_channels_dp, 1, 0.3)
    sd["duration_predictor.proj.bias"] = t(np.full((1,), log_duration))


def vits_text_encoder_state_dict(
    num_chars: int = 64,
    out_channels: int = VITS_TEXT_ENCODER["out_channels"],
    hidden_channels: int = VITS_TEXT_ENCODER["hidden_channels"],
    hidden_channels_ffn: int = VITS_TEXT_ENCODER["hidden_channels_ffn"],
    num_heads: int = VITS_TEXT_ENCODER["num_heads"],
    num_layers: int = VITS_TEXT_ENCODER["num_layers"],
    kernel_size: int = VITS_TEXT_ENCODER["kernel_size"],
    seed: int = 7531,
    language_emb_dim: int = 0,
    **_unused,
) -> "OrderedDict[str, torch.Tensor]":
    """State dict of a VITS ``TextEncoder`` (TTS/tts/layers/vits/networks.py:29-81): the
    RelativePositionTransformer keys of ``glow_encoder_state_dict`` (LayerNorm2, window 4) under
    ``encoder.``, then ``proj`` (H -> 2 out); the log-scale rows of ``proj`` are drawn small so
    exp(logs) stays O(1).  language_emb_dim L > 0: the transformer and proj at H + L, the token
    embedding at H (networks.py:58-64)."""
    ep = dict(kernel_size=kernel_size, num_layers=num_layers, num_heads=num_heads,
              hidden_channels_ffn=hidden_channels_ffn, rel_attn_window_size=4, layer_norm_type="2")
    H = hidden_channels + language_emb_dim
    g = glow_encoder_state_dict(num_chars=num_chars, out_channels=out_channels, hidden_channels=H,
                                encoder_params=ep, mean_only=True, use_prenet=False, seed=seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict(
        (k, v) for k, v in g.items() if k == "emb.weight" or k.startswith("encoder."))
    rng = np.random.default_rng(seed + 1)
    if language_emb_dim:
        e = rng.standard_normal((num_chars, hidden_channels)) * hidden_channels**-0.5  # nn.init.normal_(0, H^-0.5)
        sd["emb.weight"] = torch.from_numpy(e.astype(np.float32))
    w = rng.standard_normal((2 * out_channels, H, 1)) / np.sqrt(H)
    w[out_channels:] *= 0.3
    sd["proj.weight"] = torch.from_numpy(w.astype(np.float32))
    sd["proj.bias"] = torch.from_numpy((rng.standard_normal(2 * out_channels) * 0.02).astype(np.float32))
    return sd


def vits_sdp_state_dict(
    in_channels: int = VITS_SDP["in_channels"],
    hidden_channels: int = VITS_SDP["hidden_channels"],
    kernel_size: int = VITS_SDP["kernel_size"],
    num_flows: int = VITS_SDP["num_flows"],
    cond_channels: int = 0,
    seed: int = 9753,
    log_duration: float = 1.6,
    language_emb_dim: int = 0,
    **_unused,
) -> "OrderedDict[str, torch.Tensor]":
    """State dict of a VITS ``StochasticDurationPredictor`` (stochastic_duration_predictor.py:
    150-227), every key including the training-only posterior side (post_*).

    * 1x1 convs variance-preserving, depthwise convs ~ N(0, 1/k), LayerNorm2 gamma ~ 1 + 0.1 N
    * the ConvFlow ``proj`` (zero-initialised by the reference, an identity spline) ~ N(0, 0.5/H)
      with widths / heights / derivatives of O(1) after the 1/sqrt(H) scaling
    * ElementwiseAffine translation ~ -log_duration + 0.2 N on channel 0 (the logw channel at the
      end of the reverse chain: logw = (z0 - t0) exp(-log_scale0)), log_scale ~ 0.1 N, so exp(logw)
      is a few frames per token
    """
    rng = np.random.default_rng(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    H = hidden_channels
    nb = 10

    def t(a):
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))

    def conv(name, cout, cin, k, scale=1.0, groups=1, bias_std=0.02):
        sd[f"{name}.weight"] = t(rng.standard_normal((cout, cin // groups, k)) * (scale / np.sqrt(cin // groups * k)))
        sd[f"{name}.bias"] = t(rng.standard_normal((cout,)) * bias_std)

    def dds(pre):
        for i in range(3):
            conv(f"{pre}.convs_sep.{i}", H, H, kernel_size, groups=H)
        for i in range(3):
            conv(f"{pre}.convs_1x1.{i}", H, H, 1)
        for n in ("norms_1", "norms_2"):
            for i in range(3):
                sd[f"{pre}.{n}.{i}.gamma"] = t(1.0 + 0.1 * rng.standard_normal(H))
                sd[f"{pre}.{n}.{i}.beta"] = t(0.1 * rng.standard_normal(H))

    def affine(name):
        tr = 0.2 * rng.standard_normal((2, 1))
        tr[0, 0] -= log_duration
        sd[f"{name}.translation"] = t(tr)
        sd[f"{name}.log_scale"] = t(0.1 * rng.standard_normal((2, 1)))

    def conv_flow(name):
        conv(f"{name}.pre", H, 1, 1)
        dds(f"{name}.convs")
        conv(f"{name}.proj", 3 * nb - 1, H, 1, scale=np.sqrt(0.5), bias_std=0.1)

    conv("pre", H, in_channels, 1)
    dds("convs")
    conv("proj", H, H, 1)
    affine("flows.0")
    for f in range(num_flows):
        conv_flow(f"flows.{f + 1}")
    conv("post_pre", H, 1, 1)
    dds("post_convs")
    conv("post_proj", H, H, 1)
    affine("post_flows.0")
    for f in range(num_flows):
        conv_flow(f"post_flows.{f + 1}")
    if cond_channels:
        conv("cond", H, cond_channels, 1)
    if language_emb_dim:  # cond_lang (:226-227)
        conv("cond_lang", H, language_emb_dim, 1)
    return sd


def vits_dp_state_dict(
    in_channels: int = 192,
    hidden_channels: int = 256,
    kernel_size: int = 3,
    cond_channels: int = 0,
    language_emb_dim: int = 0,
    seed: int = 4711,
    log_duration: float = 1.6,
    **_unused,
) -> "OrderedDict[str, torch.Tensor]":
    """State dict of the deterministic ``DurationPredictor`` VITS builds with use_sdp=False
    (TTS/tts/layers/glow_tts/duration_predictor.py:21-47; in = in_channels + language_emb_dim):
    variance-preserving convs, LayerNorm gamma ~ 1 + 0.1 N, and a proj whose bias puts exp(logw) at a
    few frames per token."""
    rng = np.random.default_rng(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    I, F, k = in_channels + language_emb_dim, hidden_channels, kernel_size

    def t(a):
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))

    def conv(name, cout, cin, kk, scale=1.0, bias_std=0.02, bias_mean=0.0):
        sd[f"{name}.weight"] = t(rng.standard_normal((cout, cin, kk)) * (scale / np.sqrt(cin * kk)))
        sd[f"{name}.bias"] = t(bias_mean + rng.standard_normal((cout,)) * bias_std)

    def norm(name):
        sd[f"{name}.gamma"] = t((1.0 + 0.1 * rng.standard_normal(F)).reshape(1, F, 1))
        sd[f"{name}.beta"] = t((0.1 * rng.standard_normal(F)).reshape(1, F, 1))

    conv("conv_1", F, I, k)
    norm("norm_1")
    conv("conv_2", F, F, k)
    norm("norm_2")
    conv("proj", 1, F, 1, scale=0.3, bias_mean=log_duration)
    if cond_channels:
        conv("cond", I, cond_channels, 1, scale=0.5)
    if language_emb_dim:
        conv("cond_lang", I, language_emb_dim, 1, scale=0.5)
    return sd


def tokens(batch: int, length: int, num_chars: int, seed: int = 0) -> torch.Tensor:
    """Synthetic token ids [B, T] uniform in [0, num_chars) (int64, CPU)."""
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, num_chars, (batch, length), generator=g)


def mel(batch: int, frames: int, channels: int = 80, seed: int = 0) -> torch.Tensor:
    """Synthetic N(0,1) mel [B, C, T] (torch generator, CPU)."""
    g = torch.Generator().manual_seed(seed)
    return torch.randn(batch, channels, frames, generator=g)
