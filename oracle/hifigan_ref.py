"""ORACLE — test infrastructure only.  Never imported by the product path (tts-3_amd/).

CPU restatement of the reference HiFiGAN generator forward, written against
``torch.nn.functional`` (the same ATen CPU conv kernels the reference runs), usable in fp32
(parity checker and bench.py's ``cpu_baseline`` leg) or fp64 (the accuracy anchor for the
tolerance gates).  It follows, line by line, Coqui TTS 0.22.0:

* ``TTS/vocoder/models/hifigan_generator.py:11``       LRELU_SLOPE = 0.1
* ``:14-15``    get_padding(k, d) = (k*d - d) // 2
* ``:84-99``    ResBlock1.forward: 3x [lrelu -> convs1[m] (dil d_m) -> lrelu -> convs2[m] -> + x]
* ``:150-155``  ResBlock2.forward: 2x [lrelu -> convs[m] (dil d_m) -> + x]
* ``:236-265``  forward: conv_pre [+ cond_layer(g)] -> per upsample: lrelu(0.1) -> ups[i] ->
                z_sum = sum_j resblocks[i*nk+j](o) -> o = z_sum / nk; then lrelu (default
                slope 0.01) -> conv_post -> tanh
* ``:267-282``  inference: replicate pad of inference_padding frames on both sides
* ``:284-291``  remove_weight_norm: w = g * v / ||v|| with the norm over all dims but 0
* ``TTS/tts/layers/xtts/hifigan_decoder.py:240-244, :276-279``  the XTTS generator's
  cond_in_each_up_layer: o = ups[i](o) + conds[i](g)

Pinned against golden vectors produced by the reference module itself
(tests/golden/make_goldens.py, checked by tests/test_oracle_golden.py).
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import torch
import torch.nn.functional as F

LRELU_SLOPE = 0.1


def get_padding(k: int, d: int) -> int:
    return int((k * d - d) / 2)


def fold_weight_norm(sd: Dict[str, torch.Tensor], dtype=torch.float64, fold_dtype=torch.float32) -> Dict[str, torch.Tensor]:
    """Replace ``X.parametrizations.weight.original0/1`` (g, v) by ``X.weight = g*v/||v||``.

    The fold is ``torch._weight_norm(v, g, 0)`` (what weight_norm's parametrization evaluates
    and ``remove_parametrizations`` stores) computed in ``fold_dtype``: fp32 reproduces the
    reference's eval load of an fp32 module (gan.py:249-252) bit for bit; fp64 reproduces a
    module that keeps its parametrization and is run in double (VITS, vits.py:704-718).
    """
    out: Dict[str, torch.Tensor] = {}
    for k, v in sd.items():
        if k.endswith(".parametrizations.weight.original0"):
            base = k[: -len(".parametrizations.weight.original0")]
            g = v.to(fold_dtype)
            vv = sd[base + ".parametrizations.weight.original1"].to(fold_dtype)
            out[base + ".weight"] = torch._weight_norm(vv, g, 0).to(dtype)
        elif k.endswith(".parametrizations.weight.original1"):
            continue
        else:
            out[k] = v.to(dtype)
    return out


def hifigan_forward(
    sd: Dict[str, torch.Tensor],
    x: torch.Tensor,
    resblock_type: str,
    resblock_dilation_sizes: Sequence[Sequence[int]],
    resblock_kernel_sizes: Sequence[int],
    upsample_kernel_sizes: Sequence[int],
    upsample_factors: Sequence[int],
    pad: int = 0,
    g: Optional[torch.Tensor] = None,
    dtype=torch.float64,
    fold_dtype=torch.float32,
    return_stages: bool = False,
    **_unused,
):
    """Generator forward on CPU.  ``sd`` may hold parametrized or folded weights."""
    w = fold_weight_norm(sd, dtype, fold_dtype)
    x = x.to(dtype)
    if pad:
        x = F.pad(x, (pad, pad), "replicate")  # :281
    stages = {}
    o = F.conv1d(x, w["conv_pre.weight"], w["conv_pre.bias"], padding=3)  # :249
    if "cond_layer.weight" in w:  # :250-251
        o = o + F.conv1d(g.to(dtype), w["cond_layer.weight"], w["cond_layer.bias"])
    stages["conv_pre"] = o
    nk = len(resblock_kernel_sizes)
    for i, (u, k) in enumerate(zip(upsample_factors, upsample_kernel_sizes)):
        o = F.leaky_relu(o, LRELU_SLOPE)  # :253
        o = F.conv_transpose1d(o, w[f"ups.{i}.weight"], w[f"ups.{i}.bias"], stride=u, padding=(k - u) // 2)
        if f"conds.{i}.weight" in w:  # XTTS cond_in_each_up_layer (xtts/hifigan_decoder.py:276-279)
            o = o + F.conv1d(g.to(dtype), w[f"conds.{i}.weight"], w[f"conds.{i}.bias"])
        stages[f"ups.{i}"] = o
        z_sum = None
        for j, (kk, dil) in enumerate(zip(resblock_kernel_sizes, resblock_dilation_sizes)):
            r = f"resblocks.{i * nk + j}"
            xr = o
            if resblock_type == "1":
                for m in range(3):  # :93-98
                    xt = F.leaky_relu(xr, LRELU_SLOPE)
                    xt = F.conv1d(xt, w[f"{r}.convs1.{m}.weight"], w[f"{r}.convs1.{m}.bias"],
                                  dilation=dil[m], padding=get_padding(kk, dil[m]))
                    xt = F.leaky_relu(xt, LRELU_SLOPE)
                    xt = F.conv1d(xt, w[f"{r}.convs2.{m}.weight"], w[f"{r}.convs2.{m}.bias"],
                                  dilation=1, padding=get_padding(kk, 1))
                    xr = xt + xr
            else:
                for m in range(2):  # :151-154
                    xt = F.leaky_relu(xr, LRELU_SLOPE)
                    xt = F.conv1d(xt, w[f"{r}.convs.{m}.weight"], w[f"{r}.convs.{m}.bias"],
                                  dilation=dil[m], padding=get_padding(kk, dil[m]))
                    xr = xt + xr
            z_sum = xr if z_sum is None else z_sum + xr  # :257-260
        o = z_sum / nk  # :261
        stages[f"mrf.{i}"] = o
    o = F.leaky_relu(o)  # :262 — default negative_slope 0.01
    o = F.conv1d(o, w["conv_post.weight"], w.get("conv_post.bias"), padding=3)
    o = torch.tanh(o)
    if return_stages:
        return o, stages
    return o
