"""The fp64 oracle chain of ``Vits.inference`` for a ``vits_text`` golden (tests/golden/make_goldens.py
vits_text): weights regenerated from the fixture's seeds, every VitsArgs switch the fixture records
(speaker vector, language embedding, SDP or deterministic duration predictor, upsampling_z).
Test infrastructure: it calls only oracle/ and tts_amd.synthetic (numpy weights)."""
from __future__ import annotations

from typing import Optional

import torch

from oracle import hifigan_ref, vits_ref, vits_text_ref
from tts_amd import synthetic


def state_dicts(meta):
    gin, L = meta["gin"], meta.get("lang", 0)
    tcfg, scfg = meta["text_encoder"], meta["sdp"]
    tsd = synthetic.vits_text_encoder_state_dict(**tcfg, language_emb_dim=L, seed=meta["seeds"][0])
    if meta.get("use_sdp", True):
        dsd = synthetic.vits_sdp_state_dict(**dict(scfg, in_channels=scfg["in_channels"] + L), cond_channels=gin,
                                            language_emb_dim=L, seed=meta["seeds"][1])
    else:
        dsd = synthetic.vits_dp_state_dict(tcfg["hidden_channels"], 256, 3, cond_channels=gin, language_emb_dim=L,
                                           seed=meta["seeds"][1])
    fsd = synthetic.vits_flow_state_dict(**dict(meta["flow"], cond_channels=gin), seed=meta["seeds"][2])
    dec = synthetic.hifigan_state_dict(**dict(meta["decoder"], cond_channels=gin), seed=meta["seeds"][3],
                                       weight_norm=True)
    return tsd, dsd, fsd, dec


def oracle_chain(meta, arr, w_ceil: Optional[torch.Tensor] = None, noise_z: Optional[torch.Tensor] = None,
                 start_from_reference: bool = False):
    """Tokens -> waveform in fp64.  ``w_ceil`` replaces the predicted durations (a bf16 device run's own);
    ``noise_z`` [B, C, >= T_y] replaces the stored draw; ``start_from_reference``: the expansion starts
    from the fixture's fp64 encoder outputs instead of the oracle's."""
    gin, L = meta["gin"], meta.get("lang", 0)
    tsd, dsd, fsd, dec = state_dicts(meta)
    tok, lens = torch.from_numpy(arr["tokens"]), torch.from_numpy(arr["lengths"])
    g = torch.from_numpy(arr["g"]).double() if gin else None
    le = torch.from_numpy(arr["lang_emb"]).double() if L else None
    out = {}
    x, m, logs, xm = vits_text_ref.text_encoder(tsd, tok, lens, dtype=torch.float64, lang_emb=le, **meta["text_encoder"])
    out.update(x=x, m_p=m, logs_p=logs, x_mask=xm)
    if meta.get("use_sdp", True):
        logw = vits_text_ref.sdp_reverse(dsd, x, xm, torch.from_numpy(arr["noise_dp"]), g=g, lang_emb=le,
                                         noise_scale=meta["noise_scale_dp"], dtype=torch.float64, **meta["sdp"])
    else:
        logw = vits_text_ref.dp_forward(dsd, x, xm, g=g, lang_emb=le, dtype=torch.float64)
    out["logw"] = logw
    wc, y_len = vits_text_ref.vits_durations(logw, xm, meta["length_scale"])
    if w_ceil is not None:
        wc = w_ceil.double()
        y_len = torch.clamp_min(torch.sum(wc, [1, 2]), 1).long()
    out.update(w_ceil=wc, y_lengths=y_len)
    if start_from_reference:
        m, logs = torch.from_numpy(arr["m_p_ref_fp64"]), torch.from_numpy(arr["logs_p_ref_fp64"])
    nz = torch.from_numpy(arr["noise_z"]) if noise_z is None else noise_z
    T_y = int(y_len.max())
    z_p, y_mask, mp, lp, attn = vits_text_ref.vits_expand(wc, xm, y_len, m, logs, nz[:, :, :T_y].double(),
                                                          meta["noise_scale"])
    out.update(z_p=z_p, y_mask=y_mask, m_p_exp=mp, logs_p_exp=lp, attn=attn)
    fcfg = dict(meta["flow"], cond_channels=gin)
    z = vits_ref.vits_flow_reverse(fsd, z_p, y_mask, g=g, dtype=torch.float64, **fcfg)
    if meta.get("up_factor"):
        z, y_mask = vits_text_ref.upsample_z(z, y_len, meta["up_factor"])
        out["y_mask_up"] = y_mask
    out["z"] = z
    dcfg = dict(meta["decoder"], cond_channels=gin)
    out["wav"] = hifigan_ref.hifigan_forward(dec, z * y_mask, pad=0, g=g, dtype=torch.float64,
                                             fold_dtype=torch.float64, **dcfg)
    return out
