"""Generate the golden fixtures under tests/golden/ by running the REFERENCE modules.

Run in the development container only (it imports /root/reference, which does not exist on
the GPU box):   python tests/golden/make_goldens.py        (HiFiGAN + Glow fixtures)
                python tests/golden/make_goldens.py vits   (VITS flow fixtures)
                python tests/golden/make_goldens.py glow_tts (Glow-TTS encoder + inference glue)
                python tests/golden/make_goldens.py glow_cond (speaker-conditioned Glow decoder)
                python tests/golden/make_goldens.py glow_enc_types (gated / residual-BN / TDS encoders)
                python tests/golden/make_goldens.py vits_text (Vits.inference: text encoder, SDP, glue)

Import recipe: the hot-path leaf modules need only torch/fsspec/packaging,
but ``TTS/vocoder/models/__init__.py`` and ``TTS/tts/layers/__init__.py`` import coqpit
(absent), so those two packages are pre-registered as bare namespace packages.

Weights are NOT stored: they are regenerated from the seed with tts_amd.synthetic (a
deterministic numpy stream), and each fixture records its config and seed.  Every fixture
holds the reference's fp32 CPU output and the same module run in fp64 (``.double()``), the
accuracy anchor for the tolerance gates.
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import torch
from torch.nn.functional import embedding as F_embedding

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("TTS_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(REPO, "tts-3_amd"))

from tts_amd import synthetic  # noqa: E402  (numpy/torch only; no native library needed)


def import_reference():
    sys.path.insert(0, REF)
    import TTS  # noqa: F401

    for name, sub in [
        ("TTS.tts", "TTS/tts"),
        ("TTS.tts.layers", "TTS/tts/layers"),
        ("TTS.vocoder", "TTS/vocoder"),
        ("TTS.vocoder.models", "TTS/vocoder/models"),
    ]:
        if name not in sys.modules:
            m = types.ModuleType(name)
            m.__path__ = [os.path.join(REF, sub)]
            sys.modules[name] = m
    from TTS.vocoder.models.hifigan_generator import HifiganGenerator
    from TTS.tts.layers.glow_tts.decoder import Decoder

    return HifiganGenerator, Decoder


def import_reference_vits_flow():
    import_reference()
    from TTS.tts.layers.vits.networks import ResidualCouplingBlocks

    return ResidualCouplingBlocks


def import_reference_vits_posterior():
    import_reference()
    from TTS.tts.layers.vits.networks import PosteriorEncoder

    return PosteriorEncoder


def import_reference_glow_tts():
    import_reference()
    from TTS.tts.layers.glow_tts.decoder import Decoder
    from TTS.tts.layers.glow_tts.encoder import Encoder
    from TTS.tts.utils.helpers import generate_path, sequence_mask

    return Encoder, Decoder, generate_path, sequence_mask


def _ref_encoder(Encoder, cfg, seed):
    torch.manual_seed(0)
    ref = Encoder(cfg["num_chars"], cfg["out_channels"], cfg["hidden_channels"], cfg["hidden_channels_dp"],
                  cfg.get("encoder_type", "rel_pos_transformer"), dict(cfg["encoder_params"]), dropout_p_dp=0.1,
                  mean_only=cfg["mean_only"], use_prenet=cfg["use_prenet"],
                  c_in_channels=cfg.get("c_in_channels", 0))
    sd = synthetic.glow_encoder_state_dict(**cfg, seed=seed)
    ref.load_state_dict(sd)
    ref.eval()
    return ref


def glow_encoder_case(Encoder, name, cfg, seed, B, T, lengths, tok_seed):
    ref = _ref_encoder(Encoder, cfg, seed)
    tok = synthetic.tokens(B, T, cfg["num_chars"], seed=tok_seed)
    lens = torch.tensor(lengths)
    with torch.no_grad():
        o32 = ref(tok, lens)
        o64 = ref.double()(tok, lens)
    names = ["x_m", "x_logs", "logw", "x_mask"]
    arrays = dict(tokens=tok.numpy(), lengths=lens.numpy())
    for n, a, b in zip(names, o32, o64):
        arrays[f"{n}_ref_fp32"] = a.float().numpy()
        arrays[f"{n}_ref_fp64"] = b.numpy()
    meta = dict(kind="glow_encoder", config=cfg, seed=seed, tok_seed=tok_seed, B=B, T=T, lengths=lengths)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, meta=json.dumps(meta), **arrays)
    print(f"wrote {path}: x_m std {o32[0].std():.3f} logw mean {o32[2].sum() / o32[3].sum():.3f} "
          f"max|fp32-fp64| x_m {np.abs(arrays['x_m_ref_fp32'] - arrays['x_m_ref_fp64']).max():.2e}")


def glow_tts_case(Encoder, Decoder, generate_path, sequence_mask, name, ecfg, dcfg, eseed, dseed, B, T, lengths,
                  tok_seed, noise_scale, length_scale):
    """Tokens -> Encoder -> GlowTTS.inference glue (glow_tts.py:349-363) -> Decoder reverse, fp32 and
    fp64.  GlowTTS itself imports coqpit/trainer (absent), so the glue's 12 lines are restated here
    around the reference's own generate_path / sequence_mask; the noise is drawn here and stored.
    With ``c_in_channels`` in the configs (multi-speaker), d-vectors are drawn and stored and
    g = F.normalize(d).unsqueeze(-1) as _speaker_embedding does (glow_tts.py:189-190)."""
    enc = _ref_encoder(Encoder, ecfg, eseed)
    torch.manual_seed(0)
    dec = Decoder(dcfg["in_channels"], dcfg["hidden_channels"], dcfg["kernel_size"], dcfg["dilation_rate"],
                  dcfg["num_flow_blocks"], dcfg["num_coupling_layers"], dropout_p=0.05,
                  num_splits=dcfg["num_splits"], num_squeeze=dcfg["num_squeeze"], sigmoid_scale=False,
                  c_in_channels=dcfg.get("c_in_channels", 0))
    dec.load_state_dict(synthetic.glow_decoder_state_dict(**dcfg, seed=dseed))
    dec.eval()
    dec.store_inverse()
    tok = synthetic.tokens(B, T, ecfg["num_chars"], seed=tok_seed)
    lens = torch.tensor(lengths)
    arrays = dict(tokens=tok.numpy(), lengths=lens.numpy())
    c_in = ecfg.get("c_in_channels", 0)
    assert c_in == dcfg.get("c_in_channels", 0)
    d_vectors = None
    if c_in:
        d_vectors = torch.randn(B, c_in, generator=torch.Generator().manual_seed(tok_seed + 200))
        arrays["d_vectors"] = d_vectors.numpy()

    def infer(e, d, dtype, noise):
        g = None if d_vectors is None else torch.nn.functional.normalize(d_vectors.to(dtype)).unsqueeze(-1)
        with torch.no_grad():
            o_mean, o_log_scale, o_dur_log, x_mask = e(tok, lens, g=g)
            w = (torch.exp(o_dur_log) - 1) * x_mask * length_scale
            w_ceil = torch.clamp_min(torch.ceil(w), 1)
            y_lengths = torch.clamp_min(torch.sum(w_ceil, [1, 2]), 1).long()
            y_mask = torch.unsqueeze(sequence_mask(y_lengths, None), 1).to(x_mask.dtype)
            attn_mask = torch.unsqueeze(x_mask, -1) * torch.unsqueeze(y_mask, 2)
            attn = generate_path(w_ceil.squeeze(1), attn_mask.squeeze(1)).unsqueeze(1)
            y_mean = torch.matmul(attn.squeeze(1).transpose(1, 2), o_mean.transpose(1, 2)).transpose(1, 2)
            y_log_scale = torch.matmul(attn.squeeze(1).transpose(1, 2), o_log_scale.transpose(1, 2)).transpose(1, 2)
            o_attn_dur = torch.log(1 + torch.sum(attn, -1)) * x_mask
            if noise is None:
                noise = torch.randn(y_mean.shape, generator=torch.Generator().manual_seed(tok_seed + 100))
            z = (y_mean + torch.exp(y_log_scale) * noise.to(dtype) * noise_scale) * y_mask
            y, _ = d(z, y_mask, g=g, reverse=True)
        out = dict(x_m=o_mean, logw=o_dur_log, x_mask=x_mask, w=w, w_ceil=w_ceil, y_lengths=y_lengths,
                   y_mask=y_mask, attn=attn.squeeze(1), y_mean=y_mean, o_attn_dur=o_attn_dur, z=z, mel=y)
        return out, noise

    o32, noise = infer(enc, dec, torch.float32, None)
    o64, _ = infer(enc.double(), dec.double(), torch.float64, noise)
    for k in ("w_ceil", "y_lengths"):
        assert torch.equal(o32[k].double(), o64[k].double()), f"{k}: fp32 and fp64 reference disagree"
    arrays["noise"] = noise.numpy()
    for k, v in o32.items():
        arrays[f"{k}_ref_fp32"] = v.numpy()
    for k, v in o64.items():
        arrays[f"{k}_ref_fp64"] = v.numpy()
    wv = o64["w"][o64["x_mask"] > 0]
    frac = (wv - torch.floor(wv)).numpy()
    margin = float(np.minimum(frac, 1 - frac).min())
    meta = dict(kind="glow_tts", encoder=ecfg, decoder=dcfg, eseed=eseed, dseed=dseed, tok_seed=tok_seed, B=B, T=T,
                lengths=lengths, noise_scale=noise_scale, length_scale=length_scale, ceil_margin=margin)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, meta=json.dumps(meta), **arrays)
    print(f"wrote {path}: y_lengths {o32['y_lengths'].tolist()} mel {tuple(o32['mel'].shape)} "
          f"ceil margin {margin:.2e} max|fp32-fp64| mel {np.abs(arrays['mel_ref_fp32'] - arrays['mel_ref_fp64']).max():.2e}")


def hifigan_case(HifiganGenerator, name, cfg, seed, B, T, mel_seed, stage_B=None, stage_T=None, with_forward=True):
    torch.manual_seed(0)
    ctor = {k: v for k, v in cfg.items() if k != "seed"}
    ref = HifiganGenerator(**ctor)
    sd = synthetic.hifigan_state_dict(**cfg, seed=seed, weight_norm=True)
    ref.load_state_dict(sd)
    ref.eval()
    if cfg.get("conv_pre_weight_norm", True):
        ref.remove_weight_norm()  # eval load (gan.py:249-252); VITS keeps its parametrizations
    mel = synthetic.mel(B, T, channels=cfg["in_channels"], seed=mel_seed)
    g = None
    extra = {}
    if cfg.get("cond_channels", 0) > 0:
        gen = torch.Generator().manual_seed(mel_seed + 1)
        g = torch.randn(B, cfg["cond_channels"], 1, generator=gen)
        extra["g"] = g.numpy()

    def run(model, x, gg, pad):
        with torch.no_grad():
            if pad:
                x = torch.nn.functional.pad(x, (pad, pad), "replicate")
            return model.forward(x, gg) if gg is not None else model.forward(x)

    pad = cfg.get("inference_padding", 5)
    with torch.no_grad():
        out32 = ref.inference(mel) if g is None else run(ref, mel, g, pad)
    ref64 = ref.double()
    out64 = run(ref64, mel.double(), None if g is None else g.double(), pad)
    ref.float()
    arrays = dict(mel=mel.numpy(), out_ref_fp32=out32.numpy(), out_ref_fp64=out64.numpy(), **extra)
    if with_forward:  # forward() path: no inference padding
        arrays["fwd_ref_fp64"] = run(ref64.double(), mel.double(), None if g is None else g.double(), 0).numpy()
        ref.float()
    if stage_B:
        smel = synthetic.mel(stage_B, stage_T, channels=cfg["in_channels"], seed=mel_seed + 7)
        hooks, caps = [], {}
        ref64 = ref.double()
        hooks.append(ref64.conv_pre.register_forward_hook(lambda m, i, o: caps.__setitem__("conv_pre", o)))
        for i, u in enumerate(ref64.ups):
            hooks.append(u.register_forward_hook(lambda m, inp, o, i=i: caps.__setitem__(f"ups.{i}", o)))
        with torch.no_grad():
            ref64.inference(smel.double())
        for h in hooks:
            h.remove()
        ref.float()
        arrays["stage_mel"] = smel.numpy()
        for k, v in caps.items():
            arrays["stage_" + k] = v.float().numpy()
    meta = dict(kind="hifigan", config=cfg, seed=seed, mel_seed=mel_seed, B=B, T=T, pad=pad,
                stage_B=stage_B, stage_T=stage_T)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, meta=json.dumps(meta), **arrays)
    print(f"wrote {path}: out {tuple(out32.shape)} std {out32.std():.4f} "
          f"max|fp32-fp64| {np.abs(out32.numpy() - out64.numpy()).max():.2e}")


def glow_case(Decoder, name, cfg, seed, B, T, lengths, x_seed):
    torch.manual_seed(0)
    ref = Decoder(
        in_channels=cfg["in_channels"], hidden_channels=cfg["hidden_channels"], kernel_size=cfg["kernel_size"],
        dilation_rate=cfg["dilation_rate"], num_flow_blocks=cfg["num_flow_blocks"],
        num_coupling_layers=cfg["num_coupling_layers"], dropout_p=0.05, num_splits=cfg["num_splits"],
        num_squeeze=cfg["num_squeeze"], sigmoid_scale=False, c_in_channels=cfg.get("c_in_channels", 0),
    )
    sd = synthetic.glow_decoder_state_dict(**cfg, seed=seed)
    ref.load_state_dict(sd)
    ref.eval()
    ref.store_inverse()  # glow_tts.py:519-520, :529 (eval load)
    gen = torch.Generator().manual_seed(x_seed)
    x = torch.randn(B, cfg["in_channels"], T, generator=gen)
    c_in = cfg.get("c_in_channels", 0)
    g = torch.randn(B, c_in, 1, generator=gen) if c_in else None  # speaker vector (decoder.py:113)
    lengths_t = torch.tensor(lengths)
    mask = (torch.arange(T)[None, :] < lengths_t[:, None]).float().unsqueeze(1)
    with torch.no_grad():
        y32, _ = ref(x, mask, g=g, reverse=True)
        ref64 = ref.double()
        g64 = g.double() if g is not None else None
        y64, _ = ref64(x.double(), mask.double(), g=g64, reverse=True)
        # round trip through the reference's own forward direction
        z64, logdet = ref64(y64, mask.double()[:, :, : y64.size(2)], g=g64, reverse=False)
    meta = dict(kind="glow", config=cfg, seed=seed, x_seed=x_seed, B=B, T=T, lengths=lengths)
    path = os.path.join(HERE, f"{name}.npz")
    extra = {"g": g.numpy()} if g is not None else {}
    np.savez_compressed(path, meta=json.dumps(meta), x=x.numpy(), mask=mask.numpy(), out_ref_fp32=y32.numpy(),
                        out_ref_fp64=y64.numpy(), roundtrip_fp64=z64.numpy(), logdet_fp64=logdet.numpy(), **extra)
    print(f"wrote {path}: out {tuple(y32.shape)} std {y32.std():.4f} "
          f"max|fp32-fp64| {np.abs(y32.numpy() - y64.numpy()).max():.2e}")


def vits_flow_case(ResidualCouplingBlocks, name, cfg, seed, B, T, lengths, x_seed):
    torch.manual_seed(0)
    ref = ResidualCouplingBlocks(cfg["channels"], cfg["hidden_channels"], kernel_size=cfg["kernel_size"],
                                 dilation_rate=cfg["dilation_rate"], num_layers=cfg["num_layers"],
                                 num_flows=cfg["num_flows"], cond_channels=cfg["cond_channels"])
    sd = synthetic.vits_flow_state_dict(**cfg, seed=seed)
    ref.load_state_dict(sd)
    ref.eval()
    gen = torch.Generator().manual_seed(x_seed)
    x = torch.randn(B, cfg["channels"], T, generator=gen)
    g = torch.randn(B, cfg["cond_channels"], 1, generator=gen) if cfg["cond_channels"] else None
    lengths_t = torch.tensor(lengths)
    mask = (torch.arange(T)[None, :] < lengths_t[:, None]).float().unsqueeze(1)
    with torch.no_grad():
        y32 = ref(x, mask, g=g, reverse=True)
        ref64 = ref.double()
        y64 = ref64(x.double(), mask.double(), g=g.double() if g is not None else None, reverse=True)
        z64 = ref64(y64, mask.double(), g=g.double() if g is not None else None, reverse=False)
    meta = dict(kind="vits_flow", config=cfg, seed=seed, x_seed=x_seed, B=B, T=T, lengths=lengths)
    arrays = dict(x=x.numpy(), mask=mask.numpy(), out_ref_fp32=y32.numpy(), out_ref_fp64=y64.numpy(),
                  roundtrip_fp64=z64.numpy())
    if g is not None:
        arrays["g"] = g.numpy()
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, meta=json.dumps(meta), **arrays)
    print(f"wrote {path}: out {tuple(y32.shape)} std {y32.std():.4f} "
          f"max|fp32-fp64| {np.abs(y32.numpy() - y64.numpy()).max():.2e}")


def vits_posterior_case(PosteriorEncoder, name, cfg, seed, B, T, lengths, x_seed):
    """G13: VITS PosteriorEncoder (networks.py:235-288).  The reference draws its noise with
    torch.randn_like(mean) (:287): the fp32 run draws it from a fixed seed, the same draw is stored
    as ``eps``, and the fp64 z is formed from the fp64 mean / log_scale with that eps."""
    torch.manual_seed(0)
    ref = PosteriorEncoder(cfg["in_channels"], cfg["out_channels"], cfg["hidden_channels"], cfg["kernel_size"],
                           cfg["dilation_rate"], cfg["num_layers"], cond_channels=cfg["cond_channels"])
    sd = synthetic.vits_posterior_state_dict(**cfg, seed=seed)
    ref.load_state_dict(sd)
    ref.eval()
    gen = torch.Generator().manual_seed(x_seed)
    x = torch.randn(B, cfg["in_channels"], T, generator=gen)
    g = torch.randn(B, cfg["cond_channels"], 1, generator=gen) if cfg["cond_channels"] else None
    lengths_t = torch.tensor(lengths)
    with torch.no_grad():
        torch.manual_seed(777)
        z32, m32, ls32, mask = ref(x, lengths_t, g=g)
        torch.manual_seed(777)
        eps = torch.randn(B, cfg["out_channels"], T)  # the draw randn_like(mean) made
        assert torch.equal(z32, (m32 + eps * torch.exp(ls32)) * mask)
        ref64 = ref.double()
        _, m64, ls64, mask64 = ref64(x.double(), lengths_t, g=g.double() if g is not None else None)
        z64 = (m64 + eps.double() * torch.exp(ls64)) * mask64
    meta = dict(kind="vits_posterior", config=cfg, seed=seed, x_seed=x_seed, B=B, T=T, lengths=lengths)
    arrays = dict(x=x.numpy(), lengths=np.array(lengths), eps=eps.numpy(), mask=mask.numpy(), z_ref_fp32=z32.numpy(),
                  m_ref_fp64=m64.numpy(), logs_ref_fp64=ls64.numpy(), z_ref_fp64=z64.numpy())
    if g is not None:
        arrays["g"] = g.numpy()
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, meta=json.dumps(meta), **arrays)
    print(f"wrote {path}: z {tuple(z32.shape)} std {z32.std():.4f} "
          f"max|fp32-fp64| {np.abs(z32.numpy() - z64.numpy()).max():.2e}")


def import_reference_vits_text():
    HifiganGenerator, _ = import_reference()
    from TTS.tts.layers.vits.networks import ResidualCouplingBlocks, TextEncoder
    from TTS.tts.layers.vits.stochastic_duration_predictor import StochasticDurationPredictor
    from TTS.tts.utils.helpers import generate_path, sequence_mask

    return TextEncoder, StochasticDurationPredictor, ResidualCouplingBlocks, HifiganGenerator, generate_path, sequence_mask


def import_reference_duration_predictor():
    import_reference()
    from TTS.tts.layers.glow_tts.duration_predictor import DurationPredictor

    return DurationPredictor


def vits_text_case(refs, name, tcfg, scfg, fcfg, dcfg, seeds, B, T, lengths, tok_seed, gin=0, lang=0, lids=None,
                   use_sdp=True, up_factor=None):
    """G14: Vits.inference (vits.py:1121-1162) tokens -> waveform through the reference's TextEncoder,
    StochasticDurationPredictor(reverse=True), generate_path / sequence_mask, ResidualCouplingBlocks
    and HifiganGenerator.  Vits itself imports torchaudio / librosa / coqpit (absent), so the glue's
    lines are restated here around the reference modules.  Both noise draws (the SDP's torch.randn
    at stochastic_duration_predictor.py:277 and randn_like(m_p) at vits.py:1154) are made here with
    fixed seeds and stored; the fp64 run reuses them.  gin > 0: a speaker vector g [B, gin, 1] drawn
    and stored, fed to the SDP (condition_dp_on_speaker), the flow and the decoder as vits.py does.
    lang > 0 (YourTTS, vits.py:796-801, :1119-1124): an emb_l table [3, lang] and per-utterance ids
    ``lids`` stored, lang_emb = emb_l(lid).unsqueeze(-1) into the TextEncoder (language_emb_dim) and the
    duration predictor.  use_sdp False: the reference's glow_tts DurationPredictor(H, 256, 3, 0.5,
    cond_channels=gin, language_emb_dim=lang) (vits.py:694-702, :1136-1139).  up_factor: upsampling_z
    (vits.py:944-959) with interpolate_factor = up_factor, restated around the reference's own
    sequence_mask (Vits imports torchaudio)."""
    TextEncoder, SDP, RCB, HifiganGenerator, generate_path, sequence_mask = refs
    torch.manual_seed(0)
    te = TextEncoder(tcfg["num_chars"], tcfg["out_channels"], tcfg["hidden_channels"], tcfg["hidden_channels_ffn"],
                     tcfg["num_heads"], tcfg["num_layers"], tcfg["kernel_size"], 0.1, language_emb_dim=lang or None)
    te.load_state_dict(synthetic.vits_text_encoder_state_dict(**tcfg, language_emb_dim=lang, seed=seeds[0]))
    if use_sdp:
        dp = SDP(scfg["in_channels"], scfg["hidden_channels"], scfg["kernel_size"], 0.5, scfg["num_flows"],
                 cond_channels=gin, language_emb_dim=lang)
        dp.load_state_dict(synthetic.vits_sdp_state_dict(**dict(scfg, in_channels=scfg["in_channels"] + lang),
                                                         cond_channels=gin, language_emb_dim=lang, seed=seeds[1]))
    else:
        DP = import_reference_duration_predictor()
        dp = DP(tcfg["hidden_channels"], 256, 3, 0.5, cond_channels=gin, language_emb_dim=lang)
        dp.load_state_dict(synthetic.vits_dp_state_dict(tcfg["hidden_channels"], 256, 3, cond_channels=gin,
                                                        language_emb_dim=lang, seed=seeds[1]))
    fl = RCB(fcfg["channels"], fcfg["hidden_channels"], fcfg["kernel_size"], fcfg["dilation_rate"], fcfg["num_layers"],
             num_flows=fcfg["num_flows"], cond_channels=gin)
    fl.load_state_dict(synthetic.vits_flow_state_dict(**dict(fcfg, cond_channels=gin), seed=seeds[2]))
    dec = HifiganGenerator(**{k: v for k, v in dict(dcfg, cond_channels=gin).items() if k != "num_chars"})
    dec.load_state_dict(synthetic.hifigan_state_dict(**dict(dcfg, cond_channels=gin), seed=seeds[3], weight_norm=True))
    for m in (te, dp, fl, dec):
        m.eval()
    tok = synthetic.tokens(B, T, tcfg["num_chars"], seed=tok_seed)
    lens = torch.tensor(lengths)
    gen = torch.Generator().manual_seed(tok_seed + 300)
    g = torch.randn(B, gin, 1, generator=gen) if gin else None
    noise_dp = torch.randn(B, 2, T, generator=gen)
    emb_l = torch.randn(3, lang, generator=gen) if lang else None
    lang_emb = F_embedding(torch.tensor(lids), emb_l).unsqueeze(-1) if lang else None  # emb_l(lid).unsqueeze(-1)
    ns, ls, ns_dp = 0.667, 1.0, 1.0  # VitsArgs inference_noise_scale, length_scale, inference_noise_scale_dp

    def infer(dtype, noise_z):
        mods = [m.to(dtype) for m in (te, dp, fl, dec)]
        gg = g.to(dtype) if g is not None else None
        le = lang_emb.to(dtype) if lang_emb is not None else None
        with torch.no_grad():
            x, m_p, logs_p, x_mask = mods[0](tok, lens, lang_emb=le)
            if use_sdp:
                # the SDP's own draw replaced by the stored one (torch.randn(x.size(0), 2, x.size(2)))
                orig = torch.randn
                torch.randn = lambda *a, **k: noise_dp.clone()
                try:
                    logw = mods[1](x, x_mask, g=gg, reverse=True, noise_scale=ns_dp, lang_emb=le)
                finally:
                    torch.randn = orig
            else:
                logw = mods[1](x, x_mask, g=gg, lang_emb=le)
            w = torch.exp(logw) * x_mask * ls
            w_ceil = torch.ceil(w)
            y_lengths = torch.clamp_min(torch.sum(w_ceil, [1, 2]), 1).long()
            y_mask = sequence_mask(y_lengths, None).to(x_mask.dtype).unsqueeze(1)
            attn_mask = x_mask * y_mask.transpose(1, 2)
            attn = generate_path(w_ceil.squeeze(1), attn_mask.squeeze(1).transpose(1, 2))
            mp = torch.matmul(attn.transpose(1, 2), m_p.transpose(1, 2)).transpose(1, 2)
            lp = torch.matmul(attn.transpose(1, 2), logs_p.transpose(1, 2)).transpose(1, 2)
            if noise_z is None:
                noise_z = torch.randn(mp.shape, generator=torch.Generator().manual_seed(tok_seed + 301))
            z_p = mp + noise_z.to(dtype) * torch.exp(lp) * ns
            z = mods[2](z_p, y_mask, g=gg, reverse=True)
            if up_factor:  # upsampling_z (vits.py:951-957)
                z = torch.nn.functional.interpolate(z, scale_factor=[up_factor], mode="linear").squeeze(0)
                y_mask = sequence_mask(y_lengths * up_factor, None).to(y_mask.dtype).unsqueeze(1)
            wav = mods[3](z * y_mask, g=gg)
        out = dict(x=x, m_p=m_p, logs_p=logs_p, x_mask=x_mask, logw=logw, w=w, w_ceil=w_ceil, y_lengths=y_lengths,
                   y_mask=y_mask, attn=attn, m_p_exp=mp, logs_p_exp=lp, z_p=z_p, z=z, wav=wav)
        return out, noise_z

    o32, noise_z = infer(torch.float32, None)
    o64, _ = infer(torch.float64, noise_z)
    for k in ("w_ceil", "y_lengths"):
        assert torch.equal(o32[k].double(), o64[k].double()), f"{k}: fp32 and fp64 reference disagree"
    arrays = dict(tokens=tok.numpy(), lengths=lens.numpy(), noise_dp=noise_dp.numpy(), noise_z=noise_z.numpy())
    if g is not None:
        arrays["g"] = g.numpy()
    if lang:
        arrays["emb_l"] = emb_l.numpy()
        arrays["lids"] = np.asarray(lids, np.int64)
        arrays["lang_emb"] = lang_emb.numpy()
    for k, v in o32.items():
        arrays[f"{k}_ref_fp32"] = v.numpy()
    for k, v in o64.items():
        arrays[f"{k}_ref_fp64"] = v.numpy()
    wv = o64["w"][o64["x_mask"] > 0]
    frac = (wv - torch.floor(wv)).numpy()
    margin = float(np.minimum(frac, 1 - frac).min())
    meta = dict(kind="vits_text", text_encoder=tcfg, sdp=scfg, flow=fcfg, decoder=dcfg, seeds=list(seeds),
                tok_seed=tok_seed, B=B, T=T, lengths=lengths, gin=gin, noise_scale=ns, length_scale=ls,
                noise_scale_dp=ns_dp, ceil_margin=margin, lang=lang, use_sdp=use_sdp, up_factor=up_factor)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, meta=json.dumps(meta), **arrays)
    print(f"wrote {path}: y_lengths {o32['y_lengths'].tolist()} wav {tuple(o32['wav'].shape)} ceil margin "
          f"{margin:.2e} max|fp32-fp64| logw {np.abs(arrays['logw_ref_fp32'] - arrays['logw_ref_fp64']).max():.2e} "
          f"wav {np.abs(arrays['wav_ref_fp32'] - arrays['wav_ref_fp64']).max():.2e}")


def main_vits_text():
    refs = import_reference_vits_text()
    from tts_amd.config import VITS_FLOW, VITS_SDP, VITS_TEXT_ENCODER

    tcfg = dict(VITS_TEXT_ENCODER, num_chars=64)
    dcfg = dict(in_channels=192, out_channels=1, resblock_type="1",
                resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], resblock_kernel_sizes=[3, 7, 11],
                upsample_kernel_sizes=[16, 16, 4, 4], upsample_initial_channel=128, upsample_factors=[8, 8, 2, 2],
                inference_padding=0, conv_pre_weight_norm=False, conv_post_weight_norm=False, conv_post_bias=False)
    fcfg = dict(VITS_FLOW, cond_channels=0)
    vits_text_case(refs, "vits_text_b3_t13", tcfg, dict(VITS_SDP), fcfg, dcfg, (7531, 9753, 2470, 101), B=3, T=13,
                   lengths=[13, 8, 1], tok_seed=51)
    vits_text_case(refs, "vits_text_spk_b2_t11", tcfg, dict(VITS_SDP), fcfg, dcfg, (7532, 9754, 2471, 102), B=2,
                   T=11, lengths=[11, 6], tok_seed=52, gin=16)
    if len(sys.argv) > 2 and sys.argv[2] == "r6":  # round 6: the remaining VitsArgs switches
        # YourTTS language embeddings (4 channels, 3 languages) through the SDP
        vits_text_case(refs, "vits_text_lang_b3_t13", tcfg, dict(VITS_SDP), fcfg, dcfg, (7533, 9755, 2472, 103), B=3,
                       T=13, lengths=[13, 9, 4], tok_seed=53, lang=4, lids=[2, 0, 1])
        # use_sdp=False with speaker + language conditioning, and upsampling_z x2 (44.1 kHz from 22.05 kHz)
        vits_text_case(refs, "vits_text_dp_up_b2_t11", tcfg, dict(VITS_SDP), fcfg, dcfg, (7534, 4712, 2473, 104), B=2,
                       T=11, lengths=[11, 7], tok_seed=54, gin=16, lang=4, lids=[1, 2], use_sdp=False, up_factor=2.0)


def main_vits_posterior():
    PosteriorEncoder = import_reference_vits_posterior()
    from tts_amd.config import VITS_POSTERIOR

    vits_posterior_case(PosteriorEncoder, "vits_posterior_b2_t37", dict(VITS_POSTERIOR, cond_channels=0), seed=1357,
                        B=2, T=37, lengths=[37, 20], x_seed=51)
    small = dict(in_channels=40, out_channels=16, hidden_channels=32, kernel_size=5, dilation_rate=2, num_layers=3,
                 cond_channels=8)
    vits_posterior_case(PosteriorEncoder, "vits_posterior_cond_b3_t29", small, seed=1358, B=3, T=29,
                        lengths=[29, 13, 1], x_seed=52)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "vits_text":
        return main_vits_text()
    if len(sys.argv) > 1 and sys.argv[1] == "vits_posterior":
        return main_vits_posterior()
    if len(sys.argv) > 1 and sys.argv[1] == "vits":
        return main_vits()
    if len(sys.argv) > 1 and sys.argv[1] == "glow_tts":
        return main_glow_tts()
    if len(sys.argv) > 1 and sys.argv[1] == "handoff":
        main_handoff_range()
        return main_handoff()
    if len(sys.argv) > 1 and sys.argv[1] == "xtts":
        return main_xtts()
    if len(sys.argv) > 1 and sys.argv[1] == "glow_enc_types":
        return main_glow_enc_types()
    if len(sys.argv) > 1 and sys.argv[1] == "glow_tts_spk":
        return main_glow_tts_spk()
    if len(sys.argv) > 1 and sys.argv[1] == "glow_cond":
        return main_glow_cond()
    HifiganGenerator, Decoder = import_reference()
    v1 = dict(in_channels=80, out_channels=1, resblock_type="1",
              resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], resblock_kernel_sizes=[3, 7, 11],
              upsample_kernel_sizes=[16, 16, 4, 4], upsample_initial_channel=512, upsample_factors=[8, 8, 2, 2],
              inference_padding=5)
    # G1: HiFiGAN-v1 (the benchmark architecture), full output + per-stage intermediates
    hifigan_case(HifiganGenerator, "hifigan_v1_b2_t32", v1, seed=1234, B=2, T=32, mel_seed=0,
                 stage_B=1, stage_T=4)
    # G1b: single frame (smallest input the reference accepts with inference padding)
    hifigan_case(HifiganGenerator, "hifigan_v1_b1_t1", v1, seed=1234, B=1, T=1, mel_seed=3, with_forward=False)
    # G2: HiFiGAN-v3 topology (ResBlock2, dilations up to 12, x4 upsample) at reduced width
    v3s = dict(in_channels=80, out_channels=1, resblock_type="2",
               resblock_dilation_sizes=[[1, 2], [2, 6], [3, 12]], resblock_kernel_sizes=[3, 5, 7],
               upsample_kernel_sizes=[16, 16, 8], upsample_initial_channel=128, upsample_factors=[8, 8, 4],
               inference_padding=5)
    hifigan_case(HifiganGenerator, "hifigan_small_rb2_b2_t16", v3s, seed=77, B=2, T=16, mel_seed=5)
    # G4: VITS-style decoder (vits.py:704-718): in 192, cond, no conv_post bias, no padding, no WN
    vits = dict(in_channels=192, out_channels=1, resblock_type="1",
                resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], resblock_kernel_sizes=[3, 7, 11],
                upsample_kernel_sizes=[16, 16, 4, 4], upsample_initial_channel=128, upsample_factors=[8, 8, 2, 2],
                inference_padding=0, cond_channels=16, conv_pre_weight_norm=False, conv_post_weight_norm=False,
                conv_post_bias=False)
    hifigan_case(HifiganGenerator, "hifigan_vits_cond_b2_t12", vits, seed=99, B=2, T=12, mel_seed=11,
                 with_forward=False)
    # G3: Glow-TTS decoder reverse, LJSpeech config, ragged mask with an odd length
    glow = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=12,
                num_coupling_layers=4, num_splits=4, num_squeeze=2)
    glow_case(Decoder, "glow_decoder_b2_t64", glow, seed=4321, B=2, T=64, lengths=[64, 41], x_seed=21)
    glow_case(Decoder, "glow_decoder_b3_t33", glow, seed=4322, B=3, T=33, lengths=[33, 20, 1], x_seed=22)


def main_glow_cond():
    _, Decoder = import_reference()
    # G3b: multi-speaker Glow-TTS decoder (c_in_channels > 0: every WN's cond_layer, wavenet.py:64-66,
    # :98-107), ragged mask with an odd length
    glow = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=12,
                num_coupling_layers=4, num_splits=4, num_squeeze=2, c_in_channels=24)
    glow_case(Decoder, "glow_decoder_cond_b3_t37", glow, seed=4323, B=3, T=37, lengths=[37, 22, 5], x_seed=23)


def main_vits():
    ResidualCouplingBlocks = import_reference_vits_flow()
    # G5: VITS reverse flow (vits.py:675-682 defaults), ragged mask; and with a speaker embedding
    flow = dict(channels=192, hidden_channels=192, kernel_size=5, dilation_rate=1, num_layers=4, num_flows=4,
                cond_channels=0)
    vits_flow_case(ResidualCouplingBlocks, "vits_flow_b2_t40", flow, seed=2468, B=2, T=40, lengths=[40, 27], x_seed=31)
    vits_flow_case(ResidualCouplingBlocks, "vits_flow_cond_b3_t17", dict(flow, cond_channels=8), seed=2469, B=3,
                   T=17, lengths=[17, 9, 1], x_seed=32)


def main_glow_tts():
    Encoder, Decoder, generate_path, sequence_mask = import_reference_glow_tts()
    from tts_amd.config import GLOW_TTS_ENCODER

    # G6: LJSpeech Glow-TTS (glow_tts_config.py defaults), tokens -> mel through encoder, glue and decoder
    ecfg = dict(GLOW_TTS_ENCODER, num_chars=64)
    dcfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=12,
                num_coupling_layers=4, num_splits=4, num_squeeze=2)
    glow_tts_case(Encoder, Decoder, generate_path, sequence_mask, "glow_tts_b3_t23", ecfg, dcfg, eseed=8642,
                  dseed=4321, B=3, T=23, lengths=[23, 17, 1], tok_seed=41, noise_scale=0.33, length_scale=1.0)
    # G7: encoder variant: relative attention window 4 (VITS text encoder style), proj_s, no prenet
    rcfg = dict(num_chars=40, out_channels=24, hidden_channels=96, hidden_channels_dp=64,
                encoder_params={"kernel_size": 3, "dropout_p": 0.1, "num_layers": 2, "num_heads": 2,
                                "hidden_channels_ffn": 192, "rel_attn_window_size": 4},
                mean_only=False, use_prenet=False)
    glow_encoder_case(Encoder, "glow_encoder_rel_b2_t19", rcfg, seed=97, B=2, T=19, lengths=[19, 11], tok_seed=43)


def main_glow_enc_types():
    """G13: the other Glow-TTS encoder types (encoder.py:112-127) with random BatchNorm statistics:
    gated_conv (3 layers, k5), residual_conv_bn (k4 -- an even kernel -- dilations 1,2,4,1,2, no
    prenet: the reference's prenet call raises), time_depth_separable (3 layers, k5, prenet)."""
    Encoder, _, _, _ = import_reference_glow_tts()
    base = dict(num_chars=30, out_channels=16, hidden_channels=64, hidden_channels_dp=48)
    cases = [
        ("glow_encoder_gated_b3_t37", dict(base, encoder_type="gated_conv", mean_only=False, use_prenet=True,
                                           encoder_params={"kernel_size": 5, "dropout_p": 0.1, "num_layers": 3})),
        ("glow_encoder_rescbn_b3_t37", dict(base, encoder_type="residual_conv_bn", mean_only=False, use_prenet=False,
                                            encoder_params={"kernel_size": 4, "dilations": [1, 2, 4, 1, 2],
                                                            "num_conv_blocks": 2, "num_res_blocks": 5})),
        ("glow_encoder_tds_b3_t37", dict(base, encoder_type="time_depth_separable", mean_only=True, use_prenet=True,
                                         encoder_params={"kernel_size": 5, "num_layers": 3})),
    ]
    for i, (name, cfg) in enumerate(cases):
        glow_encoder_case(Encoder, name, cfg, seed=301 + i, B=3, T=37, lengths=[37, 29, 13], tok_seed=51 + i)
    # rel_pos_transformer with LayerNorm2 (layer_norm_type "2") and block-limited attention
    # (input_length 3, transformer.py:148-150) beside relative embeddings (window 4)
    lcfg = dict(base, encoder_type="rel_pos_transformer", mean_only=False, use_prenet=True,
                encoder_params={"kernel_size": 3, "dropout_p": 0.1, "num_layers": 2, "num_heads": 2,
                                "hidden_channels_ffn": 128, "rel_attn_window_size": 4, "input_length": 3,
                                "layer_norm_type": "2"})
    glow_encoder_case(Encoder, "glow_encoder_ln2_band_b3_t37", lcfg, seed=311, B=3, T=37, lengths=[37, 29, 13],
                      tok_seed=61)


def main_glow_tts_spk():
    """G12: multi-speaker Glow-TTS (use_d_vector_file, d_vector_dim 72): g conditions the duration
    predictor's input (encoder.py:166-168) and every flow's WN cond_layer (glow.py:143-150)."""
    Encoder, Decoder, generate_path, sequence_mask = import_reference_glow_tts()
    from tts_amd.config import GLOW_TTS_ENCODER

    dcfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=12,
                num_coupling_layers=4, num_splits=4, num_squeeze=2)
    ecfg_s = dict(GLOW_TTS_ENCODER, num_chars=64, c_in_channels=72)
    dcfg_s = dict(dcfg, c_in_channels=72)
    glow_tts_case(Encoder, Decoder, generate_path, sequence_mask, "glow_tts_spk_b2_t19", ecfg_s, dcfg_s, eseed=2468,
                  dseed=1357, B=2, T=19, lengths=[19, 12], tok_seed=47, noise_scale=0.33, length_scale=1.0)


def main_xtts():
    """G9: the XTTS waveform decoder (TTS/tts/layers/xtts/hifigan_decoder.py HifiDecoder.forward :688-700
    around its HifiganGenerator with cond_in_each_up_layer).  That module imports torchaudio (absent),
    so the reference's vocoder HifiganGenerator (identical except for the per-layer conditioning) runs
    the network, and forward hooks on ups[i] add conds[i](g) exactly where the XTTS forward does
    (:276-279); the two latent interpolations are the reference's F.interpolate calls."""
    HifiganGenerator, _ = import_reference()
    cfg = dict(in_channels=1024, out_channels=1, resblock_type="1",
               resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], resblock_kernel_sizes=[3, 7, 11],
               upsample_kernel_sizes=[16, 16, 4, 4], upsample_initial_channel=512, upsample_factors=[8, 8, 2, 2],
               inference_padding=0, cond_channels=512, conv_pre_weight_norm=False, conv_post_weight_norm=False,
               conv_post_bias=False, cond_in_each_up_layer=True)
    seed, B, T = 321, 2, 6
    torch.manual_seed(0)
    ref = HifiganGenerator(**{k: v for k, v in cfg.items() if k != "cond_in_each_up_layer"})
    sd = synthetic.hifigan_state_dict(**cfg, seed=seed, weight_norm=True)
    conds = {k: v for k, v in sd.items() if k.startswith("conds.")}
    ref.load_state_dict({k: v for k, v in sd.items() if not k.startswith("conds.")})
    ref.eval()
    gen = torch.Generator().manual_seed(17)
    latents = torch.randn(B, T, 1024, generator=gen)  # GPT latents [B, T, C]
    g = torch.randn(B, 512, 1, generator=gen) * 0.5

    def run(model, dtype):
        gg = g.to(dtype)
        hooks = [u.register_forward_hook(
            lambda m, inp, o, i=i: o + torch.nn.functional.conv1d(gg, conds[f"conds.{i}.weight"].to(dtype),
                                                                  conds[f"conds.{i}.bias"].to(dtype)))
            for i, u in enumerate(model.ups)]
        with torch.no_grad():
            z = torch.nn.functional.interpolate(latents.to(dtype).transpose(1, 2), scale_factor=[1024 / 256],
                                                mode="linear").squeeze(1)
            z = torch.nn.functional.interpolate(z, scale_factor=[24000 / 22050], mode="linear").squeeze(0)
            out = model.forward(z, gg)
        for h in hooks:
            h.remove()
        return z, out

    z32, o32 = run(ref, torch.float32)
    z64, o64 = run(ref.double(), torch.float64)
    meta = dict(kind="xtts_decoder", config=cfg, seed=seed, B=B, T=T, input_sample_rate=22050,
                output_sample_rate=24000, output_hop_length=256, ar_mel_length_compression=1024)
    path = os.path.join(HERE, "xtts_decoder_b2_t6.npz")
    np.savez_compressed(path, meta=json.dumps(meta), latents=latents.numpy(), g=g.numpy(), z_ref_fp32=z32.numpy(),
                        z_ref_fp64=z64.numpy(), out_ref_fp32=o32.numpy(), out_ref_fp64=o64.numpy())
    print(f"wrote {path}: z {tuple(z32.shape)} out {tuple(o32.shape)} std {o32.std():.4f} "
          f"max|fp32-fp64| {np.abs(o32.numpy() - o64.numpy()).max():.2e}")


def reference_functions(path, names, extra_globals):
    """The named top-level functions / methods of a reference source file, compiled from that file.

    processor.py and numpy_transforms.py import librosa / soundfile at module level (absent here),
    so the modules cannot be imported; their normalize / denormalize / save_wav bodies need only
    numpy and scipy, so those function definitions are taken from the reference file with ast and
    executed as they are (nothing of their text is copied into this repository)."""
    import ast

    tree = ast.parse(open(path).read())
    out = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name in names and node.name not in out:
            mod = ast.Module(body=[node], type_ignores=[])
            ns = dict(extra_globals)
            exec(compile(mod, path, "exec"), ns)  # noqa: S102  (reference code, goldens only)
            out[node.name] = ns[node.name]
    return out


def main_handoff_range():
    """G10: AudioProcessor.normalize / denormalize (range normalisation, processor.py:259-336) and
    numpy_transforms.save_wav's int16 scaling (:430-447), executed from the reference source."""
    import tempfile
    import scipy.io.wavfile
    from types import SimpleNamespace

    proc = os.path.join(REF, "TTS/utils/audio/processor.py")
    fns = reference_functions(proc, {"normalize", "denormalize"}, {"np": np})
    nt = reference_functions(os.path.join(REF, "TTS/utils/audio/numpy_transforms.py"), {"save_wav"},
                             {"np": np, "scipy": scipy, "BytesIO": None})
    configs = [
        dict(signal_norm=True, symmetric_norm=True, clip_norm=True, max_norm=4.0, min_level_db=-100, ref_level_db=20),
        dict(signal_norm=True, symmetric_norm=False, clip_norm=True, max_norm=1.0, min_level_db=-100, ref_level_db=0),
        dict(signal_norm=True, symmetric_norm=True, clip_norm=False, max_norm=4.0, min_level_db=-100, ref_level_db=20),
        dict(signal_norm=True, symmetric_norm=False, clip_norm=False, max_norm=2.5, min_level_db=-90, ref_level_db=16),
    ]
    rng = np.random.default_rng(12)
    mel = (rng.standard_normal((45, 80)) * 3).astype(np.float32)  # model_outputs[0]: [T, C]
    arrays = dict(mel=mel)
    pairs = []
    for i, a in enumerate(configs):
        for j, v in enumerate(configs):
            ap_t = SimpleNamespace(**a)
            ap_v = SimpleNamespace(**v)
            den = fns["denormalize"](ap_t, mel.T).T   # synthesizer.py:414
            voc = fns["normalize"](ap_v, den.T)       # :416
            arrays[f"out_{i}_{j}"] = np.asarray(voc)
            pairs.append([i, j])
    wavs = [np.tanh(rng.standard_normal(20011)).astype(np.float32) * s_ for s_ in (1.0, 0.3, 0.004)]
    wavs.append(np.zeros(513, np.float32))
    for k, w in enumerate(wavs):
        with tempfile.TemporaryDirectory() as d:
            fpath = os.path.join(d, "x.wav")
            nt["save_wav"](wav=w, path=fpath, sample_rate=22050)
            _, pcm = scipy.io.wavfile.read(fpath)
        arrays[f"wav_{k}"] = w
        arrays[f"pcm_{k}"] = pcm
    meta = dict(kind="handoff_range", configs=configs, pairs=pairs, n_wavs=len(wavs))
    path = os.path.join(HERE, "handoff_range_t45.npz")
    np.savez_compressed(path, meta=json.dumps(meta), **arrays)
    print(f"wrote {path}: {len(pairs)} config pairs, {len(wavs)} wavs; pcm dtype {arrays['pcm_0'].dtype}")


def main_handoff():
    """G8: mel_scaler mean-var (de)normalisation through the reference's StandardScaler
    (TTS/tts/utils/helpers.py:14-39, as AudioProcessor applies it at processor.py:277 / :318) and
    interpolate_vocoder_input's F.interpolate call (vocoder/utils/generic_utils.py:24-27)."""
    import_reference()
    from TTS.tts.utils.helpers import StandardScaler

    rng = np.random.default_rng(5)
    mel = (rng.standard_normal((37, 80)) * 2).astype(np.float32)  # model_outputs[0]: [T, C]
    mean = rng.standard_normal(80) * 3 - 5   # float64, like the stats file
    std = np.exp(rng.standard_normal(80) * 0.3) * 2
    sc = StandardScaler(mean, std)
    den = sc.inverse_transform(mel.copy())     # denormalize: mel_scaler.inverse_transform(S.T).T on [C,T]^T
    ren = sc.transform(den.copy())
    spec = torch.tensor(den.T.copy()).unsqueeze(0).unsqueeze(0)
    interp = torch.nn.functional.interpolate(spec, scale_factor=[1, 24000 / 22050], recompute_scale_factor=True,
                                             mode="bilinear", align_corners=False).squeeze(0)[0].numpy()
    meta = dict(kind="handoff", sr_tts=22050, sr_voc=24000)
    path = os.path.join(HERE, "handoff_meanvar_t37.npz")
    np.savez_compressed(path, meta=json.dumps(meta), mel=mel, mean=mean, std=std, denorm_ref=den, renorm_ref=ren,
                        interp_ref=interp)
    print(f"wrote {path}: denorm {den.dtype} interp {interp.shape}")


if __name__ == "__main__":
    main()
