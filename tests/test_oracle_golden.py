"""Pin the CPU oracle (oracle/) against golden vectors produced by the reference modules
(tests/golden/make_goldens.py).  CPU only."""
import numpy as np
import pytest
import torch

from _util import goldens, max_abs, rel_rms
from oracle import glow_ref, glow_tts_ref, hifigan_ref, vits_ref
from tts_amd import synthetic

HIFI = goldens("hifigan")
GLOW = goldens("glow")


def _fold_dtype(cfg):
    # modules that keep weight norm at inference (VITS) fold in the run dtype
    return torch.float32 if cfg.get("conv_pre_weight_norm", True) else torch.float64


@pytest.mark.parametrize("name,meta,arr", HIFI, ids=[h[0] for h in HIFI])
def test_hifigan_oracle_fp64_matches_reference(name, meta, arr):
    cfg = meta["config"]
    sd = synthetic.hifigan_state_dict(**cfg, seed=meta["seed"], weight_norm=True)
    g = torch.from_numpy(arr["g"]) if "g" in arr else None
    out = hifigan_ref.hifigan_forward(sd, torch.from_numpy(arr["mel"]), pad=meta["pad"], g=g,
                                      dtype=torch.float64, fold_dtype=_fold_dtype(cfg), **cfg)
    ref = arr["out_ref_fp64"]
    assert out.shape == ref.shape
    # same ops, same weights, fp64: agreement to the last few ulps of fp64
    assert max_abs(out.numpy(), ref) < 1e-12, max_abs(out.numpy(), ref)
    if "fwd_ref_fp64" in arr:
        fwd = hifigan_ref.hifigan_forward(sd, torch.from_numpy(arr["mel"]), pad=0, g=g, dtype=torch.float64,
                                          fold_dtype=_fold_dtype(cfg), **cfg)
        assert max_abs(fwd.numpy(), arr["fwd_ref_fp64"]) < 1e-12


@pytest.mark.parametrize("name,meta,arr", HIFI, ids=[h[0] for h in HIFI])
def test_hifigan_oracle_fp32_matches_reference_fp32(name, meta, arr):
    cfg = meta["config"]
    sd = synthetic.hifigan_state_dict(**cfg, seed=meta["seed"], weight_norm=True)
    g = torch.from_numpy(arr["g"]) if "g" in arr else None
    out = hifigan_ref.hifigan_forward(sd, torch.from_numpy(arr["mel"]), pad=meta["pad"], g=g,
                                      dtype=torch.float32, fold_dtype=torch.float32, **cfg)
    # same ATen CPU kernels in fp32: identical up to threading-dependent reduction order
    assert max_abs(out.numpy(), arr["out_ref_fp32"]) < 2e-6
    # and the reference's own fp32 error vs fp64 is what the fp32 gates are calibrated on
    assert rel_rms(arr["out_ref_fp32"], arr["out_ref_fp64"]) < 1e-5


def test_hifigan_stage_intermediates():
    name, meta, arr = [h for h in HIFI if "stage_conv_pre" in h[2]][0]
    cfg = meta["config"]
    sd = synthetic.hifigan_state_dict(**cfg, seed=meta["seed"], weight_norm=True)
    _, st = hifigan_ref.hifigan_forward(sd, torch.from_numpy(arr["stage_mel"]), pad=meta["pad"],
                                        dtype=torch.float64, return_stages=True, **cfg)
    for k in ["conv_pre"] + [f"ups.{i}" for i in range(len(cfg["upsample_factors"]))]:
        got = st[k].float().numpy()
        assert max_abs(got, arr["stage_" + k]) < 1e-6, k


@pytest.mark.parametrize("name,meta,arr", GLOW, ids=[g[0] for g in GLOW])
def test_glow_oracle_matches_reference(name, meta, arr):
    cfg = meta["config"]
    sd = synthetic.glow_decoder_state_dict(**cfg, seed=meta["seed"])
    g = torch.from_numpy(arr["g"]) if "g" in arr else None  # speaker vector (c_in_channels > 0)
    out = glow_ref.glow_decoder_reverse(sd, torch.from_numpy(arr["x"]), torch.from_numpy(arr["mask"]),
                                        dtype=torch.float64, g=g, **cfg)
    assert out.shape == arr["out_ref_fp64"].shape
    assert max_abs(out.numpy(), arr["out_ref_fp64"]) < 1e-10
    out32 = glow_ref.glow_decoder_reverse(sd, torch.from_numpy(arr["x"]), torch.from_numpy(arr["mask"]),
                                          dtype=torch.float32, g=g, **cfg)
    assert max_abs(out32.numpy(), arr["out_ref_fp32"]) < 1e-5


@pytest.mark.parametrize("name,meta,arr", GLOW, ids=[g[0] for g in GLOW])
def test_glow_reference_roundtrip_fixture(name, meta, arr):
    # the reference's forward direction inverts its reverse direction on the frames the
    # squeeze keeps: frame pair (2t, 2t+1) survives iff mask[2t+1] (decoder.py:25); W^-1 is
    # an fp32 inverse, so the round trip is exact only to ~1e-6
    T2 = arr["out_ref_fp64"].shape[2]
    m = arr["mask"][:, :, 1:T2:2].repeat(2, axis=2)
    x = arr["x"][:, :, :T2] * m
    assert max_abs(arr["roundtrip_fp64"] * m, x) < 1e-4


@pytest.mark.parametrize("name,meta,arr", GLOW, ids=[g[0] for g in GLOW])
def test_glow_forward_oracle_matches_reference(name, meta, arr):
    """The forward direction (reverse=False) against the reference's own forward pass, which the
    fixture ran on its fp64 reverse output (make_goldens.py glow_case): z and logdet."""
    cfg = meta["config"]
    sd = synthetic.glow_decoder_state_dict(**cfg, seed=meta["seed"])
    g = torch.from_numpy(arr["g"]) if "g" in arr else None
    y = torch.from_numpy(arr["out_ref_fp64"])
    m = torch.from_numpy(arr["mask"])[:, :, : y.shape[2]]
    z, logdet = glow_ref.glow_decoder_forward(sd, y, m, dtype=torch.float64, g=g, **cfg)
    assert z.shape == arr["roundtrip_fp64"].shape
    assert max_abs(z.numpy(), arr["roundtrip_fp64"]) < 1e-10
    assert np.abs(logdet.numpy() - arr["logdet_fp64"]).max() < 1e-8 * max(1.0, np.abs(arr["logdet_fp64"]).max())


VITS = goldens("vits_flow")


@pytest.mark.parametrize("name,meta,arr", VITS, ids=[g[0] for g in VITS])
def test_vits_flow_oracle_matches_reference(name, meta, arr):
    cfg = meta["config"]
    sd = synthetic.vits_flow_state_dict(**cfg, seed=meta["seed"])
    g = torch.from_numpy(arr["g"]) if "g" in arr else None
    x, m = torch.from_numpy(arr["x"]), torch.from_numpy(arr["mask"])
    out = vits_ref.vits_flow_reverse(sd, x, m, g, dtype=torch.float64, **cfg)
    assert out.shape == arr["out_ref_fp64"].shape
    assert max_abs(out.numpy(), arr["out_ref_fp64"]) < 1e-10
    out32 = vits_ref.vits_flow_reverse(sd, x, m, g, dtype=torch.float32, **cfg)
    assert max_abs(out32.numpy(), arr["out_ref_fp32"]) < 1e-5


@pytest.mark.parametrize("name,meta,arr", VITS, ids=[g[0] for g in VITS])
def test_vits_flow_reference_roundtrip_fixture(name, meta, arr):
    # the reference's forward direction inverts its reverse on the unmasked frames; masked
    # frames of x1 are zeroed by every block, so compare under the mask
    m = arr["mask"]
    assert max_abs(arr["roundtrip_fp64"] * m, arr["x"] * m) < 1e-9
    assert len(VITS) == 2


@pytest.mark.parametrize("name,meta,arr", VITS, ids=[g[0] for g in VITS])
def test_vits_flow_forward_oracle_matches_reference(name, meta, arr):
    cfg = meta["config"]
    sd = synthetic.vits_flow_state_dict(**cfg, seed=meta["seed"])
    g = torch.from_numpy(arr["g"]) if "g" in arr else None
    z = vits_ref.vits_flow_forward(sd, torch.from_numpy(arr["out_ref_fp64"]), torch.from_numpy(arr["mask"]), g,
                                   dtype=torch.float64, **cfg)
    assert max_abs(z.numpy(), arr["roundtrip_fp64"]) < 1e-10


POSTERIOR = goldens("vits_posterior")


@pytest.mark.parametrize("name,meta,arr", POSTERIOR, ids=[g[0] for g in POSTERIOR])
def test_vits_posterior_oracle_matches_reference(name, meta, arr):
    cfg = meta["config"]
    sd = synthetic.vits_posterior_state_dict(**cfg, seed=meta["seed"])
    g = torch.from_numpy(arr["g"]) if "g" in arr else None
    x, m, eps = torch.from_numpy(arr["x"]), torch.from_numpy(arr["mask"]), torch.from_numpy(arr["eps"])
    z, mean, logs = vits_ref.vits_posterior(sd, x, m, eps, g, dtype=torch.float64, **cfg)
    assert max_abs(z.numpy(), arr["z_ref_fp64"]) < 1e-10
    assert max_abs(mean.numpy(), arr["m_ref_fp64"]) < 1e-10 and max_abs(logs.numpy(), arr["logs_ref_fp64"]) < 1e-10
    z32, _, _ = vits_ref.vits_posterior(sd, x, m, eps, g, dtype=torch.float32, **cfg)
    assert max_abs(z32.numpy(), arr["z_ref_fp32"]) < 1e-5
    assert len(POSTERIOR) == 2


def test_synthetic_weights_deterministic():
    a = synthetic.hifigan_state_dict(seed=3)
    b = synthetic.hifigan_state_dict(seed=3)
    assert list(a) == list(b)
    for k in a:
        assert torch.equal(a[k], b[k])
    c = synthetic.hifigan_state_dict(seed=4)
    assert not torch.equal(a["conv_pre.bias"], c["conv_pre.bias"])


GENC = goldens("glow_encoder")
GTTS = goldens("glow_tts")


def _enc_args(cfg):
    return dict(hidden_channels=cfg["hidden_channels"], encoder_params=cfg["encoder_params"],
                mean_only=cfg["mean_only"], use_prenet=cfg["use_prenet"],
                encoder_type=cfg.get("encoder_type", "rel_pos_transformer"))


@pytest.mark.parametrize("name,meta,arr", GENC + [(n, dict(m, config=m["encoder"], seed=m["eseed"]), a)
                                                   for n, m, a in GTTS],
                         ids=[g[0] for g in GENC + GTTS])
def test_glow_encoder_oracle_matches_reference(name, meta, arr):
    cfg = meta["config"]
    sd = synthetic.glow_encoder_state_dict(**cfg, seed=meta["seed"])
    tok, lens = torch.from_numpy(arr["tokens"]), torch.from_numpy(arr["lengths"])
    g = _speaker_g(arr)
    out = glow_tts_ref.encoder_forward(sd, tok, lens, dtype=torch.float64, g=g, **_enc_args(cfg))
    for n, o in zip(["x_m", "x_logs", "logw", "x_mask"], out):
        if f"{n}_ref_fp64" in arr:
            assert max_abs(o.numpy(), arr[f"{n}_ref_fp64"]) < 1e-10, n
    out32 = glow_tts_ref.encoder_forward(sd, tok, lens, dtype=torch.float32, g=g, **_enc_args(cfg))
    assert max_abs(out32[0].numpy(), arr["x_m_ref_fp32"]) < 1e-5
    assert max_abs(out32[2].numpy(), arr["logw_ref_fp32"]) < 1e-5


def _speaker_g(arr):
    """multi-speaker fixtures store d-vectors; g = F.normalize(d).unsqueeze(-1) (glow_tts.py:189-190)"""
    if "d_vectors" not in arr:
        return None
    return torch.nn.functional.normalize(torch.from_numpy(arr["d_vectors"]).double()).unsqueeze(-1)


@pytest.mark.parametrize("name,meta,arr", GTTS, ids=[g[0] for g in GTTS])
def test_glow_tts_glue_oracle_matches_reference(name, meta, arr):
    # durations -> path -> y_mean -> z from the reference's own fp64 encoder outputs
    logw = torch.from_numpy(arr["logw_ref_fp64"])
    xm = torch.from_numpy(arr["x_mask_ref_fp64"])
    w_ceil, y_len = glow_tts_ref.durations(logw, xm, meta["length_scale"])
    assert torch.equal(w_ceil, torch.from_numpy(arr["w_ceil_ref_fp64"]))
    assert torch.equal(y_len, torch.from_numpy(arr["y_lengths_ref_fp64"]))
    o_mean = torch.from_numpy(arr["x_m_ref_fp64"])
    z, y_mask, y_mean, _, attn, dur = glow_tts_ref.expand(w_ceil, xm, y_len, o_mean, torch.zeros_like(o_mean),
                                                          torch.from_numpy(arr["noise"]), meta["noise_scale"])
    assert torch.equal(attn, torch.from_numpy(arr["attn_ref_fp64"]))
    assert torch.equal(y_mask, torch.from_numpy(arr["y_mask_ref_fp64"]))
    assert max_abs(y_mean.numpy(), arr["y_mean_ref_fp64"]) == 0.0
    assert max_abs(dur.numpy(), arr["o_attn_dur_ref_fp64"]) < 1e-14
    assert max_abs(z.numpy(), arr["z_ref_fp64"]) < 1e-14
    # then the decoder oracle closes the chain to the reference's mel
    dcfg = meta["decoder"]
    dsd = synthetic.glow_decoder_state_dict(**dcfg, seed=meta["dseed"])
    mel = glow_ref.glow_decoder_reverse(dsd, z, y_mask, dtype=torch.float64, g=_speaker_g(arr), **dcfg)
    assert max_abs(mel.numpy(), arr["mel_ref_fp64"]) < 1e-10
    # ceil() margin: no duration of the fixture sits within 1e-3 of an integer, so an fp32
    # implementation that matches the encoder to ~1e-6 must reproduce w_ceil exactly
    assert meta["ceil_margin"] > 1e-3


HANDOFF = goldens("handoff")


@pytest.mark.parametrize("name,meta,arr", HANDOFF, ids=[g[0] for g in HANDOFF])
def test_handoff_oracle_matches_reference(name, meta, arr):
    from oracle import handoff_ref

    a = dict(signal_norm=True, symmetric_norm=True, clip_norm=True, max_norm=4.0, min_level_db=-100, ref_level_db=20,
             mel_mean=arr["mean"], mel_std=arr["std"])
    den = handoff_ref.denormalize(arr["mel"].T, a).T
    assert den.dtype == np.float32 and np.array_equal(den, arr["denorm_ref"])
    ren = handoff_ref.normalize(den.T, a).T
    assert np.array_equal(ren, arr["renorm_ref"])
    # the resampled hand-off of interpolate_vocoder_input
    out = handoff_ref.handoff(arr["mel"], dict(a, sample_rate=meta["sr_tts"]), dict(a, signal_norm=False,
                                                                                   sample_rate=meta["sr_voc"]))
    assert np.array_equal(out, arr["interp_ref"])


XTTS = goldens("xtts_decoder")


@pytest.mark.parametrize("name,meta,arr", XTTS, ids=[g[0] for g in XTTS])
def test_xtts_decoder_oracle_matches_reference(name, meta, arr):
    cfg = meta["config"]
    sd = synthetic.hifigan_state_dict(**cfg, seed=meta["seed"], weight_norm=True)
    z = torch.from_numpy(arr["z_ref_fp64"])
    out = hifigan_ref.hifigan_forward(sd, z, pad=0, g=torch.from_numpy(arr["g"]), dtype=torch.float64,
                                      fold_dtype=torch.float64, **cfg)
    assert max_abs(out.numpy(), arr["out_ref_fp64"]) < 1e-10


HRANGE = goldens("handoff_range")


@pytest.mark.parametrize("name,meta,arr", HRANGE, ids=[g[0] for g in HRANGE])
def test_handoff_range_oracle_matches_reference(name, meta, arr):
    """normalize / denormalize / save_wav scaling executed from the reference source (golden)."""
    from oracle import handoff_ref

    cfgs = meta["configs"]
    for i, j in meta["pairs"]:
        den = handoff_ref.denormalize(arr["mel"].T, cfgs[i]).T
        out = handoff_ref.normalize(den.T, cfgs[j])
        assert out.dtype == np.float32 and np.array_equal(out, arr[f"out_{i}_{j}"]), (i, j)
    for k in range(meta["n_wavs"]):
        assert np.array_equal(handoff_ref.wav_int16(arr[f"wav_{k}"]), arr[f"pcm_{k}"]), k


def test_wav_int16_nonfinite_contract():
    """save_wav (numpy_transforms.py:436-438) on non-finite samples, as numpy does it on x86: a NaN
    makes np.max NaN and max(0.01, nan) = 0.01; the int16 cast goes through int32 (NaN, inf and
    |v| >= 2^31 -> INT_MIN -> 0) and wraps.  tts_wav_to_int16 implements exactly this contract."""
    from oracle import handoff_ref

    with np.errstate(invalid="ignore", over="ignore"):
        w = np.array([0.5, np.nan, -0.2, np.inf, 1e-3, 700.0], dtype=np.float32)
        assert handoff_ref.wav_int16(w).tolist() == [-50, 0, 20, 0, 3276, 0]  # scale 32767 / 0.01
        w = np.array([0.5, -0.2, -np.inf, 0.0], dtype=np.float32)  # max = inf: scale 0, inf * 0 = NaN
        assert handoff_ref.wav_int16(w).tolist() == [0, 0, 0, 0]


VTEXT = goldens("vits_text")


@pytest.mark.parametrize("name,meta,arr", VTEXT, ids=[g[0] for g in VTEXT])
def test_vits_text_oracle_matches_reference(name, meta, arr):
    """oracle/vits_text_ref.py against the reference's Vits.inference chain (make_goldens.py
    vits_text): TextEncoder (with the language embedding concatenated when the fixture has one), the
    SDP reverse with the stored noise or the deterministic DurationPredictor (use_sdp=False), the
    duration glue, the flow, upsampling_z when recorded, and the decoder (fp64 throughout)."""
    from _vits_chain import oracle_chain, state_dicts
    from oracle import vits_text_ref

    o = oracle_chain(meta, arr)
    for n in ("x", "m_p", "logs_p", "x_mask", "logw"):
        assert max_abs(o[n].numpy(), arr[f"{n}_ref_fp64"]) < 1e-10, n
    assert torch.equal(o["w_ceil"], torch.from_numpy(arr["w_ceil_ref_fp64"]))
    assert torch.equal(o["y_lengths"], torch.from_numpy(arr["y_lengths_ref_fp64"]))
    assert torch.equal(o["attn"], torch.from_numpy(arr["attn_ref_fp64"]))
    assert max_abs(o["m_p_exp"].numpy(), arr["m_p_exp_ref_fp64"]) < 1e-12
    assert max_abs(o["z_p"].numpy(), arr["z_p_ref_fp64"]) < 1e-12
    assert torch.equal(o.get("y_mask_up", o["y_mask"]), torch.from_numpy(arr["y_mask_ref_fp64"]))
    assert max_abs(o["z"].numpy(), arr["z_ref_fp64"]) < 1e-10
    assert max_abs(o["wav"].numpy(), arr["wav_ref_fp64"]) < 1e-10
    # fp32 oracle vs the reference's fp32 run, and the duration ceil() margin
    tsd = state_dicts(meta)[0]
    le = torch.from_numpy(arr["lang_emb"]) if meta.get("lang") else None
    x32, _, _, _ = vits_text_ref.text_encoder(tsd, torch.from_numpy(arr["tokens"]), torch.from_numpy(arr["lengths"]),
                                              dtype=torch.float32, lang_emb=le, **meta["text_encoder"])
    assert max_abs(x32.numpy(), arr["x_ref_fp32"]) < 1e-4
    assert meta["ceil_margin"] > 1e-3


def test_vits_upsample_z_oracle_matches_interpolate():
    """upsample_z at non-integer factors: the same F.interpolate call and the float-length sequence
    mask (helpers.sequence_mask on y_lengths * factor) as vits.py:951-957."""
    from oracle import vits_text_ref

    z = torch.randn(2, 3, 10, generator=torch.Generator().manual_seed(3))
    for f in (2.0, 1.5, 3.0):
        z2, m = vits_text_ref.upsample_z(z, torch.tensor([10, 7]), f)
        assert z2.shape[2] == int(10 * f) and m.shape == (2, 1, int(10 * f))
        assert m[1, 0].sum() == np.ceil(7 * f)


def test_rq_spline_inverse_roundtrip():
    """The rational-quadratic spline restatement: forward then inverse returns the input inside the
    tail bound and the identity outside it; log|det| of the two directions cancel."""
    from oracle import vits_text_ref

    gen = torch.Generator().manual_seed(5)
    x = torch.linspace(-6, 6, 97, dtype=torch.float64)
    uw, uh = torch.randn(97, 10, generator=gen).double(), torch.randn(97, 10, generator=gen).double()
    ud = torch.randn(97, 9, generator=gen).double()
    y, l1 = vits_text_ref.rq_spline(x, uw, uh, ud, False, 5.0)
    x2, l2 = vits_text_ref.rq_spline(y, uw, uh, ud, True, 5.0)
    assert max_abs(x2.numpy(), x.numpy()) < 1e-12
    assert max_abs((l1 + l2).numpy(), np.zeros(97)) < 1e-12
    out = (x.abs() > 5.0)
    assert torch.equal(y[out], x[out])
