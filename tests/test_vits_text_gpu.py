"""VITS text side on MI355X through the C-ABI: TextEncoder, StochasticDurationPredictor (reverse),
the duration / alignment glue and the whole Vits.inference chain, against the reference's own
outputs (tests/golden/vits_text_*.npz, make_goldens.py vits_text) and the fp64 oracle
(oracle/vits_text_ref.py).

Gates (tests/_util.py): fp32-faithful modes rel-RMS <= 5e-6; waveform max|d| <= 1e-5; the text
side's unbounded outputs max|d| <= 1e-4 (x, m_p, logs_p, logw are O(1..10)); durations, y_lengths,
the alignment and y_mask bit-exact (every fixture duration is >= 1e-3 from an integer,
``ceil_margin``); bf16: SURVEY §8c's rel-RMS 3e-2.
"""
import numpy as np
import pytest
import torch

from _util import assert_close_fp32, goldens, tol
from _vits_chain import oracle_chain, state_dicts
from oracle import vits_text_ref
from tts_amd import synthetic
from tts_amd.config import VITS_SDP, VITS_TEXT_ENCODER
from tts_amd.tts import DurationPredictor, StochasticDurationPredictor, TextEncoder, Vits
from tts_amd.tts.vits_text import vits_durations, vits_expand

pytestmark = pytest.mark.gpu
VT = goldens("vits_text")
TEXT_MODES = ["fp32", "fp32x6", "bf16"]  # the text side has no f16x3 statistics (like the Glow encoder)


def _te(meta, dev, mode):
    c = meta["text_encoder"]
    L = meta.get("lang", 0)
    te = TextEncoder(c["num_chars"], c["out_channels"], c["hidden_channels"], c["hidden_channels_ffn"], c["num_heads"],
                     c["num_layers"], c["kernel_size"], 0.1, language_emb_dim=L or None, math_mode=mode)
    te.load_state_dict(state_dicts(meta)[0])
    return te.to(dev)


def _lang(meta, arr, dev):
    return torch.from_numpy(arr["lang_emb"]).to(dev) if meta.get("lang") else None


def _dp(meta, dev, mode):
    """The fixture's duration predictor: the SDP, or the deterministic one (use_sdp=False)."""
    c, L = meta["sdp"], meta.get("lang", 0)
    if meta.get("use_sdp", True):
        dp = StochasticDurationPredictor(c["in_channels"], c["hidden_channels"], c["kernel_size"], 0.5, c["num_flows"],
                                         cond_channels=meta["gin"], language_emb_dim=L, math_mode=mode)
    else:
        dp = DurationPredictor(meta["text_encoder"]["hidden_channels"], 256, 3, 0.5, cond_channels=meta["gin"],
                               language_emb_dim=L, math_mode=mode)
    dp.load_state_dict(state_dicts(meta)[1])
    return dp.to(dev)


def _op_tol(mode):
    return tol(mode, op=True) if mode == "bf16" else dict(max_abs_tol=1e-4, rel_rms_tol=5e-6)


@pytest.mark.parametrize("mode", TEXT_MODES)
@pytest.mark.parametrize("name,meta,arr", VT, ids=[v[0] for v in VT])
def test_text_encoder_vs_reference(cuda_device, name, meta, arr, mode):
    te = _te(meta, cuda_device, mode)
    x, m, logs, xm = te(torch.from_numpy(arr["tokens"]).to(cuda_device), torch.from_numpy(arr["lengths"]).to(cuda_device),
                        lang_emb=_lang(meta, arr, cuda_device))
    assert torch.equal(xm.cpu(), torch.from_numpy(arr["x_mask_ref_fp32"]))
    for n, o in (("x", x), ("m_p", m), ("logs_p", logs)):
        assert_close_fp32(o.cpu(), arr[f"{n}_ref_fp64"], f"{name} {n} ({mode})", **_op_tol(mode))


@pytest.mark.parametrize("mode", TEXT_MODES)
@pytest.mark.parametrize("name,meta,arr", VT, ids=[v[0] for v in VT])
def test_sdp_reverse_vs_reference(cuda_device, name, meta, arr, mode):
    """logw from the reference's own fp64 encoder state (and the stored noise draw for the SDP; the
    deterministic DurationPredictor for use_sdp=False fixtures, with the language embedding when
    recorded); then the durations (ceil) and y_lengths bit-exact in the fp32-faithful modes."""
    dp = _dp(meta, cuda_device, mode)
    x = torch.from_numpy(arr["x_ref_fp64"]).float().to(cuda_device)
    xm = torch.from_numpy(arr["x_mask_ref_fp64"]).float().to(cuda_device)
    g = torch.from_numpy(arr["g"]).to(cuda_device) if meta["gin"] else None
    le = _lang(meta, arr, cuda_device)
    if meta.get("use_sdp", True):
        logw = dp(x, xm, g=g, reverse=True, noise_scale=meta["noise_scale_dp"], lang_emb=le,
                  noise=torch.from_numpy(arr["noise_dp"]).to(cuda_device))
    else:
        logw = dp(x, xm, g=g, lang_emb=le)
    assert_close_fp32(logw.cpu(), arr["logw_ref_fp64"], f"{name} logw ({mode})", **_op_tol(mode))
    if mode != "bf16":
        w_ceil, y_len = vits_durations(logw, xm, meta["length_scale"])
        assert torch.equal(w_ceil.cpu(), torch.from_numpy(arr["w_ceil_ref_fp64"]).float())
        assert torch.equal(y_len.cpu(), torch.from_numpy(arr["y_lengths_ref_fp64"]))


@pytest.mark.parametrize("name,meta,arr", VT, ids=[v[0] for v in VT])
def test_glue_bit_exact(cuda_device, name, meta, arr):
    """vits.py:1145-1154 on the reference's fp32 tensors: w_ceil, y_lengths, attn, y_mask and the
    expanded m_p / logs_p bit for bit (a gather: one product by 1.0); z_p to fp32 rounding."""
    d = cuda_device
    logw = torch.from_numpy(arr["logw_ref_fp32"]).to(d)
    xm = torch.from_numpy(arr["x_mask_ref_fp32"]).to(d)
    w_ceil, y_len = vits_durations(logw, xm, meta["length_scale"])
    assert torch.equal(w_ceil.cpu(), torch.from_numpy(arr["w_ceil_ref_fp32"]))
    assert torch.equal(y_len.cpu(), torch.from_numpy(arr["y_lengths_ref_fp32"]))
    m_p = torch.from_numpy(arr["m_p_ref_fp32"]).to(d)
    logs_p = torch.from_numpy(arr["logs_p_ref_fp32"]).to(d)
    z_p, y_mask, mp, lp, attn = vits_expand(w_ceil, xm, y_len, m_p, logs_p, torch.from_numpy(arr["noise_z"]).to(d),
                                            meta["noise_scale"])
    assert torch.equal(attn.cpu(), torch.from_numpy(arr["attn_ref_fp32"]))
    if meta.get("up_factor"):  # the fixture's y_mask is upsampling_z's (checked in the tokens -> wav test)
        yl = torch.from_numpy(arr["y_lengths_ref_fp32"])
        ref_mask = (torch.arange(y_mask.shape[2])[None] < yl[:, None]).float().unsqueeze(1)
        assert torch.equal(y_mask.cpu(), ref_mask)
    else:
        assert torch.equal(y_mask.cpu(), torch.from_numpy(arr["y_mask_ref_fp32"]))
    assert torch.equal(mp.cpu(), torch.from_numpy(arr["m_p_exp_ref_fp32"]))
    assert torch.equal(lp.cpu(), torch.from_numpy(arr["logs_p_exp_ref_fp32"]))
    assert np.abs(z_p.cpu().numpy() - arr["z_p_ref_fp32"]).max() <= 1e-6


def _vits(meta, dev, text_mode, flow_mode, dec_mode, arr=None):
    gin, L = meta["gin"], meta.get("lang", 0)
    dc = meta["decoder"]
    args = dict(num_chars=meta["text_encoder"]["num_chars"], hidden_channels=meta["text_encoder"]["hidden_channels"],
                num_layers_text_encoder=meta["text_encoder"]["num_layers"],
                upsample_initial_channel_decoder=dc["upsample_initial_channel"],
                use_d_vector_file=bool(gin), d_vector_dim=gin, use_sdp=meta.get("use_sdp", True))
    if L:
        args.update(use_language_embedding=True, num_languages=arr["emb_l"].shape[0], embedded_language_dim=L)
    if meta.get("up_factor"):  # interpolate_factor = sample_rate / encoder_sample_rate
        args.update(sample_rate=int(22050 * meta["up_factor"]), encoder_sample_rate=22050)
    v = Vits(args, text_math_mode=text_mode, flow_math_mode=flow_mode, decoder_math_mode=dec_mode)
    tsd, dsd, fsd, dec = state_dicts(meta)
    v.text_encoder.load_state_dict(tsd)
    v.duration_predictor.load_state_dict(dsd)
    v.flow.load_state_dict(fsd)
    v.waveform_decoder.load_state_dict(dec)
    if L:
        v.emb_l.weight.data.copy_(torch.from_numpy(arr["emb_l"]))
    return v.to(dev)


@pytest.mark.parametrize("modes", [("fp32", "fp32", "fp32"), ("fp32x6", "f16x3", "f16x3"), ("bf16", "bf16", "bf16")],
                         ids=["fp32", "faithful", "bf16"])
@pytest.mark.parametrize("name,meta,arr", VT, ids=[v[0] for v in VT])
def test_vits_inference_tokens_to_wav(cuda_device, name, meta, arr, modes):
    """Vits.inference end to end (tokens -> waveform) with the reference's two noise draws, against
    the reference chain's fp64 output; the durations bit-exact in the fp32-faithful modes.  In bf16
    the durations may cross a ceil boundary (at most one frame per token is allowed), so the
    waveform is always compared against the fp64 chain run on the device's own durations (and
    against the reference's golden as well when they agree)."""
    d = cuda_device
    v = _vits(meta, d, *modes, arr=arr)
    noise_z = torch.from_numpy(arr["noise_z"])
    faithful = modes[0] != "bf16"
    if not faithful:  # room for longer bf16 durations: the stored draw, then seeded normal frames
        extra = torch.randn(noise_z.shape[0], noise_z.shape[1], 64, generator=torch.Generator().manual_seed(5))
        noise_z = torch.cat([noise_z, extra], 2)
    aux = {"x_lengths": torch.from_numpy(arr["lengths"]).to(d), "noise_dp": torch.from_numpy(arr["noise_dp"]).to(d),
           "noise_z": noise_z.to(d)}
    if meta.get("lang"):
        aux["language_ids"] = torch.from_numpy(arr["lids"]).to(d)  # emb_l(lid) on the device
    if meta["gin"]:
        # the fixture's g is the raw [B, gin, 1] vector; d_vectors are normalised by _set_cond_input,
        # so feed a d-vector whose normalisation is g itself only when |g| = 1: pass g straight instead
        v._set_cond_input = lambda a: (None, torch.from_numpy(arr["g"]).to(d), a.get("language_ids"), None)
    out = v.inference(torch.from_numpy(arr["tokens"]).to(d), aux)
    if faithful:
        assert torch.equal(out["durations"].cpu(), torch.from_numpy(arr["w_ceil_ref_fp64"]).float())
        assert torch.equal(out["alignments"].cpu(), torch.from_numpy(arr["attn_ref_fp64"]).float())
        assert_close_fp32(out["z"].cpu(), arr["z_ref_fp64"], f"{name} z ({modes})", max_abs_tol=1e-4)
        assert_close_fp32(out["model_outputs"].cpu(), arr["wav_ref_fp64"], f"{name} wav ({modes})")
    else:
        wc = out["durations"].cpu().double()
        wc_ref = torch.from_numpy(arr["w_ceil_ref_fp64"])
        assert (wc - wc_ref).abs().max() <= 1, "bf16 durations more than one frame off the reference's"
        ref = oracle_chain(meta, arr, w_ceil=wc, noise_z=noise_z, start_from_reference=True)["wav"]
        assert_close_fp32(out["model_outputs"].cpu(), ref, f"{name} wav (bf16, device durations)", **tol("bf16"))
        if torch.equal(wc, wc_ref):
            assert_close_fp32(out["model_outputs"].cpu(), arr["wav_ref_fp64"], f"{name} wav (bf16)", **tol("bf16"))


@pytest.mark.parametrize("noise_scale", [0.0, 1.0, 4.0])
def test_sdp_vs_oracle_ragged_and_tails(cuda_device, noise_scale):
    """The SDP on a ragged batch (lengths 37, 20, 1) against the fp64 oracle; noise_scale 4 puts many
    spline inputs outside the tail bound 5 (the linear-tail identity branch)."""
    gen = torch.Generator().manual_seed(17)
    B, T = 3, 37
    lens = torch.tensor([37, 20, 1])
    xm = (torch.arange(T)[None] < lens[:, None]).float().unsqueeze(1)
    x = torch.randn(B, 192, T, generator=gen) * xm
    noise = torch.randn(B, 2, T, generator=gen)
    sd = synthetic.vits_sdp_state_dict(**VITS_SDP, seed=31)
    ref = vits_text_ref.sdp_reverse(sd, x, xm, noise, noise_scale=noise_scale, dtype=torch.float64, **VITS_SDP)
    sdp = StochasticDurationPredictor(192, 192, 3, 0.5, 4, math_mode="fp32x6")
    sdp.load_state_dict(sd)
    sdp = sdp.to(cuda_device)
    out = sdp(x.to(cuda_device), xm.to(cuda_device), reverse=True, noise_scale=noise_scale, noise=noise.to(cuda_device))
    assert_close_fp32(out.cpu(), ref, f"sdp noise_scale={noise_scale}", max_abs_tol=1e-4)


def test_text_encoder_batch_invariance(cuda_device):
    """A full-length utterance alone equals its row of a padded batch bit for bit."""
    meta, arr = VT[0][1], VT[0][2]
    te = _te(meta, cuda_device, "fp32x6")
    tok = torch.from_numpy(arr["tokens"]).to(cuda_device)
    lens = torch.from_numpy(arr["lengths"]).to(cuda_device)
    full = te(tok, lens)
    one = te(tok[:1], lens[:1])
    for a, b in zip(full, one):
        assert torch.equal(a[:1], b)


def test_vits_glue_kernels_vs_torch(cuda_device):
    """The round-6 glue kernels against the reference's own torch expressions (vits.py:1141-1161,
    :884-886, :944-959): given durations, the masked slice, upsampling_z (F.interpolate + the
    float-length sequence mask), embedding rows and the d-vector normalisation."""
    from tts_amd.tts.vits_text import (embedding_rows, l2_normalize_rows, vits_durations_given, vits_mask_slice,
                                       vits_upsample_z)

    d = cuda_device
    gen = torch.Generator().manual_seed(23)
    dur = torch.rand(1, 9, generator=gen) * 6  # durations [1, T_x] (vits.py:1143: unsqueeze(0))
    dur[0, 3] = 0.0
    w_ceil, y_len = vits_durations_given(dur.to(d), 3, 9, d)
    ref_w = torch.ceil(dur.unsqueeze(0)).expand(3, 1, 9)
    assert torch.equal(w_ceil.cpu(), ref_w)
    assert torch.equal(y_len.cpu(), torch.clamp_min(torch.sum(ref_w, [1, 2]), 1).long())
    per = torch.rand(3, 9, generator=gen) * 4  # one row per utterance
    w2, y2 = vits_durations_given(per.to(d), 3, 9, d)
    assert torch.equal(w2.cpu(), torch.ceil(per).unsqueeze(1))
    z = torch.randn(3, 5, 40, generator=gen)
    ym = (torch.arange(40)[None] < torch.tensor([40, 31, 7])[:, None]).float().unsqueeze(1)
    for T_out in (None, 33, 1):
        got = vits_mask_slice(z.to(d), ym.to(d), T_out)
        assert torch.equal(got.cpu(), (z * ym)[:, :, :T_out])
    for T, f in ((40, 2.0), (40, 1.5), (37, 3.0), (16, 1.0)):
        yl = torch.tensor([T, T - 9, 3])
        z2, m2 = vits_upsample_z(z[:, :, :T].to(d), yl.to(d), f)
        r2, rm = vits_text_ref.upsample_z(z[:, :, :T], yl, f)
        assert z2.shape == r2.shape and torch.equal(m2.cpu(), rm)
        assert (z2.cpu() - r2).abs().max() <= 1e-6 * max(1.0, r2.abs().max().item()), (T, f)
    table = torch.nn.Embedding(5, 7).to(d)
    ids = torch.tensor([4, 0, 2], device=d)
    assert torch.equal(embedding_rows(table, ids), table(ids).detach())
    dv = torch.randn(3, 64, generator=gen)
    dv[2] = 0.0  # the eps branch
    assert (l2_normalize_rows(dv.to(d), d).cpu() - torch.nn.functional.normalize(dv)).abs().max() <= 1e-7


@pytest.mark.parametrize("name,meta,arr", VT[:1], ids=[v[0] for v in VT[:1]])
def test_vits_inference_given_durations(cuda_device, name, meta, arr):
    """aux_input["durations"] (vits.py:1141-1146): the predictor is skipped, w_ceil = ceil(durations) for
    every utterance, and the waveform matches the fp64 chain on those durations."""
    d = cuda_device
    v = _vits(meta, d, "fp32x6", "f16x3", "f16x3", arr=arr)
    B, T = arr["tokens"].shape
    dur = torch.linspace(0.5, 4.2, T).reshape(1, T)
    noise_z = torch.randn(B, 192, 64, generator=torch.Generator().manual_seed(8))
    out = v.inference(torch.from_numpy(arr["tokens"]).to(d), {"x_lengths": torch.from_numpy(arr["lengths"]).to(d),
                                                             "durations": dur.to(d), "noise_z": noise_z.to(d)})
    wc = torch.ceil(dur).reshape(1, 1, T).expand(B, 1, T).contiguous()
    assert torch.equal(out["durations"].cpu(), wc)
    ref = oracle_chain(meta, arr, w_ceil=wc, noise_z=noise_z)
    assert_close_fp32(out["model_outputs"].cpu(), ref["wav"], f"{name} wav (given durations)")


def test_sdp_widest_hidden_vs_oracle(cuda_device):
    """The SDP at the widest hidden width its validation accepts (512: the depthwise / LayerNorm
    kernels stage [C][64] floats, 128 KiB of LDS, past the 64 KiB default dynamic limit)."""
    gen = torch.Generator().manual_seed(29)
    B, T, H = 2, 21, 512
    lens = torch.tensor([21, 12])
    xm = (torch.arange(T)[None] < lens[:, None]).float().unsqueeze(1)
    x = torch.randn(B, 192, T, generator=gen) * xm
    noise = torch.randn(B, 2, T, generator=gen)
    cfg = dict(VITS_SDP, hidden_channels=H)
    sd = synthetic.vits_sdp_state_dict(**cfg, seed=37)
    ref = vits_text_ref.sdp_reverse(sd, x, xm, noise, noise_scale=1.0, dtype=torch.float64, **cfg)
    sdp = StochasticDurationPredictor(192, H, 3, 0.5, 4, math_mode="fp32x6")
    sdp.load_state_dict(sd)
    out = sdp.to(cuda_device)(x.to(cuda_device), xm.to(cuda_device), reverse=True, noise_scale=1.0,
                              noise=noise.to(cuda_device))
    assert_close_fp32(out.cpu(), ref, "sdp hidden 512", max_abs_tol=1e-4)


def test_vits_inference_upsampling_non_integer_factor(cuda_device):
    """upsampling_z at a non-integer interpolate_factor (24 kHz audio from a 16 kHz encoder: 1.5) through
    Vits.inference with given durations (an even T_y, so the reference's z * y_mask shapes agree), against
    the fp64 chain; an odd T_y raises as the reference's broadcast does."""
    meta, arr = VT[0][1], VT[0][2]
    d = cuda_device
    m = dict(meta, up_factor=1.5)
    v = _vits(m, d, "fp32x6", "f16x3", "f16x3", arr=arr)
    assert abs(v.interpolate_factor - 1.5) < 1e-12
    B, T = arr["tokens"].shape
    dur = torch.full((1, T), 2.0)
    dur[0, 0] = 3.0  # two 3-frame tokens: T_y = 2 T + 2, even
    dur[0, 1] = 3.0
    noise_z = torch.randn(B, 192, 64, generator=torch.Generator().manual_seed(12))
    aux = {"x_lengths": torch.from_numpy(arr["lengths"]).to(d), "durations": dur.to(d), "noise_z": noise_z.to(d)}
    out = v.inference(torch.from_numpy(arr["tokens"]).to(d), aux)
    T_y = int(dur.sum())
    assert T_y % 2 == 0 and out["z"].shape[2] == int(T_y * 1.5)
    wc = torch.ceil(dur).reshape(1, 1, T).expand(B, 1, T).contiguous()
    ref = oracle_chain(m, arr, w_ceil=wc, noise_z=noise_z)
    assert torch.equal(out["y_mask"].cpu(), ref["y_mask_up"])
    assert_close_fp32(out["z"].cpu(), ref["z"], "upsampled z (x1.5)", max_abs_tol=1e-4)
    assert_close_fp32(out["model_outputs"].cpu(), ref["wav"], "wav (upsampling x1.5)")
    dur[0, 2] = 3.0  # odd T_y: floor(1.5 T_y) frames of z against ceil(1.5 T_y) of mask
    aux["durations"] = dur.to(d)
    with pytest.raises(RuntimeError, match="upsampling_z"):
        v.inference(torch.from_numpy(arr["tokens"]).to(d), aux)
