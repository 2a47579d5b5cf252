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
from oracle import vits_text_ref
from tts_amd import synthetic
from tts_amd.config import VITS_SDP, VITS_TEXT_ENCODER
from tts_amd.tts import StochasticDurationPredictor, TextEncoder, Vits
from tts_amd.tts.vits_text import vits_durations, vits_expand

pytestmark = pytest.mark.gpu
VT = goldens("vits_text")
TEXT_MODES = ["fp32", "fp32x6", "bf16"]  # the text side has no f16x3 statistics (like the Glow encoder)


def _te(meta, dev, mode):
    c = meta["text_encoder"]
    te = TextEncoder(c["num_chars"], c["out_channels"], c["hidden_channels"], c["hidden_channels_ffn"], c["num_heads"],
                     c["num_layers"], c["kernel_size"], 0.1, math_mode=mode)
    te.load_state_dict(synthetic.vits_text_encoder_state_dict(**c, seed=meta["seeds"][0]))
    return te.to(dev)


def _sdp(meta, dev, mode):
    c = meta["sdp"]
    sdp = StochasticDurationPredictor(c["in_channels"], c["hidden_channels"], c["kernel_size"], 0.5, c["num_flows"],
                                      cond_channels=meta["gin"], math_mode=mode)
    sdp.load_state_dict(synthetic.vits_sdp_state_dict(**c, cond_channels=meta["gin"], seed=meta["seeds"][1]))
    return sdp.to(dev)


def _op_tol(mode):
    return tol(mode) if mode == "bf16" else dict(max_abs_tol=1e-4, rel_rms_tol=5e-6)


@pytest.mark.parametrize("mode", TEXT_MODES)
@pytest.mark.parametrize("name,meta,arr", VT, ids=[v[0] for v in VT])
def test_text_encoder_vs_reference(cuda_device, name, meta, arr, mode):
    te = _te(meta, cuda_device, mode)
    x, m, logs, xm = te(torch.from_numpy(arr["tokens"]).to(cuda_device), torch.from_numpy(arr["lengths"]).to(cuda_device))
    assert torch.equal(xm.cpu(), torch.from_numpy(arr["x_mask_ref_fp32"]))
    for n, o in (("x", x), ("m_p", m), ("logs_p", logs)):
        assert_close_fp32(o.cpu(), arr[f"{n}_ref_fp64"], f"{name} {n} ({mode})", **_op_tol(mode))


@pytest.mark.parametrize("mode", TEXT_MODES)
@pytest.mark.parametrize("name,meta,arr", VT, ids=[v[0] for v in VT])
def test_sdp_reverse_vs_reference(cuda_device, name, meta, arr, mode):
    """logw from the reference's own fp64 encoder state and the stored noise draw; then the durations
    (ceil) and y_lengths bit-exact in the fp32-faithful modes."""
    sdp = _sdp(meta, cuda_device, mode)
    x = torch.from_numpy(arr["x_ref_fp64"]).float().to(cuda_device)
    xm = torch.from_numpy(arr["x_mask_ref_fp64"]).float().to(cuda_device)
    g = torch.from_numpy(arr["g"]).to(cuda_device) if meta["gin"] else None
    logw = sdp(x, xm, g=g, reverse=True, noise_scale=meta["noise_scale_dp"],
               noise=torch.from_numpy(arr["noise_dp"]).to(cuda_device))
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
    assert torch.equal(y_mask.cpu(), torch.from_numpy(arr["y_mask_ref_fp32"]))
    assert torch.equal(mp.cpu(), torch.from_numpy(arr["m_p_exp_ref_fp32"]))
    assert torch.equal(lp.cpu(), torch.from_numpy(arr["logs_p_exp_ref_fp32"]))
    assert np.abs(z_p.cpu().numpy() - arr["z_p_ref_fp32"]).max() <= 1e-6


def _vits(meta, dev, text_mode, flow_mode, dec_mode):
    gin = meta["gin"]
    dc = meta["decoder"]
    args = dict(num_chars=meta["text_encoder"]["num_chars"], hidden_channels=meta["text_encoder"]["hidden_channels"],
                num_layers_text_encoder=meta["text_encoder"]["num_layers"],
                upsample_initial_channel_decoder=dc["upsample_initial_channel"],
                use_d_vector_file=bool(gin), d_vector_dim=gin)
    v = Vits(args, text_math_mode=text_mode, flow_math_mode=flow_mode, decoder_math_mode=dec_mode)
    v.text_encoder.load_state_dict(synthetic.vits_text_encoder_state_dict(**meta["text_encoder"],
                                                                          seed=meta["seeds"][0]))
    v.duration_predictor.load_state_dict(synthetic.vits_sdp_state_dict(**meta["sdp"], cond_channels=gin,
                                                                       seed=meta["seeds"][1]))
    v.flow.load_state_dict(synthetic.vits_flow_state_dict(**dict(meta["flow"], cond_channels=gin), seed=meta["seeds"][2]))
    v.waveform_decoder.load_state_dict(synthetic.hifigan_state_dict(**dict(dc, cond_channels=gin), seed=meta["seeds"][3],
                                                                    weight_norm=True))
    return v.to(dev)


@pytest.mark.parametrize("modes", [("fp32", "fp32", "fp32"), ("fp32x6", "f16x3", "f16x3"), ("bf16", "bf16", "bf16")],
                         ids=["fp32", "faithful", "bf16"])
@pytest.mark.parametrize("name,meta,arr", VT, ids=[v[0] for v in VT])
def test_vits_inference_tokens_to_wav(cuda_device, name, meta, arr, modes):
    """Vits.inference end to end (tokens -> waveform) with the reference's two noise draws, against
    the reference chain's fp64 output; the durations bit-exact in the fp32-faithful modes."""
    d = cuda_device
    v = _vits(meta, d, *modes)
    aux = {"x_lengths": torch.from_numpy(arr["lengths"]).to(d), "noise_dp": torch.from_numpy(arr["noise_dp"]).to(d),
           "noise_z": torch.from_numpy(arr["noise_z"]).to(d)}
    if meta["gin"]:
        # the fixture's g is the raw [B, gin, 1] vector; d_vectors are normalised by _set_cond_input,
        # so feed a d-vector whose normalisation is g itself only when |g| = 1: pass g straight instead
        v._set_cond_input = lambda a: (None, torch.from_numpy(arr["g"]).to(d), None)
    out = v.inference(torch.from_numpy(arr["tokens"]).to(d), aux)
    faithful = modes[0] != "bf16"
    if faithful:
        assert torch.equal(out["durations"].cpu(), torch.from_numpy(arr["w_ceil_ref_fp64"]).float())
        assert torch.equal(out["alignments"].cpu(), torch.from_numpy(arr["attn_ref_fp64"]).float())
        assert_close_fp32(out["z"].cpu(), arr["z_ref_fp64"], f"{name} z ({modes})", max_abs_tol=1e-4)
        assert_close_fp32(out["model_outputs"].cpu(), arr["wav_ref_fp64"], f"{name} wav ({modes})")
    else:
        # bf16: the durations may round differently, so compare where the lengths agree
        if torch.equal(out["durations"].cpu(), torch.from_numpy(arr["w_ceil_ref_fp64"]).float()):
            assert_close_fp32(out["model_outputs"].cpu(), arr["wav_ref_fp64"], f"{name} wav (bf16)", **tol("bf16"))
        assert torch.isfinite(out["model_outputs"]).all()


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
