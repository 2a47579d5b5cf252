"""Glow-TTS text side on MI355X: the Encoder (rel_pos_transformer and the gated_conv /
residual_conv_bn / time_depth_separable types), the duration / alignment glue and GlowTTS.inference
end to end (tokens -> mel), against the reference goldens and the oracle."""
import numpy as np
import pytest
import torch

from _util import assert_close_fp32, goldens, max_abs
from oracle import glow_ref, glow_tts_ref
from tts_amd import _native as N
from tts_amd import synthetic
from tts_amd.config import GLOW_TTS_ENCODER
from tts_amd.tts import Encoder, GlowTTS

pytestmark = pytest.mark.gpu
GENC = goldens("glow_encoder")
GTTS = goldens("glow_tts")
# encoder outputs: 6 transformer layers of fp32 (LayerNorm, softmax); the reference's own
# fp32-vs-fp64 error on x_m is 1.3e-6
# (measured on MI355X: max 4.4e-6, rel-RMS 1.2e-6)
ENC_MAX_ABS = 5e-5
ENC_REL_RMS = 5e-6
# mel after the 12-flow decoder (reference fp32 vs fp64: 5.5e-6)
# (measured on MI355X: max 1.2e-5, rel-RMS 9.5e-7)
MEL_MAX_ABS = 5e-5
MEL_REL_RMS = 5e-6


def build_encoder(cfg, seed, device, math_mode="fp32x6"):
    e = Encoder(cfg["num_chars"], cfg["out_channels"], cfg["hidden_channels"], cfg["hidden_channels_dp"],
                cfg.get("encoder_type", "rel_pos_transformer"), cfg["encoder_params"], mean_only=cfg["mean_only"],
                use_prenet=cfg["use_prenet"], c_in_channels=cfg.get("c_in_channels", 0), math_mode=math_mode)
    e.load_state_dict(synthetic.glow_encoder_state_dict(**cfg, seed=seed))
    e.eval()
    return e.to(device)


def speaker_g(arr):
    """the fixture's d-vectors -> g = F.normalize(d).unsqueeze(-1) (glow_tts.py:189-190), or None"""
    if "d_vectors" not in arr:
        return None
    return torch.nn.functional.normalize(torch.from_numpy(arr["d_vectors"])).unsqueeze(-1)


def build_glow_tts(meta, device, decoder_math_mode="fp32", **speaker):
    ecfg, dcfg = meta["encoder"], meta["decoder"]
    c_in = ecfg.get("c_in_channels", 0)
    if c_in and not speaker:
        speaker = dict(use_d_vector_file=True, d_vector_dim=c_in)
    m = GlowTTS(dict(num_chars=ecfg["num_chars"], inference_noise_scale=meta["noise_scale"],
                     length_scale=meta["length_scale"], **speaker), decoder_math_mode=decoder_math_mode)
    sd = {f"encoder.{k}": v for k, v in synthetic.glow_encoder_state_dict(**ecfg, seed=meta["eseed"]).items()}
    sd.update({f"decoder.{k}": v for k, v in synthetic.glow_decoder_state_dict(**dcfg, seed=meta["dseed"]).items()})
    if hasattr(m, "emb_g"):
        sd["emb_g.weight"] = meta["emb_g"]
    m.load_state_dict(sd)
    m.eval()
    m.store_inverse()
    return m.to(device)


@pytest.mark.parametrize("name,meta,arr", GENC + [(n, dict(m, config=m["encoder"], seed=m["eseed"]), a)
                                                   for n, m, a in GTTS],
                         ids=[g[0] for g in GENC + GTTS])
@pytest.mark.parametrize("mode", ["fp32", "fp32x6"])
def test_encoder_vs_reference(cuda_device, name, meta, arr, mode):
    e = build_encoder(meta["config"], meta["seed"], cuda_device, mode)
    tok = torch.from_numpy(arr["tokens"]).to(cuda_device)
    lens = torch.from_numpy(arr["lengths"]).to(cuda_device)
    g = speaker_g(arr)
    x_m, x_logs, logw, x_mask = e(tok, lens, None if g is None else g.to(cuda_device))
    assert torch.equal(x_mask.cpu(), torch.from_numpy(arr["x_mask_ref_fp64"]).float())
    assert_close_fp32(x_m.cpu(), arr["x_m_ref_fp64"], f"{name} x_m", ENC_MAX_ABS, ENC_REL_RMS)
    assert_close_fp32(logw.cpu(), arr["logw_ref_fp64"], f"{name} logw", ENC_MAX_ABS, ENC_REL_RMS)
    if "x_logs_ref_fp64" in arr:
        assert_close_fp32(x_logs.cpu(), arr["x_logs_ref_fp64"], f"{name} x_logs", ENC_MAX_ABS, ENC_REL_RMS)


@pytest.mark.parametrize("B,T,lengths,window", [
    (1, 1, [1], None), (2, 9, [9, 4], 4), (3, 70, [70, 65, 1], None), (4, 200, [200, 133, 64, 7], 4),
])
@pytest.mark.parametrize("mode", ["fp32", "fp32x6"])
def test_encoder_vs_oracle(cuda_device, B, T, lengths, window, mode):
    """Shapes around the kernels' tile edges (8-query blocks, 64-key chunks, 16-column LayerNorm
    blocks, 128-column conv tiles), and T = 1."""
    ep = dict(GLOW_TTS_ENCODER["encoder_params"], rel_attn_window_size=window)
    cfg = dict(GLOW_TTS_ENCODER, num_chars=50, encoder_params=ep)
    e = build_encoder(cfg, 7 + T, cuda_device, mode)
    tok = synthetic.tokens(B, T, 50, seed=T)
    lens = torch.tensor(lengths)
    outs = e(tok.to(cuda_device), lens.to(cuda_device))
    sd = synthetic.glow_encoder_state_dict(**cfg, seed=7 + T)
    ref = glow_tts_ref.encoder_forward(sd, tok, lens, hidden_channels=192, encoder_params=ep, mean_only=True,
                                       use_prenet=True)
    for n, o, r in zip(["x_m", "x_logs", "logw"], outs, ref):
        assert_close_fp32(o.cpu(), r, f"{n} B={B} T={T}", ENC_MAX_ABS, ENC_REL_RMS)


ENC_TYPE_CFGS = {
    "gated_conv": dict(encoder_params={"kernel_size": 5, "dropout_p": 0.1, "num_layers": 3}, use_prenet=True),
    "residual_conv_bn": dict(encoder_params={"kernel_size": 4, "dilations": [1, 2, 4], "num_conv_blocks": 2,
                                             "num_res_blocks": 3}, use_prenet=False),
    "time_depth_separable": dict(encoder_params={"kernel_size": 5, "num_layers": 3}, use_prenet=True),
}


@pytest.mark.parametrize("et", list(ENC_TYPE_CFGS))
@pytest.mark.parametrize("B,T,lengths", [(1, 13, [13]), (2, 70, [70, 33]), (3, 130, [130, 129, 16])])
@pytest.mark.parametrize("mode", ["fp32", "fp32x6"])
def test_encoder_types_vs_oracle(cuda_device, et, B, T, lengths, mode):
    """The other encoder types at the default width (H = 192: 2H = 384-channel LayerNorm / GLU)
    on ragged batches; the shortest span the residual_conv_bn kernels allow (3 * 4 + 1 tokens)."""
    cfg = dict(GLOW_TTS_ENCODER, num_chars=50, encoder_type=et, mean_only=False, **ENC_TYPE_CFGS[et])
    e = build_encoder(cfg, 11 + T, cuda_device, mode)
    tok = synthetic.tokens(B, T, 50, seed=T + 1)
    lens = torch.tensor(lengths)
    outs = e(tok.to(cuda_device), lens.to(cuda_device))
    sd = synthetic.glow_encoder_state_dict(**cfg, seed=11 + T)
    ref = glow_tts_ref.encoder_forward(sd, tok, lens, hidden_channels=192, encoder_params=cfg["encoder_params"],
                                       mean_only=False, use_prenet=cfg["use_prenet"], encoder_type=et)
    for n, o, r in zip(["x_m", "x_logs", "logw"], outs, ref):
        assert_close_fp32(o.cpu(), r, f"{et} {n} B={B} T={T}", ENC_MAX_ABS, ENC_REL_RMS)


def test_encoder_residual_bn_too_short_raises(cuda_device):
    """the reference's unpadded dilated conv raises on fewer tokens than its span (res_conv_bn.py:39)"""
    cfg = dict(GLOW_TTS_ENCODER, num_chars=50, encoder_type="residual_conv_bn", mean_only=False,
               **ENC_TYPE_CFGS["residual_conv_bn"])
    e = build_encoder(cfg, 3, cuda_device, "fp32")
    tok = synthetic.tokens(1, 12, 50, seed=1).to(cuda_device)
    with pytest.raises(N.NativeError):
        e(tok, torch.tensor([12], device=cuda_device))


@pytest.mark.parametrize("name,meta,arr", GTTS, ids=[g[0] for g in GTTS])
def test_glue_vs_reference_exact(cuda_device, name, meta, arr):
    """durations + generate_path + compute_outputs + z on the reference's own encoder outputs:
    integer / selection work, bit-exact (z: one fp32 fma chain per element, identical order)."""
    dev = cuda_device
    logw = torch.from_numpy(arr["logw_ref_fp32"]).to(dev)
    xm = torch.from_numpy(arr["x_mask_ref_fp32"]).to(dev)
    B, _, Tx = logw.shape
    w_ceil = torch.empty(B, 1, Tx, device=dev)
    y_len = torch.empty(B, dtype=torch.int64, device=dev)
    dur = torch.empty(B, 1, Tx, device=dev)
    s = N.stream_ptr(dev)
    N.call("tts_glow_durations", N.ptr(logw), N.ptr(xm), B, Tx, float(meta["length_scale"]), N.ptr(w_ceil),
           N.ptr(y_len), N.ptr(dur), s)
    assert torch.equal(w_ceil.cpu(), torch.from_numpy(arr["w_ceil_ref_fp32"]))
    assert torch.equal(y_len.cpu(), torch.from_numpy(arr["y_lengths_ref_fp32"]))
    np.testing.assert_allclose(dur.cpu().numpy(), arr["o_attn_dur_ref_fp32"], rtol=0, atol=1e-6)
    Ty = int(y_len.max())
    om = torch.from_numpy(arr["x_m_ref_fp32"]).to(dev)
    C = om.shape[1]
    noise = torch.from_numpy(arr["noise"]).to(dev)
    z = torch.empty(B, C, Ty, device=dev)
    ym = torch.empty(B, 1, Ty, device=dev)
    ymean = torch.empty(B, C, Ty, device=dev)
    yls = torch.empty(B, C, Ty, device=dev)
    attn = torch.empty(B, Tx, Ty, device=dev)
    N.call("tts_glow_expand", N.ptr(w_ceil), N.ptr(xm), N.ptr(y_len), N.ptr(om), N.ptr(None), N.ptr(noise),
           float(meta["noise_scale"]), B, C, Tx, Ty, N.ptr(z), N.ptr(ym), N.ptr(ymean), N.ptr(yls), N.ptr(attn), s)
    assert torch.equal(attn.cpu(), torch.from_numpy(arr["attn_ref_fp32"]))
    assert torch.equal(ym.cpu(), torch.from_numpy(arr["y_mask_ref_fp32"]))
    assert torch.equal(ymean.cpu(), torch.from_numpy(arr["y_mean_ref_fp32"]))
    assert torch.equal(yls.cpu(), torch.zeros(B, C, Ty))
    assert max_abs(z.cpu().numpy(), arr["z_ref_fp32"]) <= 1e-6


@pytest.mark.parametrize("name,meta,arr", GTTS, ids=[g[0] for g in GTTS])
def test_glow_tts_inference_end_to_end(cuda_device, name, meta, arr):
    """tokens -> GlowTTS.inference -> mel, with the fixture's sampling noise."""
    m = build_glow_tts(meta, cuda_device)
    tok = torch.from_numpy(arr["tokens"])
    aux = {"x_lengths": torch.from_numpy(arr["lengths"]), "noise": torch.from_numpy(arr["noise"])}
    if "d_vectors" in arr:
        aux["d_vectors"] = torch.from_numpy(arr["d_vectors"])
    out = m.inference(tok, aux)
    # durations are ceil()-quantised: the fixture keeps every w >= 1.8e-2 away from an integer
    # (meta ceil_margin), so the fp32 encoder must reproduce the reference alignment exactly
    assert torch.equal(out["alignments"].cpu(), torch.from_numpy(arr["attn_ref_fp64"]).permute(0, 2, 1).float())
    mel = out["model_outputs"].transpose(1, 2)
    assert_close_fp32(mel.cpu(), arr["mel_ref_fp64"], f"{name} mel", MEL_MAX_ABS, MEL_REL_RMS)
    assert_close_fp32(out["durations_log"].transpose(1, 2).cpu(), arr["logw_ref_fp64"], "durations_log",
                      ENC_MAX_ABS, ENC_REL_RMS)
    np.testing.assert_allclose(out["total_durations_log"].transpose(1, 2).cpu().numpy(),
                               arr["o_attn_dur_ref_fp64"], rtol=0, atol=1e-6)
    assert out["logdet"] is None


def test_glow_tts_batch_invariance_and_determinism(cuda_device):
    """Config-3 shape (16 utterances x 128 tokens).  A full-length utterance alone gives bit-identical
    durations and mel (the batch's longest y_length only pads), and two runs are bitwise equal.
    A ragged utterance is NOT batch-invariant in the reference itself: its padded tokens keep
    duration 1 (clamp_min after the mask, glow_tts.py:351) and extend its y_length with z = 0
    frames, so it is checked against the oracle chain run on the same padded batch row."""
    meta = dict(encoder=dict(GLOW_TTS_ENCODER, num_chars=64), eseed=5, dseed=6, noise_scale=0.0, length_scale=1.0,
                decoder=dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=12,
                             num_coupling_layers=4, num_splits=4, num_squeeze=2))
    m = build_glow_tts(meta, cuda_device)
    tok = synthetic.tokens(16, 128, 64, seed=3)
    lens = torch.full((16,), 128, dtype=torch.int64)
    lens[5] = 77
    a = m.inference(tok, {"x_lengths": lens})
    b = m.inference(tok, {"x_lengths": lens})
    assert torch.equal(a["model_outputs"], b["model_outputs"])
    assert torch.isfinite(a["model_outputs"]).all()
    one = m.inference(tok[3:4], {"x_lengths": lens[3:4]})
    T1 = one["model_outputs"].shape[1]
    assert torch.equal(a["alignments"][3, :T1], one["alignments"][0])
    assert torch.equal(a["model_outputs"][3, :T1], one["model_outputs"][0])
    # ragged row 5 against the oracle chain (fp64) on the same padded row
    esd = synthetic.glow_encoder_state_dict(**meta["encoder"], seed=5)
    xm_, _, logw, xmask = glow_tts_ref.encoder_forward(esd, tok[5:6], lens[5:6])
    w_ceil, ylen = glow_tts_ref.durations(logw, xmask)
    z, ymask, *_ = glow_tts_ref.expand(w_ceil, xmask, ylen, xm_, torch.zeros_like(xm_))
    dsd = synthetic.glow_decoder_state_dict(**meta["decoder"], seed=6)
    mel = glow_ref.glow_decoder_reverse(dsd, z, ymask, **meta["decoder"])
    T5 = mel.shape[2]
    assert_close_fp32(a["model_outputs"][5, :T5].transpose(0, 1).cpu(), mel[0], "ragged row 5", MEL_MAX_ABS,
                      MEL_REL_RMS)


def test_multispeaker_speaker_ids_vs_oracle(cuda_device):
    """use_speaker_embedding (glow_tts.py:129-133): g = F.normalize(emb_g(speaker_ids)) of width
    hidden_channels_enc conditions the duration predictor and the 12 flows; each utterance against
    the oracle chain (fp64) with its own speaker vector, and a speaker swap changes durations and mel."""
    H = GLOW_TTS_ENCODER["hidden_channels"]
    ecfg = dict(GLOW_TTS_ENCODER, num_chars=64, c_in_channels=H)
    dcfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=12,
                num_coupling_layers=4, num_splits=4, num_squeeze=2, c_in_channels=H)
    emb = torch.rand(5, H, generator=torch.Generator().manual_seed(9)) * 0.2 - 0.1
    meta = dict(encoder=ecfg, decoder=dcfg, eseed=21, dseed=22, noise_scale=0.0, length_scale=1.0, emb_g=emb)
    m = build_glow_tts(meta, cuda_device, use_speaker_embedding=True, num_speakers=5)
    assert m.c_in_channels == H and m.encoder.c_in_channels == H and m.decoder.c_in_channels == H
    tok = synthetic.tokens(3, 31, 64, seed=12)
    lens = torch.tensor([31, 25, 9])
    sid = torch.tensor([4, 0, 2])
    out = m.inference(tok, {"x_lengths": lens, "speaker_ids": sid})
    esd = synthetic.glow_encoder_state_dict(**ecfg, seed=21)
    dsd = synthetic.glow_decoder_state_dict(**dcfg, seed=22)
    g = torch.nn.functional.normalize(emb[sid].double()).unsqueeze(-1)
    for b in range(3):
        xm_, _, logw, xmask = glow_tts_ref.encoder_forward(esd, tok[b:b + 1], lens[b:b + 1], g=g[b:b + 1])
        w_ceil, ylen = glow_tts_ref.durations(logw, xmask)
        z, ymask, *_ = glow_tts_ref.expand(w_ceil, xmask, ylen, xm_, torch.zeros_like(xm_))
        mel = glow_ref.glow_decoder_reverse(dsd, z, ymask, g=g[b:b + 1], **dcfg)
        Tb = mel.shape[2]
        assert_close_fp32(out["durations_log"][b, :lens[b]].transpose(0, 1).cpu(), logw[0, :, :lens[b]],
                          f"logw spk {int(sid[b])}", ENC_MAX_ABS, ENC_REL_RMS)
        assert_close_fp32(out["model_outputs"][b, :Tb].transpose(0, 1).cpu(), mel[0], f"mel spk {int(sid[b])}",
                          MEL_MAX_ABS, MEL_REL_RMS)
    other = m.inference(tok, {"x_lengths": lens, "speaker_ids": torch.tensor([1, 3, 0])})
    assert not torch.equal(other["durations_log"], out["durations_log"])
    with pytest.raises(ValueError):
        m.inference(tok, {"x_lengths": lens})
    with pytest.raises(ValueError):
        m.inference(tok, {"x_lengths": lens, "speaker_ids": sid, "d_vectors": torch.zeros(3, H)})


@pytest.mark.parametrize("mode", ["fp32", "f16x3"])
def test_decoder_inference_vs_oracle(cuda_device, mode):
    """GlowTTS.decoder_inference (glow_tts.py:319-339): decoder forward (mel -> z) then reverse, on
    device, against the fp64 oracle chain; the forward-reverse pair returns the mel on the frames
    the squeeze keeps."""
    name, meta, arr = goldens("glow_tts")[0]
    m = build_glow_tts(meta, cuda_device, decoder_math_mode=mode)
    gen = torch.Generator().manual_seed(13)
    B, T = 3, 91
    y = torch.randn(B, T, 80, generator=gen)
    lengths = torch.tensor([91, 60, 2])
    out = m.decoder_inference(y.to(cuda_device), lengths.to(cuda_device))
    assert out["logdet"] is None
    yo = out["model_outputs"].cpu()
    T2 = yo.shape[1]
    dcfg = meta["decoder"]
    sd = synthetic.glow_decoder_state_dict(**dcfg, seed=meta["dseed"])
    mask = (torch.arange(T)[None] < lengths[:, None]).float().unsqueeze(1)
    z, _ = glow_ref.glow_decoder_forward(sd, y.transpose(1, 2), mask, **dcfg)
    ref = glow_ref.glow_decoder_reverse(sd, z, mask[:, :, :T2], **dcfg)
    assert_close_fp32(yo.transpose(1, 2), ref, f"decoder_inference ({mode})", MEL_MAX_ABS, MEL_REL_RMS)
    keep = mask[:, :, 1:T2:2].repeat_interleave(2, dim=2)
    assert max_abs((yo.transpose(1, 2) * keep).numpy(), (y.transpose(1, 2)[:, :, :T2] * keep).numpy()) < 1e-4
