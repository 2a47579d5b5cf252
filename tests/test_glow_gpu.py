"""Glow-TTS decoder (reverse flow) parity on MI355X vs the reference goldens and the oracle."""
import numpy as np
import pytest
import torch

from _util import BF16_MAX_ABS, BF16_REL_RMS, assert_close_fp32, goldens, max_abs
from oracle import glow_ref
from tts_amd import synthetic
from tts_amd.tts import Decoder

pytestmark = pytest.mark.gpu
GLOW = goldens("glow")
# the reference's own fp32-vs-fp64 error on this flow is 2.9e-6 (12 flows, exp() of scales)
# (max); measured on MI355X: max 4.7e-6, rel-RMS 3.5e-7 (profiles/parity_errors_r03.jsonl)
GLOW_MAX_ABS = 5e-5
GLOW_REL_RMS = 5e-6


def build(cfg, seed, device, math_mode="fp32"):
    d = Decoder(cfg["in_channels"], cfg["hidden_channels"], cfg["kernel_size"], cfg["dilation_rate"],
                cfg["num_flow_blocks"], cfg["num_coupling_layers"], dropout_p=0.05,
                num_splits=cfg["num_splits"], num_squeeze=cfg["num_squeeze"],
                c_in_channels=cfg.get("c_in_channels", 0), math_mode=math_mode)
    d.load_state_dict(synthetic.glow_decoder_state_dict(**cfg, seed=seed))
    d.eval()
    d.store_inverse()
    return d.to(device)


@pytest.mark.parametrize("mode", ["fp32", "fp32x6", "f16x3", "bf16"])
@pytest.mark.parametrize("name,meta,arr", GLOW, ids=[g[0] for g in GLOW])
def test_glow_reverse_vs_reference(cuda_device, name, meta, arr, mode):
    d = build(meta["config"], meta["seed"], cuda_device, mode)
    x = torch.from_numpy(arr["x"]).to(cuda_device)
    m = torch.from_numpy(arr["mask"]).to(cuda_device)
    g = torch.from_numpy(arr["g"]).to(cuda_device) if "g" in arr else None  # multi-speaker (c_in > 0)
    y, logdet = d(x, m, g=g, reverse=True)
    assert logdet is None
    if mode == "bf16":
        assert_close_fp32(y.cpu(), arr["out_ref_fp64"], name, BF16_MAX_ABS, BF16_REL_RMS)
    else:
        assert_close_fp32(y.cpu(), arr["out_ref_fp64"], name, GLOW_MAX_ABS, GLOW_REL_RMS)


@pytest.mark.parametrize("mode", ["fp32", "f16x3"])
@pytest.mark.parametrize("B,T,lengths", [(1, 2, [2]), (2, 7, [7, 3]), (4, 400, [400, 399, 200, 1])])
def test_glow_reverse_vs_oracle(cuda_device, B, T, lengths, mode):
    cfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=12,
               num_coupling_layers=4, num_splits=4, num_squeeze=2)
    d = build(cfg, 99, cuda_device, mode)
    g = torch.Generator().manual_seed(T)
    x = torch.randn(B, 80, T, generator=g)
    m = (torch.arange(T)[None] < torch.tensor(lengths)[:, None]).float().unsqueeze(1)
    y, _ = d(x.to(cuda_device), m.to(cuda_device), reverse=True)
    ref = glow_ref.glow_decoder_reverse(synthetic.glow_decoder_state_dict(**cfg, seed=99), x, m, **cfg)
    assert_close_fp32(y.cpu(), ref, f"glow B={B} T={T}", GLOW_MAX_ABS, GLOW_REL_RMS)


@pytest.mark.parametrize("mode", ["fp32", "f16x3"])
def test_glow_batch_invariance(cuda_device, mode):
    cfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=12,
               num_coupling_layers=4, num_splits=4, num_squeeze=2)
    d = build(cfg, 5, cuda_device, mode)
    x = torch.randn(16, 80, 768, generator=torch.Generator().manual_seed(1)).to(cuda_device)
    m = torch.ones(16, 1, 768, device=cuda_device)
    y, _ = d(x, m, reverse=True)
    y1, _ = d(x[3:4], m[3:4], reverse=True)
    assert torch.equal(y[3], y1[0])
    y2, _ = d(x, m, reverse=True)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("mode", ["fp32x6", "f16x3", "bf16"])
def test_glow_gate_fusion_bitwise(cuda_device, mode, monkeypatch):
    """The WN gate fused into the in_layer conv epilogue (kSplitGateTile) computes the same fp32
    operations as the separate gate kernel: bitwise equal outputs, ragged mask included."""
    cfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=3,
               num_coupling_layers=4, num_splits=4, num_squeeze=2)
    g = torch.Generator().manual_seed(17)
    x = torch.randn(3, 80, 301, generator=g).to(cuda_device)
    m = (torch.arange(301)[None] < torch.tensor([301, 150, 9])[:, None]).float().unsqueeze(1).to(cuda_device)
    outs, names = [], []
    monkeypatch.setenv("TTS_MI355X_WN_LAYER", "0")  # the per-conv launches (the one-launch layer is below)
    for fused in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_FLOW_GATE", fused)
        d = build(cfg, 23, cuda_device, mode)
        outs.append(d(x, m, reverse=True)[0])
        names.append({r["name"] for r in d.profile(x, m)[1]})
    assert "glow_wn_in_gate" in names[0] and "glow_gate" not in names[0]
    assert "glow_gate" in names[1] and "glow_wn_in_gate" not in names[1]
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("mode", ["fp32x6", "f16x3", "bf16"])
@pytest.mark.parametrize("reverse", [True, False])
def test_glow_wn_update_fusion_bitwise(cuda_device, mode, reverse, monkeypatch):
    """The WN residual / skip update inside the res_skip conv epilogue (Conv1dArgs::wn_rows, every
    layer but the last) computes glow_wn_update_kernel's fp32 operations in the same order: bitwise
    equal outputs (and logdet) with and without it, ragged mask included."""
    cfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=3,
               num_coupling_layers=4, num_splits=4, num_squeeze=2)
    g = torch.Generator().manual_seed(19)
    x = torch.randn(3, 80, 301, generator=g).to(cuda_device)
    m = (torch.arange(301)[None] < torch.tensor([301, 150, 9])[:, None]).float().unsqueeze(1).to(cuda_device)
    outs, names = [], []
    monkeypatch.setenv("TTS_MI355X_WN_LAYER", "0")
    for fused in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_WN_FUSION", fused)
        d = build(cfg, 23, cuda_device, mode)
        outs.append(d(x, m, reverse=reverse))
        names.append([r["name"] for r in d.profile(x, m)[1]])
    assert names[0].count("glow_wn_res_skip_update") == 3 * 3 and names[0].count("glow_wn_update") == 3
    assert names[1].count("glow_wn_update") == 3 * 4
    assert torch.equal(outs[0][0], outs[1][0])
    if not reverse:
        assert torch.equal(outs[0][1], outs[1][1])


def test_glow_x0_statistics_match_prepass(cuda_device, monkeypatch):
    """f16x3: every flow's x0 max-abs published by the previous flow's tail kernel equals the
    strided pre-pass it replaced (TTS_MI355X_FLOW_AMAX_PREPASS=1): bitwise equal outputs, ragged
    masks included.  An under-reported max would overflow fp16 and show up here first."""
    cfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=4,
               num_coupling_layers=4, num_splits=4, num_squeeze=2)
    g = torch.Generator().manual_seed(29)
    x = (torch.randn(3, 80, 257, generator=g) * 3).to(cuda_device)
    m = (torch.arange(257)[None] < torch.tensor([257, 120, 7])[:, None]).float().unsqueeze(1).to(cuda_device)
    outs, names = [], []
    for prepass in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_FLOW_AMAX_PREPASS", prepass)
        d = build(cfg, 41, cuda_device, "f16x3")
        outs.append(d(x, m, reverse=True)[0])
        names.append([r["name"] for r in d.profile(x, m)[1]])
    assert names[0].count("glow_amax_x0") == 4 and names[1].count("glow_amax_x0") == 1
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("mode", ["fp32", "fp32x6", "f16x3", "bf16"])
def test_glow_speaker_conditioned_vs_oracle(cuda_device, mode):
    """Multi-speaker decoder (c_in_channels > 0, decoder.py:113 with g): every flow's WN projects g
    with its cond_layer and adds rows [2Hl, 2H(l+1)) to in_layer l (wavenet.py:98-107).  Longer and
    ragged against the fp64 oracle; the same utterance alone is bit-identical (batch invariance)."""
    cfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=12,
               num_coupling_layers=4, num_splits=4, num_squeeze=2, c_in_channels=256)
    d = build(cfg, 57, cuda_device, mode)
    gen = torch.Generator().manual_seed(58)
    B, T = 4, 301
    x = torch.randn(B, 80, T, generator=gen)
    g = torch.randn(B, 256, 1, generator=gen)
    m = (torch.arange(T)[None] < torch.tensor([301, 300, 128, 3])[:, None]).float().unsqueeze(1)
    y, _ = d(x.to(cuda_device), m.to(cuda_device), g=g.to(cuda_device), reverse=True)
    ref = glow_ref.glow_decoder_reverse(synthetic.glow_decoder_state_dict(**cfg, seed=57), x, m, g=g, **cfg)
    if mode == "bf16":
        assert_close_fp32(y.cpu(), ref, "glow cond (bf16)", BF16_MAX_ABS, BF16_REL_RMS)
    else:
        assert_close_fp32(y.cpu(), ref, f"glow cond ({mode})", GLOW_MAX_ABS, GLOW_REL_RMS)
    y2, _ = d(x[2:3].to(cuda_device), m[2:3].to(cuda_device), g=g[2:3].to(cuda_device), reverse=True)
    assert torch.equal(y2[0], y[2])
    with pytest.raises(ValueError):
        d(x.to(cuda_device), m.to(cuda_device), reverse=True)  # conditioned decoder without g


@pytest.mark.parametrize("mode", ["fp32x6", "f16x3"])
def test_glow_speaker_gate_fusion_bitwise(cuda_device, mode, monkeypatch):
    """The speaker term g_l rides in the fused gate epilogue (cvec, original row order) exactly as in
    the separate in_layer + gate launches."""
    cfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=2,
               num_coupling_layers=4, num_splits=4, num_squeeze=2, c_in_channels=16)
    gen = torch.Generator().manual_seed(19)
    x = torch.randn(2, 80, 211, generator=gen).to(cuda_device)
    g = torch.randn(2, 16, 1, generator=gen).to(cuda_device)
    m = (torch.arange(211)[None] < torch.tensor([211, 90])[:, None]).float().unsqueeze(1).to(cuda_device)
    outs = []
    monkeypatch.setenv("TTS_MI355X_WN_LAYER", "0")
    for fused in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_FLOW_GATE", fused)
        outs.append(build(cfg, 29, cuda_device, mode)(x, m, g=g, reverse=True)[0])
    assert torch.equal(outs[0], outs[1])


WN_LAYER_CFGS = {
    "ljspeech": dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=3,
                     num_coupling_layers=4, num_splits=4, num_squeeze=2),
    "spk_c16": dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=2,
                    num_coupling_layers=4, num_splits=4, num_squeeze=2, c_in_channels=16),
    "h128_k3_dil2": dict(in_channels=40, hidden_channels=128, kernel_size=3, dilation_rate=2, num_flow_blocks=2,
                         num_coupling_layers=4, num_splits=4, num_squeeze=2),
    "h256_l1": dict(in_channels=40, hidden_channels=256, kernel_size=5, dilation_rate=1, num_flow_blocks=2,
                    num_coupling_layers=1, num_splits=2, num_squeeze=1),
}


@pytest.mark.parametrize("mode", ["fp32x6", "f16x3", "bf16"])
@pytest.mark.parametrize("reverse", [True, False])
@pytest.mark.parametrize("cname", list(WN_LAYER_CFGS))
def test_glow_wn_layer_matches_unfused(cuda_device, mode, reverse, cname, monkeypatch):
    """One launch per WaveNet layer (kernels_glow_wn.hip: in_layer -> cond -> gate -> res_skip ->
    update with xin / acts / rs in LDS) against the four launches per layer: the same fp32
    operations in the same order, so bf16 is bitwise equal (outputs and logdet); in f16x3 the acts
    operand takes the fixed exponent of |acts| < 1 instead of its per-utterance one (equal whenever
    max |acts| >= 0.5; bitwise on these inputs in scripts/wn_debug.py), and bf16x6 differs in the
    last bit of ~10% of the outputs (cause not isolated), so those two are held to the
    fp32-faithful tolerance.
    Ragged masks (tile edges at 32 columns, a 9-frame item), speaker cond, K 3 / 5, dilations
    1-8, H 128 / 192 / 256, a single-layer WN (first = last)."""
    cfg = WN_LAYER_CFGS[cname]
    C, T = cfg["in_channels"], 301
    gen = torch.Generator().manual_seed(31)
    x = torch.randn(3, C, T, generator=gen).to(cuda_device)
    m = (torch.arange(T)[None] < torch.tensor([301, 150, 9])[:, None]).float().unsqueeze(1).to(cuda_device)
    c_in = cfg.get("c_in_channels", 0)
    g = torch.randn(3, c_in, 1, generator=gen).to(cuda_device) if c_in else None
    outs, names = [], []
    for on in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_WN_LAYER", on)
        d = build(cfg, 23, cuda_device, mode)
        outs.append(d(x, m, g=g, reverse=reverse))
        names.append([r["name"] for r in d.profile(x, m, g=g)[1]])
    L, NF = cfg["num_coupling_layers"], cfg["num_flow_blocks"]
    assert names[0].count("glow_wn_layer") == NF * L and "glow_gate" not in names[0]
    # the coupling's end conv rides in the last layer's launch when C2 is whole 32-row blocks
    C2 = cfg["in_channels"] * cfg["num_squeeze"]
    assert names[0].count("glow_end") == (0 if C2 % 32 == 0 and C2 <= 2 * cfg["hidden_channels"] else NF)
    assert names[1].count("glow_gate") == NF * L and "glow_wn_layer" not in names[1]
    if mode != "bf16":
        assert_close_fp32(outs[0][0].cpu(), outs[1][0].cpu().double().numpy(), f"wn layer {cname} {mode}",
                          GLOW_MAX_ABS, GLOW_REL_RMS)
        if not reverse:
            ld0, ld1 = outs[0][1].cpu().double(), outs[1][1].cpu().double()
            assert (ld0 - ld1).abs().max() <= 1e-5 * max(1.0, ld1.abs().max().item())
    else:
        assert torch.equal(outs[0][0], outs[1][0])
        if not reverse:
            assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("mode", ["fp32x6", "f16x3", "bf16"])
def test_glow_wn_end_fusion(cuda_device, mode, monkeypatch):
    """The end conv inside the last WN layer's launch (TTS_MI355X_WN_END) against its own launch:
    bitwise in bf16 (same operations and order), the fp32-faithful tolerance otherwise (f16x3: the
    tile's max-abs exponent instead of the utterance's); both directions, logdet included."""
    cfg = WN_LAYER_CFGS["ljspeech"]
    gen = torch.Generator().manual_seed(37)
    x = torch.randn(3, 80, 301, generator=gen).to(cuda_device)
    m = (torch.arange(301)[None] < torch.tensor([301, 150, 9])[:, None]).float().unsqueeze(1).to(cuda_device)
    outs = {}
    for on in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_WN_END", on)
        d = build(cfg, 43, cuda_device, mode)
        outs[on] = (d(x, m, reverse=True)[0], d(x, m, reverse=False))
        names = [r["name"] for r in d.profile(x, m)[1]]
        assert names.count("glow_end") == (0 if on == "1" else cfg["num_flow_blocks"])
    (r1, (f1, l1)), (r0, (f0, l0)) = outs["1"], outs["0"]
    if mode == "bf16":
        assert torch.equal(r1, r0) and torch.equal(f1, f0) and torch.equal(l1, l0)
    else:
        assert_close_fp32(r1.cpu(), r0.cpu().double().numpy(), f"wn end {mode}", GLOW_MAX_ABS, GLOW_REL_RMS)
        assert_close_fp32(f1.cpu(), f0.cpu().double().numpy(), f"wn end fwd {mode}", GLOW_MAX_ABS, GLOW_REL_RMS)
        assert (l1 - l0).abs().max().item() <= 1e-5 * max(1.0, l0.abs().max().item())


@pytest.mark.parametrize("mode", ["fp32x6", "f16x3", "bf16"])
@pytest.mark.parametrize("cname", ["ljspeech", "spk_c16"])
def test_glow_wn_tail_fusion(cuda_device, mode, cname, monkeypatch):
    """Reverse flows: the inverse tail (coupling, InvConvNear, ActNorm) and the next flow's start conv
    inside the last WN layer's launch (TTS_MI355X_WN_TAIL) against their own launches: bitwise in
    bf16; the fp32-faithful tolerance otherwise (f16x3: the start operand's tile exponent); the last
    flow keeps its tail launch and the first its start launch."""
    cfg = WN_LAYER_CFGS[cname]
    NF = cfg["num_flow_blocks"]
    gen = torch.Generator().manual_seed(41)
    x = torch.randn(3, 80, 301, generator=gen).to(cuda_device)
    m = (torch.arange(301)[None] < torch.tensor([301, 150, 9])[:, None]).float().unsqueeze(1).to(cuda_device)
    c_in = cfg.get("c_in_channels", 0)
    g = torch.randn(3, c_in, 1, generator=gen).to(cuda_device) if c_in else None
    outs = {}
    for on in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_WN_TAIL", on)
        d = build(cfg, 47, cuda_device, mode)
        outs[on] = d(x, m, g=g, reverse=True)[0]
        names = [r["name"] for r in d.profile(x, m, g=g)[1]]
        assert names.count("glow_tail") == (1 if on == "1" else NF)
        assert names.count("glow_start") == (1 if on == "1" else NF)
    if mode == "bf16":
        assert torch.equal(outs["1"], outs["0"])
    else:
        assert_close_fp32(outs["1"].cpu(), outs["0"].cpu().double().numpy(), f"wn tail {cname} {mode}",
                          GLOW_MAX_ABS, GLOW_REL_RMS)


@pytest.mark.parametrize("mode", ["f16x3", "bf16"])
def test_glow_wn_tail_sigmoid_scale(cuda_device, mode, monkeypatch):
    """sigmoid_scale=True (glow.py:222-223: s = log(1e-6 + sigmoid(s + 2))) through the fused tail:
    bitwise in bf16 against the tail launch, and against the fp64 oracle."""
    cfg = WN_LAYER_CFGS["ljspeech"]
    sd = synthetic.glow_decoder_state_dict(**cfg, seed=53)
    gen = torch.Generator().manual_seed(54)
    x = torch.randn(2, 80, 203, generator=gen)
    m = (torch.arange(203)[None] < torch.tensor([203, 77])[:, None]).float().unsqueeze(1)
    outs = {}
    for on in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_WN_TAIL", on)
        d = Decoder(cfg["in_channels"], cfg["hidden_channels"], cfg["kernel_size"], cfg["dilation_rate"],
                    cfg["num_flow_blocks"], cfg["num_coupling_layers"], dropout_p=0.05,
                    num_splits=cfg["num_splits"], num_squeeze=cfg["num_squeeze"], sigmoid_scale=True,
                    math_mode=mode)
        d.load_state_dict(sd)
        d.eval()
        d.store_inverse()
        d = d.to(cuda_device)
        outs[on] = d(x.to(cuda_device), m.to(cuda_device), reverse=True)[0]
    ref = glow_ref.glow_decoder_reverse(sd, x, m, sigmoid_scale=True, **cfg)
    if mode == "bf16":
        assert torch.equal(outs["1"], outs["0"])
        assert_close_fp32(outs["1"].cpu(), ref, "wn tail sigmoid_scale (bf16)", BF16_MAX_ABS, BF16_REL_RMS)
    else:
        assert_close_fp32(outs["1"].cpu(), ref, "wn tail sigmoid_scale (f16x3)", GLOW_MAX_ABS, GLOW_REL_RMS)


@pytest.mark.parametrize("mode", ["f16x3", "bf16"])
def test_glow_wn_layer_other_shapes_vs_oracle(cuda_device, mode):
    """The one-launch WN layer at H 128 (kernel 3, dilations 1, 2, 4, 8) against the fp64 oracle."""
    cfg = WN_LAYER_CFGS["h128_k3_dil2"]
    d = build(cfg, 61, cuda_device, mode)
    gen = torch.Generator().manual_seed(62)
    B, T = 3, 203
    x = torch.randn(B, cfg["in_channels"], T, generator=gen)
    m = (torch.arange(T)[None] < torch.tensor([203, 64, 33])[:, None]).float().unsqueeze(1)
    y, _ = d(x.to(cuda_device), m.to(cuda_device), reverse=True)
    assert "glow_wn_layer" in {r["name"] for r in d.profile(x.to(cuda_device), m.to(cuda_device))[1]}
    ref = glow_ref.glow_decoder_reverse(synthetic.glow_decoder_state_dict(**cfg, seed=61), x, m, **cfg)
    if mode == "bf16":
        assert_close_fp32(y.cpu(), ref, "glow h128 (bf16)", BF16_MAX_ABS, BF16_REL_RMS)
    else:
        assert_close_fp32(y.cpu(), ref, "glow h128 (f16x3)", GLOW_MAX_ABS, GLOW_REL_RMS)


# ----------------------------------------------------------------------------- forward direction
@pytest.mark.parametrize("mode", ["fp32", "fp32x6", "f16x3", "bf16"])
@pytest.mark.parametrize("name,meta,arr", GLOW, ids=[g[0] for g in GLOW])
def test_glow_forward_vs_reference(cuda_device, name, meta, arr, mode):
    """reverse=False (GlowTTS.decoder_inference's first pass, glow_tts.py:333): the reference's own
    forward output on its fp64 reverse output (the fixture's roundtrip_fp64 / logdet_fp64)."""
    d = build(meta["config"], meta["seed"], cuda_device, mode)
    y = torch.from_numpy(arr["out_ref_fp64"]).float()
    m = torch.from_numpy(arr["mask"])[:, :, : y.shape[2]]
    g = torch.from_numpy(arr["g"]).to(cuda_device) if "g" in arr else None
    z, logdet = d(y.to(cuda_device), m.to(cuda_device), g=g, reverse=False)
    assert z.shape == arr["roundtrip_fp64"].shape and logdet.shape == (y.shape[0],)
    ref_ld = arr["logdet_fp64"]
    if mode == "bf16":
        assert_close_fp32(z.cpu(), arr["roundtrip_fp64"], f"{name} forward", BF16_MAX_ABS, BF16_REL_RMS)
        assert np.abs(logdet.cpu().numpy() - ref_ld).max() <= 3e-2 * max(1.0, np.abs(ref_ld).max())
    else:
        assert_close_fp32(z.cpu(), arr["roundtrip_fp64"], f"{name} forward", GLOW_MAX_ABS, GLOW_REL_RMS)
        # logdet sums ~1e3 terms per utterance: 1e-5 relative of its magnitude
        assert np.abs(logdet.cpu().numpy() - ref_ld).max() <= 1e-5 * max(1.0, np.abs(ref_ld).max()), (logdet, ref_ld)


@pytest.mark.parametrize("mode", ["fp32", "f16x3"])
@pytest.mark.parametrize("B,T,lengths", [(1, 2, [2]), (3, 65, [65, 30, 1]), (2, 400, [400, 223])])
def test_glow_forward_vs_oracle_and_roundtrip(cuda_device, B, T, lengths, mode):
    """Forward against the fp64 oracle (z and logdet) on ragged masks, and forward o reverse = id
    on the kept frames (decoder.py:25: frame pair (2t, 2t+1) survives iff mask[2t+1])."""
    cfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=12,
               num_coupling_layers=4, num_splits=4, num_squeeze=2)
    d = build(cfg, 98, cuda_device, mode)
    gen = torch.Generator().manual_seed(T + 1)
    x = torch.randn(B, 80, T, generator=gen)
    m = (torch.arange(T)[None] < torch.tensor(lengths)[:, None]).float().unsqueeze(1)
    z, logdet = d(x.to(cuda_device), m.to(cuda_device), reverse=False)
    zr, ldr = glow_ref.glow_decoder_forward(synthetic.glow_decoder_state_dict(**cfg, seed=98), x, m, **cfg)
    assert_close_fp32(z.cpu(), zr, f"glow forward B={B} T={T}", GLOW_MAX_ABS, GLOW_REL_RMS)
    assert np.abs(logdet.cpu().double().numpy() - ldr.numpy()).max() <= 1e-5 * max(1.0, ldr.abs().max().item())
    T2 = z.shape[2]
    y, _ = d(z, m[:, :, :T2].to(cuda_device), reverse=True)
    keep = m[:, :, 1:T2:2].repeat_interleave(2, dim=2)
    assert max_abs((y.cpu() * keep).numpy(), (x[:, :, :T2] * keep).numpy()) < 1e-4


def test_glow_forward_deterministic_and_batch_invariant(cuda_device):
    cfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=12,
               num_coupling_layers=4, num_splits=4, num_squeeze=2)
    d = build(cfg, 97, cuda_device, "f16x3")
    x = torch.randn(4, 80, 301, generator=torch.Generator().manual_seed(4)).to(cuda_device)
    m = torch.ones(4, 1, 301, device=cuda_device)
    z, ld = d(x, m, reverse=False)
    z2, ld2 = d(x, m, reverse=False)
    assert torch.equal(z, z2) and torch.equal(ld, ld2)
    z1, ld1 = d(x[2:3], m[2:3], reverse=False)
    assert torch.equal(z1[0], z[2]) and torch.equal(ld1[0], ld[2])
