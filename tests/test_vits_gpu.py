"""VITS reverse flow (ResidualCouplingBlocks, networks.py:169-232) on MI355X through the C-ABI,
against the reference's own fp64 output (golden fixtures) and the CPU oracle; plus the VITS
waveform path of config 5: flow -> z * mask -> HiFiGAN decoder (in 192, cond, no conv_post
bias, no padding; vits.py:1156-1162)."""
import numpy as np
import pytest
import torch

from _util import assert_close_fp32, goldens, tol
from oracle import hifigan_ref, vits_ref
from tts_amd import synthetic
from tts_amd.config import VITS_DECODER, VITS_FLOW
from tts_amd.tts import PosteriorEncoder, ResidualCouplingBlocks
from tts_amd.vocoder import HifiganGenerator

pytestmark = pytest.mark.gpu

VITS = goldens("vits_flow")
MODES = ["fp32", "fp32x6", "f16x3", "bf16"]


def build(cfg, seed, device, math_mode="fp32"):
    f = ResidualCouplingBlocks(cfg["channels"], cfg["hidden_channels"], cfg["kernel_size"], cfg["dilation_rate"],
                               cfg["num_layers"], num_flows=cfg["num_flows"], cond_channels=cfg["cond_channels"],
                               math_mode=math_mode)
    sd = synthetic.vits_flow_state_dict(**cfg, seed=seed)
    f.load_state_dict(sd)
    return f.to(device), sd


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("name,meta,arr", VITS, ids=[g[0] for g in VITS])
def test_vits_flow_vs_reference(cuda_device, name, meta, arr, mode):
    f, _ = build(meta["config"], meta["seed"], cuda_device, mode)
    g = torch.from_numpy(arr["g"]).to(cuda_device) if "g" in arr else None
    y = f(torch.from_numpy(arr["x"]).to(cuda_device), torch.from_numpy(arr["mask"]).to(cuda_device), g=g, reverse=True)
    assert_close_fp32(y.cpu(), arr["out_ref_fp64"], f"{name} ({mode})", **tol(mode))


@pytest.mark.parametrize("cond", [0, 4])
def test_vits_flow_vs_oracle_other_shapes(cuda_device, cond):
    cfg = dict(VITS_FLOW, channels=64, hidden_channels=96, num_layers=3, num_flows=3, dilation_rate=2,
               cond_channels=cond)
    f, sd = build(cfg, 11 + cond, cuda_device)
    gen = torch.Generator().manual_seed(5)
    B, T = 3, 77
    x = torch.randn(B, 64, T, generator=gen)
    mask = (torch.arange(T)[None, :] < torch.tensor([77, 40, 3])[:, None]).float().unsqueeze(1)
    g = torch.randn(B, cond, 1, generator=gen) if cond else None
    ref = vits_ref.vits_flow_reverse(sd, x, mask, g, dtype=torch.float64, **cfg)
    y = f(x.to(cuda_device), mask.to(cuda_device), g=g.to(cuda_device) if g is not None else None, reverse=True)
    assert_close_fp32(y.cpu(), ref, f"vits flow cond={cond}")


def test_vits_flow_batch_invariance_and_profile(cuda_device):
    name, meta, arr = VITS[0]
    f, _ = build(meta["config"], meta["seed"], cuda_device)
    x = torch.from_numpy(arr["x"]).to(cuda_device)
    m = torch.from_numpy(arr["mask"]).to(cuda_device)
    y = f(x, m, reverse=True)
    for i in range(x.shape[0]):
        assert torch.equal(f(x[i : i + 1], m[i : i + 1], reverse=True)[0], y[i])
    y2, rows = f.profile(x, m)
    assert torch.equal(y2, y)
    assert len(rows) == 4 * (2 + 4 * 4)  # pre, post, 4 x (in, gate, res_skip, update) per flow
    assert all(r["ms"] > 0 for r in rows)


@pytest.mark.parametrize("mode", ["fp32", "fp32x6", "f16x3", "bf16"])
def test_vits_waveform_path(cuda_device, mode):
    """z = flow(z_p, mask, g, reverse); wav = decoder((z * mask), g)  (vits.py:1156-1162)."""
    cond = 8
    fcfg = dict(VITS_FLOW, cond_channels=cond)
    flow, fsd = build(fcfg, 2469, cuda_device, mode)
    dcfg = dict(VITS_DECODER, upsample_initial_channel=128, cond_channels=cond)
    dsd = synthetic.hifigan_state_dict(**dcfg, seed=99, weight_norm=False)
    dec = HifiganGenerator(**dcfg, math_mode=mode)
    dec.remove_weight_norm()
    dec.load_state_dict(dsd)
    dec = dec.to(cuda_device)
    gen = torch.Generator().manual_seed(9)
    B, T = 2, 24
    zp = torch.randn(B, 192, T, generator=gen)
    mask = (torch.arange(T)[None, :] < torch.tensor([24, 13])[:, None]).float().unsqueeze(1)
    g = torch.randn(B, cond, 1, generator=gen)
    z = flow(zp.to(cuda_device), mask.to(cuda_device), g=g.to(cuda_device), reverse=True)
    wav = dec(z * mask.to(cuda_device), g=g.to(cuda_device))
    zr = vits_ref.vits_flow_reverse(fsd, zp, mask, g, dtype=torch.float64, **fcfg)
    wr = hifigan_ref.hifigan_forward(dsd, zr * mask.double(), g=g.double(), pad=0, dtype=torch.float64, **dcfg)
    assert_close_fp32(z.cpu(), zr, f"vits z ({mode})", **tol(mode))
    assert_close_fp32(wav.cpu(), wr, f"vits wav ({mode})", **tol(mode))
    assert np.isfinite(wav.cpu().numpy()).all()


@pytest.mark.parametrize("mode", ["fp32x6", "f16x3", "bf16"])
@pytest.mark.parametrize("cond", [0, 16])
def test_vits_gate_fusion_bitwise(cuda_device, mode, cond, monkeypatch):
    """Gate fused into the in_layer epilogue, with the speaker term g_l (cvec, original row order)
    added there: bitwise equal to the separate gate kernel."""
    cfg = dict(VITS_FLOW, num_flows=2, cond_channels=cond)
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(2, cfg["channels"], 257, generator=gen).to(cuda_device)
    mask = (torch.arange(257)[None] < torch.tensor([257, 100])[:, None]).float().unsqueeze(1).to(cuda_device)
    g = torch.randn(2, cond, 1, generator=gen).to(cuda_device) if cond else None
    outs = []
    monkeypatch.setenv("TTS_MI355X_WN_LAYER", "0")  # the per-conv launches (one-launch layers: below)
    for fused in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_FLOW_GATE", fused)
        f, _ = build(cfg, 31, cuda_device, mode)
        outs.append(f(x, mask, g=g, reverse=True))
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("mode", ["fp32x6", "f16x3", "bf16"])
@pytest.mark.parametrize("cond", [0, 16])
def test_vits_wn_update_fusion_bitwise(cuda_device, mode, cond, monkeypatch):
    """The WN residual / skip update inside the res_skip conv epilogue (every layer but the last):
    bitwise equal to the separate update kernel, in both flow directions and in the posterior
    encoder's 16-layer WN."""
    cfg = dict(VITS_FLOW, num_flows=2, cond_channels=cond)
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(2, cfg["channels"], 257, generator=gen).to(cuda_device)
    mask = (torch.arange(257)[None] < torch.tensor([257, 100])[:, None]).float().unsqueeze(1).to(cuda_device)
    g = torch.randn(2, cond, 1, generator=gen).to(cuda_device) if cond else None
    spec = torch.randn(2, 64, 257, generator=gen).to(cuda_device)
    eps = torch.randn(2, 48, 257, generator=gen).to(cuda_device)
    lens = torch.tensor([257, 100]).to(cuda_device)
    pcfg = dict(in_channels=64, out_channels=48, hidden_channels=96, kernel_size=5, dilation_rate=1, num_layers=6,
                cond_channels=cond)
    outs = []
    monkeypatch.setenv("TTS_MI355X_WN_LAYER", "0")
    for fused in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_WN_FUSION", fused)
        f, _ = build(cfg, 31, cuda_device, mode)
        pe = PosteriorEncoder(**pcfg, math_mode=mode)
        pe.load_state_dict(synthetic.vits_posterior_state_dict(**pcfg, seed=7))
        pe = pe.to(cuda_device)
        outs.append((f(x, mask, g=g, reverse=True), f(x, mask, g=g, reverse=False), pe(spec, lens, g=g, noise=eps)[0]))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("mode", ["fp32x6", "f16x3", "bf16"])
@pytest.mark.parametrize("cond", [0, 16])
def test_vits_wn_layer_matches_unfused(cuda_device, mode, cond, monkeypatch):
    """One launch per WaveNet layer (kernels_glow_wn.hip) in the coupling flows (both directions) and
    the posterior encoder's 16-layer WN, against the four launches per layer: bitwise in bf16, the
    fp32-faithful tolerance in f16x3 / bf16x6 (test_glow_gpu.py explains why)."""
    cfg = dict(VITS_FLOW, num_flows=2, cond_channels=cond)
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(2, cfg["channels"], 257, generator=gen).to(cuda_device)
    mask = (torch.arange(257)[None] < torch.tensor([257, 100])[:, None]).float().unsqueeze(1).to(cuda_device)
    g = torch.randn(2, cond, 1, generator=gen).to(cuda_device) if cond else None
    spec = torch.randn(2, 64, 257, generator=gen).to(cuda_device)
    eps = torch.randn(2, 48, 257, generator=gen).to(cuda_device)
    lens = torch.tensor([257, 100]).to(cuda_device)
    pcfg = dict(in_channels=64, out_channels=48, hidden_channels=192, kernel_size=5, dilation_rate=1, num_layers=16,
                cond_channels=cond)
    outs, names = [], []
    for on in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_WN_LAYER", on)
        f, _ = build(cfg, 31, cuda_device, mode)
        pe = PosteriorEncoder(**pcfg, math_mode=mode)
        pe.load_state_dict(synthetic.vits_posterior_state_dict(**pcfg, seed=7))
        pe = pe.to(cuda_device)
        outs.append((f(x, mask, g=g, reverse=True), f(x, mask, g=g, reverse=False), pe(spec, lens, g=g, noise=eps)[0]))
        names.append([r["name"] for r in f.profile(x, mask, g=g)[1]])
    L = cfg["num_layers"]
    assert names[0].count("vits_wn_layer") == 2 * L and "vits_gate" not in names[0]
    assert names[1].count("vits_gate") == 2 * L and "vits_wn_layer" not in names[1]
    for what, a, b in zip(("reverse", "forward", "posterior z"), *outs):
        if mode == "bf16":
            assert torch.equal(a, b), what
        else:
            # posterior z = m + eps * exp(logs) after 16 layers: an absolute gate scaled to its magnitude
            scale = max(1.0, b.abs().max().item())
            assert_close_fp32(a.cpu(), b.cpu().double().numpy(), f"vits wn layer {what} {mode}", 1e-5 * scale, 5e-6)


@pytest.mark.parametrize("cond", [0, 16])
def test_vits_x0_statistics_match_prepass(cuda_device, cond, monkeypatch):
    """f16x3: the next flow's x0 max-abs from the post conv epilogue equals the per-flow pre-pass
    (TTS_MI355X_FLOW_AMAX_PREPASS=1): bitwise equal outputs with a ragged mask."""
    cfg = dict(VITS_FLOW, num_flows=4, cond_channels=cond)
    gen = torch.Generator().manual_seed(8)
    x = (torch.randn(2, cfg["channels"], 211, generator=gen) * 2).to(cuda_device)
    mask = (torch.arange(211)[None] < torch.tensor([211, 64])[:, None]).float().unsqueeze(1).to(cuda_device)
    g = torch.randn(2, cond, 1, generator=gen).to(cuda_device) if cond else None
    outs = []
    for prepass in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_FLOW_AMAX_PREPASS", prepass)
        f, _ = build(cfg, 37, cuda_device, "f16x3")
        outs.append(f(x, mask, g=g, reverse=True))
    assert torch.equal(outs[0], outs[1])


# ----------------------------------------------------------------------------- forward direction
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("name,meta,arr", VITS, ids=[g[0] for g in VITS])
def test_vits_flow_forward_vs_reference(cuda_device, name, meta, arr, mode):
    """reverse=False (voice conversion's z_p = flow(z, y_mask, g), vits.py:1226): the reference's
    own forward on its fp64 reverse output (the fixture's roundtrip_fp64)."""
    f, _ = build(meta["config"], meta["seed"], cuda_device, mode)
    g = torch.from_numpy(arr["g"]).to(cuda_device) if "g" in arr else None
    z = f(torch.from_numpy(arr["out_ref_fp64"]).float().to(cuda_device), torch.from_numpy(arr["mask"]).to(cuda_device),
          g=g, reverse=False)
    assert_close_fp32(z.cpu(), arr["roundtrip_fp64"], f"{name} forward ({mode})", **tol(mode))


@pytest.mark.parametrize("num_flows,cond", [(3, 0), (4, 4), (5, 4)])
def test_vits_flow_forward_vs_oracle_and_roundtrip(cuda_device, num_flows, cond):
    """Odd and even flow counts (the up-front flip for odd counts), with and without speaker
    conditioning, against the fp64 oracle; then reverse(forward(x)) = x under the mask."""
    cfg = dict(VITS_FLOW, channels=64, hidden_channels=96, num_layers=3, num_flows=num_flows, dilation_rate=2,
               cond_channels=cond)
    f, sd = build(cfg, 21 + num_flows, cuda_device, "f16x3")
    gen = torch.Generator().manual_seed(num_flows)
    B, T = 3, 77
    x = torch.randn(B, 64, T, generator=gen)
    m = (torch.arange(T)[None] < torch.tensor([77, 40, 1])[:, None]).float().unsqueeze(1)
    g = torch.randn(B, cond, 1, generator=gen) if cond else None
    gd = g.to(cuda_device) if g is not None else None
    z = f(x.to(cuda_device), m.to(cuda_device), g=gd, reverse=False)
    zr = vits_ref.vits_flow_forward(sd, x, m, g, **cfg)
    assert_close_fp32(z.cpu(), zr, f"vits forward F={num_flows}", **tol("f16x3"))
    y = f(z, m.to(cuda_device), g=gd, reverse=True)
    assert torch.allclose((y.cpu() * m), x * m, atol=1e-4)


# ----------------------------------------------------------------------------- posterior encoder
POSTERIOR = goldens("vits_posterior")


def build_posterior(cfg, seed, device, math_mode):
    from tts_amd.tts import PosteriorEncoder

    pe = PosteriorEncoder(cfg["in_channels"], cfg["out_channels"], cfg["hidden_channels"], cfg["kernel_size"],
                          cfg["dilation_rate"], cfg["num_layers"], cond_channels=cfg["cond_channels"],
                          math_mode=math_mode)
    sd = synthetic.vits_posterior_state_dict(**cfg, seed=seed)
    pe.load_state_dict(sd)
    return pe.to(device), sd


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("name,meta,arr", POSTERIOR, ids=[g[0] for g in POSTERIOR])
def test_vits_posterior_vs_reference(cuda_device, name, meta, arr, mode):
    """PosteriorEncoder (networks.py:235-288) against the reference's own outputs, with the noise
    the reference drew (the fixture's eps) passed in."""
    pe, _ = build_posterior(meta["config"], meta["seed"], cuda_device, mode)
    g = torch.from_numpy(arr["g"]).to(cuda_device) if "g" in arr else None
    z, m, logs, mask = pe(torch.from_numpy(arr["x"]).to(cuda_device), torch.from_numpy(arr["lengths"]), g=g,
                          noise=torch.from_numpy(arr["eps"]))
    assert torch.equal(mask.cpu(), torch.from_numpy(arr["mask"]))
    t = tol(mode, op=True)
    assert_close_fp32(z.cpu(), arr["z_ref_fp64"], f"{name} z ({mode})", **t)
    assert_close_fp32(m.cpu(), arr["m_ref_fp64"], f"{name} m ({mode})", **t)
    assert_close_fp32(logs.cpu(), arr["logs_ref_fp64"], f"{name} logs ({mode})", **t)


def test_vits_voice_conversion_path(cuda_device):
    """vits.py:1202-1228 on device: posterior encoder (source speaker) -> flow forward (source g)
    -> flow reverse (target g), against the fp64 oracle chain with the same noise; the round trip
    with source = target gives z back."""
    from tts_amd.config import VITS_POSTERIOR

    cond = 16
    pcfg = dict(VITS_POSTERIOR, cond_channels=cond, num_layers=4)
    fcfg = dict(VITS_FLOW, cond_channels=cond)
    pe, psd = build_posterior(pcfg, 5, cuda_device, "f16x3")
    flow, fsd = build(fcfg, 6, cuda_device, "f16x3")
    gen = torch.Generator().manual_seed(8)
    B, T = 2, 120
    y = torch.randn(B, 513, T, generator=gen)
    lengths = torch.tensor([120, 77])
    eps = torch.randn(B, 192, T, generator=gen)
    g_src = torch.randn(B, cond, 1, generator=gen)
    g_tgt = torch.randn(B, cond, 1, generator=gen)
    z, _, _, mask = pe(y.to(cuda_device), lengths, g=g_src.to(cuda_device), noise=eps)
    z_p = flow(z, mask, g=g_src.to(cuda_device), reverse=False)
    z_hat = flow(z_p, mask, g=g_tgt.to(cuda_device), reverse=True)
    m = mask.cpu()
    zr, _, _ = vits_ref.vits_posterior(psd, y, m, eps, g_src, **pcfg)
    zpr = vits_ref.vits_flow_forward(fsd, zr, m, g_src, **fcfg)
    zhr = vits_ref.vits_flow_reverse(fsd, zpr, m, g_tgt, **fcfg)
    assert_close_fp32(z.cpu(), zr, "posterior z", **tol("f16x3", op=True))
    assert_close_fp32(z_p.cpu(), zpr, "z_p", **tol("f16x3", op=True))
    assert_close_fp32(z_hat.cpu(), zhr, "z_hat", **tol("f16x3", op=True))
    back = flow(z_p, mask, g=g_src.to(cuda_device), reverse=True)
    assert torch.allclose(back * mask, z * mask, atol=1e-4)
