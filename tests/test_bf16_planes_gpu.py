"""bf16 activation planes (MATH_BF16, round 6): the HiFiGAN executor's Z / O / X / T planes hold
bf16 instead of fp32 (hifigan.hpp ``planes16_``; every kernel family stages, gathers and stores
2-byte elements: conv_device.hpp PlaneT).  The MFMA operands were bf16 already, so the change adds
one rounding per stored plane, as the reference's own bf16 forward has (its activations are bf16
tensors).  Each case runs the generator with bf16 planes (the default) and with fp32 planes
(TTS_MI355X_BF16_PLANES=0) and holds both to the bf16 gates of the fp64 oracle (SURVEY.md §8c:
rel-RMS 3e-2, tests/_util.py), and the two to twice the max-abs gate of each other.  The cases
cover every kernel family's bf16-plane instance: conv_pre (fp32 mel -> bf16), the x8 upsampler
(convT_res_kernel) and the x2 ones (split kernel, K = 2), the Winograd convs at dilations 1 / 3 / 5
(the D = 3 window offset per workgroup), the fused pair with and without conv_post, the whole
kernel-3 blocks, ResBlock2 blocks, the per-conv split kernels (k3 / k5 / k7 / k11, wide-halo
tiles at dilation 12), the separate conv_post, the windowed long-utterance path, the VITS
decoder's cond vector and the XTTS per-stage conds.
"""
import os

import pytest
import torch

from _util import assert_close_fp32, max_abs, tol
from oracle import hifigan_ref
from tts_amd import synthetic
from tts_amd.config import HIFIGAN_V1, VITS_DECODER
from tts_amd.vocoder import HifiganGenerator

pytestmark = pytest.mark.gpu
V1 = dict(in_channels=80, out_channels=1, **HIFIGAN_V1)
RB2_V3 = dict(in_channels=80, out_channels=1, resblock_type="2",
              resblock_dilation_sizes=[[1, 2], [2, 6], [3, 12]], resblock_kernel_sizes=[3, 5, 7],
              upsample_kernel_sizes=[16, 16, 8], upsample_initial_channel=256, upsample_factors=[8, 8, 4],
              inference_padding=5)
RB2_YOURTTS = dict(in_channels=80, out_channels=1, resblock_type="2",
                   resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], resblock_kernel_sizes=[3, 7, 11],
                   upsample_kernel_sizes=[16, 16, 4, 4], upsample_initial_channel=256,
                   upsample_factors=[8, 8, 2, 2], inference_padding=5)
# every per-conv path: no pair / whole-block fusion, no Winograd, the separate conv_post
UNFUSED = {"TTS_MI355X_NO_PAIR_FUSION": "1", "TTS_MI355X_RESBLOCK3": "0", "TTS_MI355X_WINO": "0",
           "TTS_MI355X_POST_FUSION": "0"}


def _gen(cfg, sd, dev):
    g = HifiganGenerator(**cfg, math_mode="bf16")
    g.remove_weight_norm()
    g.load_state_dict(sd)
    return g.to(dev)


def _both(monkeypatch, cfg, sd, mel, dev, env=(), gvec=None, pad=None):
    """(bf16 planes, fp32 planes) outputs and the bytes the profiled forwards report."""
    for k, v in dict(env).items():
        monkeypatch.setenv(k, v)
    outs, nbytes = {}, {}
    for planes in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_BF16_PLANES", planes)
        g = _gen(cfg, sd, dev)
        x = mel.to(dev)
        gv = None if gvec is None else gvec.to(dev)
        if pad is None:
            outs[planes] = (g.inference(x) if gv is None else g.inference(x, g=gv)).cpu()
        else:
            outs[planes] = g._run(x, pad, gv).cpu()
        rows = g.profile(x, pad, g=gv)[1]
        nbytes[planes] = sum(r.get("bytes", 0.0) for r in rows if r["name"].startswith(("mrf_", "ups")))
    return outs, nbytes


def _check(outs, ref, what):
    for planes, out in outs.items():
        assert_close_fp32(out, ref, f"{what} bf16 planes={planes}", **tol("bf16"))
    assert max_abs(outs["1"].numpy(), outs["0"].numpy()) <= 2 * tol("bf16")["max_abs_tol"], what
    # the bf16 planes really are a different rounding (a mis-wired plane type reads garbage instead)
    assert not torch.equal(outs["1"], outs["0"]), what


@pytest.mark.parametrize("env", [(), tuple(UNFUSED.items())], ids=["default", "unfused"])
def test_bf16_planes_v1(cuda_device, monkeypatch, env):
    """HiFiGAN-v1 over several tiles per stage (stage 3 has 9,088 samples: Winograd D = 3 tiles start
    at t0 = 252 j, half of them 4 mod 8) in the default fused schedule and in the per-conv one."""
    sd = synthetic.hifigan_state_dict(seed=61, weight_norm=False)
    mel = synthetic.mel(2, 61, seed=6)
    outs, nb = _both(monkeypatch, V1, sd, mel, cuda_device, env)
    ref = hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **V1)
    _check(outs, ref, f"v1 {dict(env)}")
    # the executor's byte accounting follows the plane type (2 B per activation element; the
    # weights, 4 B, dominate at this size)
    assert nb["1"] < nb["0"], nb


@pytest.mark.parametrize("cfg_name", ["v3", "yourtts"])
@pytest.mark.parametrize("fused", ["all", "0"])
def test_bf16_planes_resblock2(cuda_device, monkeypatch, cfg_name, fused):
    """ResBlock2 topologies: whole-block launches (kernels 3 / 5 / 7 / 11) or per-conv launches,
    HiFiGAN-v3's kernel 7 at dilation 12 on the wide-halo split tiles, a x4 upsampler."""
    cfg = RB2_V3 if cfg_name == "v3" else RB2_YOURTTS
    sd = synthetic.hifigan_state_dict(seed=62, weight_norm=False, **cfg)
    mel = synthetic.mel(2, 23, seed=7)
    outs, _ = _both(monkeypatch, cfg, sd, mel, cuda_device, {"TTS_MI355X_RESBLOCK3": fused, "TTS_MI355X_RB2_ALL": "1"})
    ref = hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **cfg)
    _check(outs, ref, f"{cfg_name} fused={fused}")


def test_bf16_planes_vits_decoder(cuda_device, monkeypatch):
    """The VITS waveform decoder: cond_layer(g) added in conv_pre's epilogue, no padding, conv_post
    without bias, ragged latent lengths (vits.py:1156-1162)."""
    cond = 16
    dcfg = dict(VITS_DECODER, upsample_initial_channel=256, cond_channels=cond)
    sd = synthetic.hifigan_state_dict(**dcfg, seed=63, weight_norm=False)
    gen = torch.Generator().manual_seed(10)
    z = torch.randn(3, 192, 29, generator=gen) * 0.5
    g = torch.randn(3, cond, 1, generator=gen)
    outs, _ = _both(monkeypatch, dcfg, sd, z, cuda_device, gvec=g, pad=0)
    ref = hifigan_ref.hifigan_forward(sd, z, g=g.double(), pad=0, dtype=torch.float64, **dcfg)
    _check(outs, ref, "vits decoder")


def test_bf16_planes_windowed(cuda_device, monkeypatch):
    """The long-utterance path (37-frame payloads + the receptive-field halo) on bf16 planes."""
    sd = synthetic.hifigan_state_dict(seed=64, weight_norm=False)
    mel = synthetic.mel(1, 100, seed=8)
    outs, _ = _both(monkeypatch, V1, sd, mel, cuda_device, {"TTS_MI355X_WINDOW_FRAMES": "37"})
    ref = hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **V1)
    _check(outs, ref, "windowed")


def test_bf16_planes_batch_invariant_and_deterministic(cuda_device, monkeypatch):
    """Per-utterance planes: each utterance of a batch (split over the executor's lanes) is bitwise
    the utterance run alone, and two runs are bitwise equal."""
    monkeypatch.setenv("TTS_MI355X_BF16_PLANES", "1")
    sd = synthetic.hifigan_state_dict(seed=65, weight_norm=False)
    g = _gen(V1, sd, cuda_device)
    mel = synthetic.mel(4, 80, seed=9).to(cuda_device)
    y = g.inference(mel)
    assert torch.equal(y, g.inference(mel))
    for i in (0, 3):
        assert torch.equal(g.inference(mel[i:i + 1])[0], y[i])
    assert torch.isfinite(y).all() and y.abs().max() <= 1.0


@pytest.mark.parametrize("planes", ["1", "0"])
def test_bf16_pair128_matches_winograd(cuda_device, monkeypatch, planes):
    """bf16: the 128-channel kernel-7 / 11 ResBlock1 iterations as fused pairs (resblock_pair128:
    direct convs, xt in LDS; one launch per iteration) against the two Winograd launches per
    iteration (TTS_MI355X_PAIR128=0), both within the bf16 gates of the fp64 oracle and of each
    other, on either plane type; the profiled launch names show which form ran."""
    monkeypatch.setenv("TTS_MI355X_BF16_PLANES", planes)
    sd = synthetic.hifigan_state_dict(seed=66, weight_norm=False)
    mel = synthetic.mel(2, 41, seed=10)
    ref = hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **V1)
    outs = {}
    for p128 in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_PAIR128", p128)
        g = _gen(V1, sd, cuda_device)
        outs[p128] = g.inference(mel.to(cuda_device)).cpu()
        names = [r["name"] for r in g.profile(mel.to(cuda_device))[1]]
        pairs = [n for n in names if n.startswith("mrf_pair_k") and n.endswith("_c128")]
        winos = [n for n in names if n.startswith("mrf_wino_k") and n.endswith("_c128")]
        assert (len(pairs), len(winos)) == ((6, 0) if p128 == "1" else (0, 12)), names
        # the 256-channel kernel-3 / 7 iterations run as pairs in both arms (TTS_MI355X_PAIR256),
        # kernel 11 too under TTS_MI355X_PAIR256_K11=1
        n256 = 9 if os.environ.get("TTS_MI355X_PAIR256_K11") == "1" else 6
        assert sum(n.startswith("mrf_pair_k") and n.endswith("_c256") for n in names) == n256, names
        assert_close_fp32(outs[p128], ref, f"pair128={p128} planes={planes}", **tol("bf16"))
    assert max_abs(outs["1"].numpy(), outs["0"].numpy()) <= 2 * tol("bf16")["max_abs_tol"]


def test_bf16_pair256_matches_per_conv(cuda_device, monkeypatch):
    """bf16: the 256-channel kernel-3 / 7 ResBlock1 iterations as fused pairs on 128-column tiles
    against their per-conv launches (TTS_MI355X_PAIR256=0: Winograd k7, direct k3), over several
    tiles per utterance and a ragged tail."""
    sd = synthetic.hifigan_state_dict(seed=67, weight_norm=False)
    mel = synthetic.mel(2, 53, seed=11)
    ref = hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **V1)
    outs = {}
    for p256 in ("1", "0"):
        monkeypatch.setenv("TTS_MI355X_PAIR256", p256)
        g = _gen(V1, sd, cuda_device)
        outs[p256] = g.inference(mel.to(cuda_device)).cpu()
        names = [r["name"] for r in g.profile(mel.to(cuda_device))[1]]
        n256 = sum(n.startswith("mrf_pair_k") and n.endswith("_c256") for n in names)
        n256_on = 9 if os.environ.get("TTS_MI355X_PAIR256_K11") == "1" else 6
        assert n256 == (n256_on if p256 == "1" else 0), names
        assert_close_fp32(outs[p256], ref, f"pair256={p256}", **tol("bf16"))
    assert max_abs(outs["1"].numpy(), outs["0"].numpy()) <= 2 * tol("bf16")["max_abs_tol"]
