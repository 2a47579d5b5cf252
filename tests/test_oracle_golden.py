"""Pin the CPU oracle (oracle/) against golden vectors produced by the reference modules
(tests/golden/make_goldens.py).  CPU only."""
import numpy as np
import pytest
import torch

from _util import goldens, max_abs, rel_rms
from oracle import glow_ref, hifigan_ref, vits_ref
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
    out = glow_ref.glow_decoder_reverse(sd, torch.from_numpy(arr["x"]), torch.from_numpy(arr["mask"]),
                                        dtype=torch.float64, **cfg)
    assert out.shape == arr["out_ref_fp64"].shape
    assert max_abs(out.numpy(), arr["out_ref_fp64"]) < 1e-10
    out32 = glow_ref.glow_decoder_reverse(sd, torch.from_numpy(arr["x"]), torch.from_numpy(arr["mask"]),
                                          dtype=torch.float32, **cfg)
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


def test_synthetic_weights_deterministic():
    a = synthetic.hifigan_state_dict(seed=3)
    b = synthetic.hifigan_state_dict(seed=3)
    assert list(a) == list(b)
    for k in a:
        assert torch.equal(a[k], b[k])
    c = synthetic.hifigan_state_dict(seed=4)
    assert not torch.equal(a["conv_pre.bias"], c["conv_pre.bias"])
