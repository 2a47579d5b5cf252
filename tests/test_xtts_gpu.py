"""XTTS waveform decoder (HifiDecoder: latent resampling + HiFiGAN with cond_in_each_up_layer) on
MI355X against the reference-module golden (tests/golden/make_goldens.py xtts)."""
import pytest
import torch

from _util import assert_close_fp32, goldens, tol
from oracle import hifigan_ref
from tts_amd import synthetic
from tts_amd.synthesizer import mel_handoff
from tts_amd.tts import HifiDecoder

pytestmark = pytest.mark.gpu
XTTS = goldens("xtts_decoder")


def build(meta, dev, mode):
    d = HifiDecoder(math_mode=mode)
    sd = synthetic.hifigan_state_dict(**meta["config"], seed=meta["seed"], weight_norm=True)
    d.waveform_decoder.load_state_dict(sd)
    d.eval()
    return d.to(dev)


@pytest.mark.parametrize("name,meta,arr", XTTS, ids=[g[0] for g in XTTS])
def test_latent_resampling_vs_reference(cuda_device, name, meta, arr):
    lat = torch.from_numpy(arr["latents"]).to(cuda_device)
    z = mel_handoff(lat, None, None, time_major=True, scale_factor=1024 / 256)
    z = mel_handoff(z, None, None, time_major=False, scale_factor=24000 / 22050)
    assert_close_fp32(z.cpu(), arr["z_ref_fp64"], "xtts z", 1e-5, 1e-6)


@pytest.mark.parametrize("mode", ["fp32", "fp32x6", "f16x3", "bf16"])
@pytest.mark.parametrize("name,meta,arr", XTTS, ids=[g[0] for g in XTTS])
def test_xtts_decoder_vs_reference(cuda_device, name, meta, arr, mode):
    d = build(meta, cuda_device, mode)
    out = d.inference(torch.from_numpy(arr["latents"]), torch.from_numpy(arr["g"]).to(cuda_device))
    assert_close_fp32(out.cpu(), arr["out_ref_fp64"], f"xtts {mode}", **tol(mode))


def test_xtts_generator_vs_oracle_longer(cuda_device):
    """The conditioned generator alone on a longer input (3 utterances x 57 frames), fp32 mode."""
    cfg = dict(XTTS[0][1]["config"])
    sd = synthetic.hifigan_state_dict(**cfg, seed=5, weight_norm=True)
    d = HifiDecoder(math_mode="fp32")
    d.waveform_decoder.load_state_dict(sd)
    d = d.to(cuda_device)
    x = torch.randn(3, 1024, 57, generator=torch.Generator().manual_seed(1))
    g = torch.randn(3, 512, 1, generator=torch.Generator().manual_seed(2)) * 0.5
    out = d.waveform_decoder(x.to(cuda_device), g=g.to(cuda_device))
    ref = hifigan_ref.hifigan_forward(sd, x, pad=0, g=g, dtype=torch.float64, fold_dtype=torch.float64, **cfg)
    assert_close_fp32(out.cpu(), ref, "xtts generator B=3 T=57", **tol("fp32"))
