"""BASELINE configs 3 and 5 at their bench workloads, through the C-ABI, with size-independent
properties (finite, |wav| <= 1, bitwise determinism, batch invariance of a full-length row) and
one utterance against the fp64 oracle chain.

* Config 3: Glow-TTS (LJSpeech cfg) + on-device hand-off + HiFiGAN-v1, 16 x 128 tokens, decoder
  and vocoder in bf16 (``Synthesizer.tts_batch``).  Reference chain: ``glow_tts.py:342-374`` ->
  ``synthesizer.py:410-429`` (denormalize -> normalize -> vocoder.inference).
* Config 5 (one GPU's share of batch 64 over 8): VITS reverse flow (4 flows, 192 ch, speaker cond
  256) -> z * mask -> 512-channel HiFiGAN decoder (in 192, cond_layer, no conv_post bias, no
  padding), 8 x 1024 latent frames, in bf16 and f16x3.  Reference: ``vits.py:1156-1162`` with
  the decoder built at ``vits.py:704-718``.
"""
import functools

import numpy as np
import pytest
import torch

from _util import assert_close_fp32, tol
from oracle import glow_ref, glow_tts_ref, handoff_ref, hifigan_ref, vits_ref
from tts_amd import synthetic
from tts_amd.config import GLOW_TTS_DECODER as G, GLOW_TTS_ENCODER as E, HIFIGAN_V1, VITS_DECODER, VITS_FLOW
from tts_amd.synthesizer import AudioNorm, Synthesizer
from tts_amd.tts import GlowTTS, ResidualCouplingBlocks
from tts_amd.vocoder import HifiganGenerator

pytestmark = pytest.mark.gpu

# ------------------------------------------------------------------------------- config 3
ECFG = dict(E, num_chars=64)
DCFG = dict(in_channels=G["in_channels"], hidden_channels=G["hidden_channels"], kernel_size=G["kernel_size"],
            dilation_rate=G["dilation_rate"], num_flow_blocks=G["num_flow_blocks"],
            num_coupling_layers=G["num_coupling_layers"], num_splits=G["num_splits"], num_squeeze=G["num_squeeze"])
VCFG = dict(in_channels=80, out_channels=1, **HIFIGAN_V1)
ESEED, DSEED, VSEED = 8642, 4321, 1234  # bench.py glow_tts_e2e_bench


def _glow_sd():
    sd = {f"encoder.{k}": v for k, v in
          synthetic.glow_encoder_state_dict(**ECFG, seed=ESEED, log_duration=1.872).items()}
    sd.update({f"decoder.{k}": v for k, v in synthetic.glow_decoder_state_dict(**DCFG, seed=DSEED).items()})
    return sd


def _synth(dev, mode):
    m = GlowTTS(dict(num_chars=64), decoder_math_mode=mode)
    m.load_state_dict(_glow_sd())
    m.eval()
    m.store_inverse()
    m = m.to(dev)
    voc = HifiganGenerator(**VCFG, math_mode=mode)
    voc.remove_weight_norm()
    voc.load_state_dict(synthetic.hifigan_state_dict(**VCFG, seed=VSEED, weight_norm=False))
    voc.eval()
    return Synthesizer(m, voc.to(dev), AudioNorm(), AudioNorm())  # BaseAudioConfig defaults both sides


@functools.lru_cache(maxsize=None)
def _config3_oracle_row(row: int):
    """fp64 oracle chain for one utterance: encoder -> durations -> expand -> decoder reverse ->
    hand-off (numpy, the reference's dtypes) -> HiFiGAN inference."""
    tok = synthetic.tokens(16, 128, 64, seed=11)[row:row + 1]
    lens = torch.tensor([128])
    esd = synthetic.glow_encoder_state_dict(**ECFG, seed=ESEED, log_duration=1.872)
    x_m, _, logw, xmask = glow_tts_ref.encoder_forward(esd, tok, lens)
    w_ceil, ylen = glow_tts_ref.durations(logw, xmask)
    z, ymask, *_ = glow_tts_ref.expand(w_ceil, xmask, ylen, x_m, torch.zeros_like(x_m))
    mel = glow_ref.glow_decoder_reverse(synthetic.glow_decoder_state_dict(**DCFG, seed=DSEED), z, ymask, **DCFG)
    a = dict(signal_norm=True, symmetric_norm=True, clip_norm=True, max_norm=4.0, min_level_db=-100,
             ref_level_db=20, sample_rate=22050, mel_mean=None, mel_std=None)
    voc_in = handoff_ref.handoff(mel[0].T.float().numpy(), a, a)  # model_outputs[0] is fp32 [T, C]
    sd = synthetic.hifigan_state_dict(**VCFG, seed=VSEED, weight_norm=False)
    wav = hifigan_ref.hifigan_forward(sd, torch.from_numpy(np.ascontiguousarray(voc_in))[None].double(), pad=5,
                                      dtype=torch.float64, **VCFG)
    return int(ylen[0]), wav


def test_config3_text_to_wav_bf16(cuda_device):
    dev = cuda_device
    syn = _synth(dev, "bf16")
    tok = synthetic.tokens(16, 128, 64, seed=11).to(dev)
    lens = torch.full((16,), 128, dtype=torch.int64, device=dev)
    wav, voc_in = syn.tts_batch(tok, lens)
    wav2, _ = syn.tts_batch(tok, lens)
    T = voc_in.shape[2]
    assert wav.shape == (16, 1, 256 * (T + 10))
    assert T > 600  # ~6 frames per token
    assert torch.isfinite(wav).all() and wav.abs().max() <= 1.0
    assert torch.equal(wav, wav2), "config 3 is not run-to-run deterministic"
    # the longest utterance has no padded frames: alone it must give the same bits
    out = syn.tts_model.inference(tok, {"x_lengths": lens})
    align = out["alignments"]  # [B, T_y, T_x]
    frames = align.sum((1, 2)).long()
    row = int(torch.argmax(frames))
    assert int(frames[row]) // 2 * 2 == T  # the decoder's squeeze drops an odd last frame (decoder.py:19)
    w1, _ = syn.tts_batch(tok[row:row + 1], lens[row:row + 1])
    assert torch.equal(w1[0], wav[row]), "the full-length row is not batch-invariant"
    # against the fp64 oracle chain at the bf16 gate
    ylen_ref, ref = _config3_oracle_row(row)
    assert ylen_ref // 2 * 2 == T
    assert_close_fp32(wav[row:row + 1].cpu(), ref, f"config 3 row {row} (bf16)", **tol("bf16"))


# ------------------------------------------------------------------------------- config 5
COND = 256
FCFG = dict(VITS_FLOW, cond_channels=COND)
VDCFG = dict(VITS_DECODER, cond_channels=COND)
B5, T5 = 8, 1024
LENS5 = [1024, 1024, 1024, 1024, 1024, 1024, 700, 1024]


def _config5_inputs():
    gen = torch.Generator().manual_seed(9)
    zp = torch.randn(B5, 192, T5, generator=gen)
    g = torch.randn(B5, COND, 1, generator=gen)
    mask = (torch.arange(T5)[None, :] < torch.tensor(LENS5)[:, None]).float().unsqueeze(1)
    return zp, mask, g


@functools.lru_cache(maxsize=None)
def _config5_oracle(row: int):
    zp, mask, g = _config5_inputs()
    fsd = synthetic.vits_flow_state_dict(**FCFG, seed=2469)
    dsd = synthetic.hifigan_state_dict(**VDCFG, seed=99, weight_norm=False)
    z = vits_ref.vits_flow_reverse(fsd, zp[row:row + 1], mask[row:row + 1], g[row:row + 1], dtype=torch.float64,
                                   **FCFG)
    m = mask[row:row + 1].double()
    return hifigan_ref.hifigan_forward(dsd, z * m, g=g[row:row + 1].double(), pad=0, dtype=torch.float64, **VDCFG)


@pytest.mark.parametrize("mode", ["bf16", "f16x3"])
def test_config5_vits_waveform_path(cuda_device, mode):
    dev = cuda_device
    flow = ResidualCouplingBlocks(FCFG["channels"], FCFG["hidden_channels"], FCFG["kernel_size"],
                                  FCFG["dilation_rate"], FCFG["num_layers"], num_flows=FCFG["num_flows"],
                                  cond_channels=COND, math_mode=mode)
    flow.load_state_dict(synthetic.vits_flow_state_dict(**FCFG, seed=2469))
    flow = flow.to(dev)
    dec = HifiganGenerator(**VDCFG, math_mode=mode)
    dec.remove_weight_norm()
    dec.load_state_dict(synthetic.hifigan_state_dict(**VDCFG, seed=99, weight_norm=False))
    dec = dec.to(dev)
    zp, mask, g = (t.to(dev) for t in _config5_inputs())

    def run(sl):
        z = flow(zp[sl], mask[sl], g=g[sl], reverse=True)
        return dec(z * mask[sl], g=g[sl])

    wav = run(slice(0, B5))
    assert wav.shape == (B5, 1, 256 * T5)
    assert torch.isfinite(wav).all() and wav.abs().max() <= 1.0
    assert torch.equal(run(slice(0, B5)), wav), "config 5 is not run-to-run deterministic"
    assert torch.equal(run(slice(2, 3))[0], wav[2]), "a full-length row is not batch-invariant"
    assert torch.equal(run(slice(6, 7))[0], wav[6]), "the ragged row is not batch-invariant"
    for row in (0, 6):  # a full-length and the ragged utterance against fp64
        assert_close_fp32(wav[row:row + 1].cpu(), _config5_oracle(row), f"config 5 row {row} ({mode})", **tol(mode))
