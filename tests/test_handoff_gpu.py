"""TTS -> vocoder hand-off (tts_mel_handoff) and the int16 wav writer (tts_wav_to_int16) on MI355X
against the numpy oracle (oracle/handoff_ref.py, pinned by the handoff golden)."""
import numpy as np
import pytest
import torch

from _util import goldens
from oracle import handoff_ref
from tts_amd.synthesizer import AudioNorm, mel_handoff, wav_to_int16

pytestmark = pytest.mark.gpu
HANDOFF = goldens("handoff")

RANGE_SYM = dict(signal_norm=True, symmetric_norm=True, clip_norm=True, max_norm=4.0, min_level_db=-100,
                 ref_level_db=20, sample_rate=22050)
RANGE_POS = dict(signal_norm=True, symmetric_norm=False, clip_norm=True, max_norm=1.0, min_level_db=-100,
                 ref_level_db=0, sample_rate=22050)


def _norm(d):
    return AudioNorm(**{k: d[k] for k in d if k in AudioNorm.__dataclass_fields__})


def _oracle_batch(x, tts_a, voc_a):
    return np.stack([handoff_ref.handoff(x[b], tts_a, voc_a) for b in range(x.shape[0])])


@pytest.mark.parametrize("tts_a,voc_a", [
    (RANGE_SYM, RANGE_SYM), (RANGE_SYM, RANGE_POS), (RANGE_POS, RANGE_SYM),
    (dict(RANGE_SYM, clip_norm=False), dict(RANGE_POS, clip_norm=False, max_norm=2.5, ref_level_db=16)),
    (dict(RANGE_SYM, signal_norm=False), RANGE_SYM),
])
def test_handoff_range_norm_bit_exact(cuda_device, tts_a, voc_a):
    x = (np.random.default_rng(1).standard_normal((3, 91, 80)) * 3).astype(np.float32)  # [B, T, C], some clipped
    out = mel_handoff(torch.from_numpy(x).to(cuda_device), _norm(tts_a), _norm(voc_a))
    ref = _oracle_batch(x, tts_a, voc_a)
    assert out.shape == ref.shape
    assert np.array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("name,meta,arr", HANDOFF, ids=[g[0] for g in HANDOFF])
def test_handoff_mean_var_and_resample(cuda_device, name, meta, arr):
    mv = dict(RANGE_SYM, mel_mean=arr["mean"], mel_std=arr["std"])
    x = np.stack([arr["mel"], arr["mel"][::-1].copy()])  # [2, T, C]
    # mean-var denormalise -> mean-var normalise: bit-exact (fp64 statistics as numpy)
    out = mel_handoff(torch.from_numpy(x).to(cuda_device), _norm(mv), _norm(mv))
    assert np.array_equal(out[0].cpu().numpy(), arr["renorm_ref"].T)
    # denormalise only + 22.05 -> 24 kHz resampling: the reference's F.interpolate on the CPU
    voc = dict(RANGE_SYM, signal_norm=False, sample_rate=meta["sr_voc"])
    out = mel_handoff(torch.from_numpy(x).to(cuda_device), _norm(mv), _norm(voc))
    assert out.shape[2] == arr["interp_ref"].shape[1]
    np.testing.assert_allclose(out[0].cpu().numpy(), arr["interp_ref"], rtol=2e-7, atol=1e-5)


def test_handoff_channel_major_input(cuda_device):
    x = (np.random.default_rng(2).standard_normal((2, 80, 33)) * 3).astype(np.float32)  # [B, C, T]
    out = mel_handoff(torch.from_numpy(x).to(cuda_device), _norm(RANGE_SYM), _norm(RANGE_POS), time_major=False)
    ref = _oracle_batch(np.ascontiguousarray(x.transpose(0, 2, 1)), RANGE_SYM, RANGE_POS)
    assert np.array_equal(out.cpu().numpy(), ref)


def test_wav_int16_matches_save_wav_scaling(cuda_device):
    rng = np.random.default_rng(3)
    w = (np.tanh(rng.standard_normal((4, 1, 50003))) * np.array([1.0, 0.3, 0.004, 0.0])[:, None, None]).astype(np.float32)
    out = wav_to_int16(torch.from_numpy(w).to(cuda_device)).cpu().numpy()
    for b in range(4):
        assert np.array_equal(out[b], handoff_ref.wav_int16(w[b, 0])), b  # incl. the 0.01 floor and all-zero
    lens = torch.tensor([50003, 20000, 7, 1])
    out = wav_to_int16(torch.from_numpy(w).to(cuda_device), lens).cpu().numpy()
    for b in range(4):
        L = int(lens[b])
        assert np.array_equal(out[b, :L], handoff_ref.wav_int16(w[b, 0, :L]))
        assert not out[b, L:].any()


HRANGE = goldens("handoff_range")


def test_wav_int16_nonfinite_matches_numpy(cuda_device):
    """NaN / inf / overflowing samples follow numpy's x86 behaviour (see kernels_handoff.hip)."""
    rng = np.random.default_rng(5)
    w = (np.tanh(rng.standard_normal((3, 1, 4099))) * 0.7).astype(np.float32)
    w[0, 0, 17] = np.nan  # scale 32767 / 0.01: most samples wrap
    w[1, 0, 4000] = np.inf  # scale 0: finite -> 0, inf -> NaN -> 0
    w[2, 0, 5] = -np.inf
    w[2, 0, 9] = np.nan
    out = wav_to_int16(torch.from_numpy(w).to(cuda_device)).cpu().numpy()
    with np.errstate(invalid="ignore", over="ignore"):
        for b in range(3):
            assert np.array_equal(out[b], handoff_ref.wav_int16(w[b, 0])), b


def test_wav_int16_finite_overflow_matches_numpy(cuda_device):
    """Finite samples whose scaled value reaches 2^31 (a NaN forces the scale to 32767 / 0.01):
    x86 cvttss2si gives INT_MIN, whose low 16 bits are 0; just below 2^31 the value wraps."""
    rng = np.random.default_rng(6)
    w = (np.tanh(rng.standard_normal((2, 1, 1031))) * 0.5).astype(np.float32)
    w[0, 0, 0] = np.nan
    w[0, 0, 1:9] = [1000.0, -700.0, 655.0, 655.3, 656.0, -656.0, -655.3, 2.5e4]
    w[1, 0, 3] = np.nan
    w[1, 0, 100:103] = [-1e9, 654.9, 3.0e-3]
    out = wav_to_int16(torch.from_numpy(w).to(cuda_device)).cpu().numpy()
    with np.errstate(invalid="ignore", over="ignore"):
        for b in range(2):
            assert np.array_equal(out[b], handoff_ref.wav_int16(w[b, 0])), b


@pytest.mark.parametrize("name,meta,arr", HRANGE, ids=[g[0] for g in HRANGE])
def test_handoff_and_int16_vs_reference_functions(cuda_device, name, meta, arr):
    """Bit-exact against the reference's own AudioProcessor.normalize/denormalize and
    numpy_transforms.save_wav output (tests/golden/make_goldens.py handoff)."""
    cfgs = meta["configs"]
    x = torch.from_numpy(arr["mel"][None]).to(cuda_device)  # [1, T, C]
    for i, j in meta["pairs"]:
        out = mel_handoff(x, _norm(dict(cfgs[i], sample_rate=22050)), _norm(dict(cfgs[j], sample_rate=22050)))
        assert np.array_equal(out[0].cpu().numpy(), arr[f"out_{i}_{j}"]), (i, j)
    for k in range(meta["n_wavs"]):
        w = torch.from_numpy(arr[f"wav_{k}"][None]).to(cuda_device)
        assert np.array_equal(wav_to_int16(w)[0].cpu().numpy(), arr[f"pcm_{k}"]), k
