"""ORACLE — test infrastructure only.  Never imported by the product path (tts-3_amd/).

numpy restatement of the Synthesizer's TTS -> vocoder hand-off and of save_wav's int16 scaling,
with the reference's dtypes (fp32 arrays, Python scalars, fp64 mean-var statistics):

* ``TTS/utils/audio/processor.py:259-297``  AudioProcessor.normalize
* ``processor.py:299-336``                  AudioProcessor.denormalize
* ``TTS/tts/utils/helpers.py:14-39``        StandardScaler (mel_scaler) transform / inverse_transform
* ``TTS/vocoder/utils/generic_utils.py:11-29`` interpolate_vocoder_input
* ``TTS/utils/synthesizer.py:412-428``      the hand-off sequence
* ``TTS/utils/audio/numpy_transforms.py:430-447`` save_wav scaling + astype(int16)

``processor.py`` / ``numpy_transforms.py`` / ``generic_utils.py`` import librosa / soundfile /
matplotlib, absent in this container, so those functions are restated here (the arithmetic is
a few lines each; expression order kept).  ``StandardScaler`` is importable and pins the
mean-var path (tests/golden/make_goldens.py handoff).
"""
from __future__ import annotations

import numpy as np
import torch


def normalize(S: np.ndarray, a: dict) -> np.ndarray:
    S = S.copy()
    if not a["signal_norm"]:
        return S
    if a.get("mel_mean") is not None:  # mel_scaler.transform(S.T).T
        X = S.T
        X -= a["mel_mean"]
        X /= a["mel_std"]
        return X.T
    S -= a["ref_level_db"]
    S_norm = (S - a["min_level_db"]) / (-a["min_level_db"])
    if a["symmetric_norm"]:
        S_norm = ((2 * a["max_norm"]) * S_norm) - a["max_norm"]
        if a["clip_norm"]:
            S_norm = np.clip(S_norm, -a["max_norm"], a["max_norm"])
        return S_norm
    S_norm = a["max_norm"] * S_norm
    if a["clip_norm"]:
        S_norm = np.clip(S_norm, 0, a["max_norm"])
    return S_norm


def denormalize(S: np.ndarray, a: dict) -> np.ndarray:
    S_denorm = S.copy()
    if not a["signal_norm"]:
        return S_denorm
    if a.get("mel_mean") is not None:  # mel_scaler.inverse_transform(S.T).T
        X = S_denorm.T
        X *= a["mel_std"]
        X += a["mel_mean"]
        return X.T
    if a["symmetric_norm"]:
        if a["clip_norm"]:
            S_denorm = np.clip(S_denorm, -a["max_norm"], a["max_norm"])
        S_denorm = ((S_denorm + a["max_norm"]) * -a["min_level_db"] / (2 * a["max_norm"])) + a["min_level_db"]
        return S_denorm + a["ref_level_db"]
    if a["clip_norm"]:
        S_denorm = np.clip(S_denorm, 0, a["max_norm"])
    S_denorm = (S_denorm * -a["min_level_db"] / a["max_norm"]) + a["min_level_db"]
    return S_denorm + a["ref_level_db"]


def handoff(model_output: np.ndarray, tts_audio: dict, voc_audio: dict) -> np.ndarray:
    """One utterance, synthesizer.py:412-428: model_outputs[0] [T, C] fp32 -> vocoder input [C, T']."""
    mel = denormalize(model_output.T, tts_audio).T
    voc = normalize(mel.T, voc_audio)
    sf = voc_audio["sample_rate"] / tts_audio["sample_rate"]
    if sf != 1:
        spec = torch.tensor(voc).unsqueeze(0).unsqueeze(0)
        spec = torch.nn.functional.interpolate(spec, scale_factor=[1, sf], recompute_scale_factor=True,
                                               mode="bilinear", align_corners=False).squeeze(0)
        return spec[0].numpy()
    return np.asarray(voc)


def wav_int16(wav: np.ndarray) -> np.ndarray:
    wav_norm = wav * (32767 / max(0.01, np.max(np.abs(wav))))
    return wav_norm.astype(np.int16)
