"""TTS -> vocoder hand-off on the device (``TTS/utils/synthesizer.py:410-434``) and the int16 wav
writer (``TTS/utils/audio/numpy_transforms.py:430-447``).

The reference's ``Synthesizer.tts`` synthesizes one sentence at a time and moves every mel to
the host between the acoustic model and the vocoder: ``model_outputs[0].cpu().numpy()`` ->
``tts_ap.denormalize`` -> ``vocoder_ap.normalize`` -> (``interpolate_vocoder_input`` when the
sample rates differ) -> ``torch.tensor`` -> ``vocoder.inference``.  Here the whole batch stays in
HBM: ``mel_handoff`` runs both normalisations (and the resampling) in one kernel straight from the
acoustic model's ``[B, T, C]`` output into the vocoder's ``[B, C, T]`` input
(``tts_mel_handoff``), and ``wav_to_int16`` applies ``save_wav``'s peak scaling and int16 cast
per utterance on the device (``tts_wav_to_int16``).

The text frontend (``TTSTokenizer``, sentence splitting) is out of scope: ``Synthesizer`` takes
token ids.  ``AudioNorm`` mirrors the normalisation fields of ``BaseAudioConfig``
(``TTS/config/shared_configs.py:126-154``); mean-var statistics are passed as arrays
(``mel_mean`` / ``mel_std``), not loaded from a pickled ``stats_path``.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from . import _native as N


@dataclass
class AudioNorm:
    """AudioProcessor normalisation parameters (processor.py:259-336)."""

    signal_norm: bool = True
    symmetric_norm: bool = True
    clip_norm: bool = True
    max_norm: float = 4.0
    min_level_db: float = -100
    ref_level_db: float = 20
    sample_rate: int = 22050
    mel_mean: Optional[np.ndarray] = None  # mel_scaler.mean_ (float64 in the reference's stats file)
    mel_std: Optional[np.ndarray] = None   # mel_scaler.scale_

    @classmethod
    def from_config(cls, audio: dict, mel_mean=None, mel_std=None) -> "AudioNorm":
        keys = ("signal_norm", "symmetric_norm", "clip_norm", "max_norm", "min_level_db", "ref_level_db",
                "sample_rate")
        return cls(**{k: audio[k] for k in keys if k in audio}, mel_mean=mel_mean, mel_std=mel_std)

    def _native(self, device: torch.device):
        c = N.TtsAudioNormCfg()
        c.signal_norm = 1 if self.signal_norm else 0
        c.symmetric_norm = 1 if self.symmetric_norm else 0
        c.clip_norm = 1 if self.clip_norm else 0
        c.max_norm = float(self.max_norm)
        c.min_level_db = float(self.min_level_db)
        c.ref_level_db = float(self.ref_level_db)
        keep = []
        if self.mel_mean is not None:
            mean = torch.as_tensor(np.asarray(self.mel_mean, np.float64), device=device)
            std = torch.as_tensor(np.asarray(self.mel_std, np.float64), device=device)
            c.d_mel_mean, c.d_mel_scale = mean.data_ptr(), std.data_ptr()
            keep = [mean, std]
        return c, keep


def mel_handoff(model_outputs: torch.Tensor, tts_audio: Optional[AudioNorm], vocoder_audio: Optional[AudioNorm],
                time_major: bool = True, scale_factor: Optional[float] = None) -> torch.Tensor:
    """synthesizer.py:414-428 for a batch: [B, T, C] (time_major) or [B, C, T] -> vocoder input [B, C, T'].
    ``scale_factor``: resample the time axis like F.interpolate(mode="linear", scale_factor=...) (no
    recompute_scale_factor), e.g. the XTTS latent upsampling; overrides the sample-rate rule."""
    N.require_device_tensor(model_outputs, "model_outputs")
    x = model_outputs.to(torch.float32).contiguous()
    if time_major:
        B, T, C = x.shape
    else:
        B, C, T = x.shape
    T_out = T
    if tts_audio is not None and vocoder_audio is not None and vocoder_audio.sample_rate != tts_audio.sample_rate:
        # interpolate_vocoder_input (vocoder/utils/generic_utils.py:24-27): output size floor(T * scale)
        T_out = int(math.floor(T * (vocoder_audio.sample_rate / tts_audio.sample_rate)))
    src_scale = 0.0
    if scale_factor is not None:
        T_out = int(math.floor(T * float(scale_factor)))
        src_scale = 1.0 / float(scale_factor)
    dev = x.device
    de, k1 = tts_audio._native(dev) if tts_audio is not None else (None, [])
    no, k2 = vocoder_audio._native(dev) if vocoder_audio is not None else (None, [])
    out = torch.empty(B, C, T_out, device=dev)
    N.call("tts_mel_handoff", N.ptr(x), B, T, C, 1 if time_major else 0, ctypes.byref(de) if de else None,
           ctypes.byref(no) if no else None, T_out, src_scale, N.ptr(out), N.stream_ptr(dev))
    del k1, k2  # the statistics are read by the kernel before the stream moves on (stream-ordered frees)
    return out


def wav_to_int16(wav: torch.Tensor, lengths: Optional[torch.Tensor] = None) -> torch.Tensor:
    """save_wav's scaling (numpy_transforms.py:436-438) per utterance: wav [B, n] or [B, 1, n] -> int16 [B, n]."""
    N.require_device_tensor(wav, "wav")
    w = wav.to(torch.float32).reshape(wav.shape[0], -1).contiguous()
    B, n = w.shape
    dev = w.device
    out = torch.empty(B, n, dtype=torch.int16, device=dev)
    scratch = torch.empty(B, dtype=torch.int32, device=dev)
    lens = None if lengths is None else lengths.to(device=dev, dtype=torch.int64).contiguous()
    N.call("tts_wav_to_int16", N.ptr(w), B, n, N.ptr(lens), N.ptr(scratch), N.ptr(out), N.stream_ptr(dev))
    return out


def save_wav(wav: torch.Tensor, path: str, sample_rate: int, length: Optional[int] = None) -> None:
    """numpy_transforms.save_wav for one utterance: int16 scaling on the device, file write on the host."""
    import scipy.io.wavfile

    w = wav.reshape(1, -1)
    if length is not None:
        w = w[:, :length]
    pcm = wav_to_int16(w).cpu().numpy()[0]
    scipy.io.wavfile.write(path, sample_rate, pcm)


class Synthesizer:
    """Batched acoustic model -> hand-off -> vocoder, all on one device (synthesizer.py:410-434 without
    the text frontend).  ``tts_model`` has the GlowTTS ``inference(x, aux_input)`` surface,
    ``vocoder_model`` the HifiganGenerator ``inference(c)`` surface."""

    def __init__(self, tts_model, vocoder_model, tts_audio: Optional[AudioNorm] = None,
                 vocoder_audio: Optional[AudioNorm] = None):
        self.tts_model = tts_model
        self.vocoder_model = vocoder_model
        self.tts_audio = tts_audio
        self.vocoder_audio = vocoder_audio

    @torch.no_grad()
    def tts_batch(self, token_ids: torch.Tensor, lengths: torch.Tensor):
        """token ids [B, T_x] + lengths [B] -> (wav [B, 1, n] fp32 on the device, mel [B, C, T'])."""
        out = self.tts_model.inference(token_ids, {"x_lengths": lengths})
        voc_in = mel_handoff(out["model_outputs"], self.tts_audio, self.vocoder_audio, time_major=True)
        return self.vocoder_model.inference(voc_in), voc_in


__all__ = ["AudioNorm", "Synthesizer", "mel_handoff", "save_wav", "wav_to_int16"]
