"""Configuration defaults of the two reference modules this package replaces, and a plain
JSON reader (no coqpit dependency).

* ``HIFIGAN_V1``: ``HifiganConfig.generator_model_params`` (TTS/vocoder/configs/hifigan_config.py:95-104)
* ``GLOW_TTS_DECODER``: the decoder fields of ``GlowTTSConfig`` (TTS/tts/configs/glow_tts_config.py:117-131)
* ``GLOW_TTS_ENCODER``: the encoder fields of ``GlowTTSConfig`` (glow_tts_config.py:103-124) as
  ``GlowTTS.__init__`` hands them to ``Encoder`` (TTS/tts/models/glow_tts.py:80-91)
* ``VITS_FLOW`` / ``VITS_DECODER``: the flow and waveform-decoder fields of ``VitsArgs``
  (TTS/tts/models/vits.py:545-565, built at :675-682 and :704-718)
* ``VITS_TEXT_ENCODER`` / ``VITS_SDP`` / ``VITS_INFERENCE``: the text side of ``Vits.inference``
  (vits.py:653-692, :1088-1174)
"""
from __future__ import annotations

import json
from typing import Any, Dict

HIFIGAN_V1: Dict[str, Any] = {
    "upsample_factors": [8, 8, 2, 2],
    "upsample_kernel_sizes": [16, 16, 4, 4],
    "upsample_initial_channel": 512,
    "resblock_kernel_sizes": [3, 7, 11],
    "resblock_dilation_sizes": [[1, 3, 5], [1, 3, 5], [1, 3, 5]],
    "resblock_type": "1",
}

GLOW_TTS_DECODER: Dict[str, Any] = {
    "in_channels": 80,          # out_channels
    "hidden_channels": 192,     # hidden_channels_dec
    "kernel_size": 5,           # kernel_size_dec
    "dilation_rate": 1,
    "num_flow_blocks": 12,      # num_flow_blocks_dec
    "num_coupling_layers": 4,   # num_block_layers
    "dropout_p": 0.05,          # dropout_p_dec (identity at inference)
    "num_splits": 4,
    "num_squeeze": 2,
    "sigmoid_scale": False,
    "c_in_channels": 0,
}

GLOW_TTS_ENCODER: Dict[str, Any] = {
    "out_channels": 80,
    "hidden_channels": 192,     # hidden_channels_enc
    "hidden_channels_dp": 256,
    "encoder_type": "rel_pos_transformer",
    "encoder_params": {"kernel_size": 3, "dropout_p": 0.1, "num_layers": 6, "num_heads": 2,
                       "hidden_channels_ffn": 768},
    "dropout_p_dp": 0.1,
    "mean_only": True,
    "use_prenet": True,         # use_encoder_prenet
    "c_in_channels": 0,
}

# GlowTTS.inference glue (glow_tts.py:342-363): GlowTTSConfig defaults.  The dataclass declares
# inference_noise_scale twice (glow_tts_config.py:124 = 0.33, :151 = 0.0); the later one wins.
GLOW_TTS_INFERENCE: Dict[str, Any] = {"length_scale": 1.0, "inference_noise_scale": 0.0}

VITS_FLOW: Dict[str, Any] = {
    "channels": 192,            # hidden_channels
    "hidden_channels": 192,
    "kernel_size": 5,           # kernel_size_flow
    "dilation_rate": 1,         # dilation_rate_flow
    "num_layers": 4,            # num_layers_flow
    "num_flows": 4,
}

# PosteriorEncoder of VitsArgs (vits.py:594-602): the linear spectrogram (fft_size 1024 -> 513 bins)
VITS_POSTERIOR: Dict[str, Any] = {
    "in_channels": 513,         # out_channels (fft_size // 2 + 1)
    "out_channels": 192,        # hidden_channels
    "hidden_channels": 192,
    "kernel_size": 5,           # kernel_size_posterior_encoder
    "dilation_rate": 1,         # dilation_rate_posterior_encoder
    "num_layers": 16,           # num_layers_posterior_encoder
}

# TextEncoder of VitsArgs (vits.py:653-663; networks.py:29-81): n_vocab = num_chars,
# out = hidden = hidden_channels
VITS_TEXT_ENCODER: Dict[str, Any] = {
    "out_channels": 192,        # hidden_channels
    "hidden_channels": 192,
    "hidden_channels_ffn": 768,  # hidden_channels_ffn_text_encoder
    "num_heads": 2,             # num_heads_text_encoder
    "num_layers": 6,            # num_layers_text_encoder
    "kernel_size": 3,           # kernel_size_text_encoder
}

# StochasticDurationPredictor of VitsArgs (vits.py:684-692): in = hidden_channels, 192 hidden, k3, 4 flows
VITS_SDP: Dict[str, Any] = {"in_channels": 192, "hidden_channels": 192, "kernel_size": 3, "num_flows": 4}

# Vits.inference scalars (VitsArgs, vits.py:569-572)
VITS_INFERENCE: Dict[str, Any] = {"inference_noise_scale": 0.667, "length_scale": 1.0, "inference_noise_scale_dp": 1.0}

VITS_DECODER: Dict[str, Any] = {
    "in_channels": 192,
    "out_channels": 1,
    "resblock_type": "1",
    "resblock_dilation_sizes": [[1, 3, 5], [1, 3, 5], [1, 3, 5]],
    "resblock_kernel_sizes": [3, 7, 11],
    "upsample_kernel_sizes": [16, 16, 4, 4],
    "upsample_initial_channel": 512,
    "upsample_factors": [8, 8, 2, 2],
    "inference_padding": 0,
    "conv_pre_weight_norm": False,
    "conv_post_weight_norm": False,
    "conv_post_bias": False,
}


def load_config(path: str) -> Dict[str, Any]:
    """Read a Coqui JSON config (``TTS/config/__init__.py:68-100`` reads the same files)."""
    with open(path, "r", encoding="utf-8") as f:
        return json.load(f)
