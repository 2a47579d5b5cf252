"""Drop-in XTTS waveform decoder: ``HifiDecoder`` (``TTS/tts/layers/xtts/hifigan_decoder.py:603-735``)
on the MI355X path.

``forward(latents, g)`` = the two linear latent resamplings (:688-698: x ar_mel_length_compression /
output_hop_length, then x output_sample_rate / input_sample_rate, both ``F.interpolate(mode="linear")``
with the scale factor as given) run by ``tts_mel_handoff`` with ``src_scale = 1 / scale_factor``,
then the XTTS ``HifiganGenerator`` (``cond_in_each_up_layer``: ``o = ups[i](o) + conds[i](g)``,
:276-279) run by ``tts_hifigan_forward``.  The speaker encoder (``ResNetSpeakerEncoder``, used only
to compute ``g`` from reference audio) is outside the hot path: ``g`` is an input.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from ..synthesizer import mel_handoff
from ..vocoder.hifigan_generator import HifiganGenerator


class HifiDecoder(nn.Module):
    def __init__(
        self,
        input_sample_rate=22050,
        output_sample_rate=24000,
        output_hop_length=256,
        ar_mel_length_compression=1024,
        decoder_input_dim=1024,
        resblock_type_decoder="1",
        resblock_dilation_sizes_decoder=((1, 3, 5), (1, 3, 5), (1, 3, 5)),
        resblock_kernel_sizes_decoder=(3, 7, 11),
        upsample_rates_decoder=(8, 8, 2, 2),
        upsample_initial_channel_decoder=512,
        upsample_kernel_sizes_decoder=(16, 16, 4, 4),
        d_vector_dim=512,
        cond_d_vector_in_each_upsampling_layer=True,
        speaker_encoder_audio_config=None,
        math_mode: Optional[str] = None,
    ):
        super().__init__()
        self.input_sample_rate = input_sample_rate
        self.output_sample_rate = output_sample_rate
        self.output_hop_length = output_hop_length
        self.ar_mel_length_compression = ar_mel_length_compression
        self.waveform_decoder = HifiganGenerator(
            decoder_input_dim, 1, resblock_type_decoder, [list(d) for d in resblock_dilation_sizes_decoder],
            list(resblock_kernel_sizes_decoder), list(upsample_kernel_sizes_decoder),
            upsample_initial_channel_decoder, list(upsample_rates_decoder), inference_padding=0,
            cond_channels=d_vector_dim, conv_pre_weight_norm=False, conv_post_weight_norm=False,
            conv_post_bias=False, math_mode=math_mode,
            cond_in_each_up_layer=cond_d_vector_in_each_upsampling_layer)

    @property
    def device(self):
        return next(self.parameters()).device

    def forward(self, latents: torch.Tensor, g: Optional[torch.Tensor] = None) -> torch.Tensor:
        """latents [B, T, decoder_input_dim] (GPT latents), g [B, d_vector_dim, 1] -> wav [B, 1, n]."""
        if g is None:
            raise ValueError("the XTTS decoder is speaker-conditioned: pass g (d_vector)")
        dev = self.waveform_decoder._device()
        x = latents.to(device=dev, dtype=torch.float32)
        if x.dim() == 2:
            x = x.unsqueeze(0)
        z = mel_handoff(x, None, None, time_major=True,
                        scale_factor=self.ar_mel_length_compression / self.output_hop_length)
        if self.output_sample_rate != self.input_sample_rate:
            z = mel_handoff(z, None, None, time_major=False,
                            scale_factor=self.output_sample_rate / self.input_sample_rate)
        return self.waveform_decoder(z, g=g)

    @torch.no_grad()
    def inference(self, c: torch.Tensor, g: torch.Tensor) -> torch.Tensor:  # :702-717
        return self.forward(c, g=g)

    def load_checkpoint(self, checkpoint_path, eval=False):  # :719-735 (speaker_encoder keys dropped)
        state = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        state = state["model"] if "model" in state else state
        state = {k[len("waveform_decoder."):]: v for k, v in state.items() if k.startswith("waveform_decoder.")}
        self.waveform_decoder.load_state_dict(state)
        if eval:
            self.eval()
            self.waveform_decoder.remove_weight_norm()


__all__ = ["HifiDecoder"]
