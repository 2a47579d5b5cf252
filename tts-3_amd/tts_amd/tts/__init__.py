"""Acoustic-model surface: the Glow-TTS ``Encoder`` / ``Decoder`` (both directions) /
``GlowTTS.inference`` / ``GlowTTS.decoder_inference``, and the VITS ``ResidualCouplingBlocks`` flow
(both directions) and ``PosteriorEncoder``, on MI355X."""
from .glow_decoder import Decoder
from .glow_tts import Encoder, GlowTTS
from .vits_flow import PosteriorEncoder, ResidualCouplingBlocks
from .xtts_decoder import HifiDecoder

__all__ = ["Decoder", "Encoder", "GlowTTS", "HifiDecoder", "PosteriorEncoder", "ResidualCouplingBlocks"]
