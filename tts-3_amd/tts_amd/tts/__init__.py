"""Acoustic-model surface: the Glow-TTS ``Encoder`` / ``Decoder`` / ``GlowTTS.inference`` and the
VITS ``ResidualCouplingBlocks`` flow, on MI355X."""
from .glow_decoder import Decoder
from .glow_tts import Encoder, GlowTTS
from .vits_flow import ResidualCouplingBlocks
from .xtts_decoder import HifiDecoder

__all__ = ["Decoder", "Encoder", "GlowTTS", "HifiDecoder", "ResidualCouplingBlocks"]
