"""Acoustic-model surface: the Glow-TTS ``Encoder`` / ``Decoder`` (both directions) /
``GlowTTS.inference`` / ``GlowTTS.decoder_inference``, and the VITS ``ResidualCouplingBlocks`` flow
(both directions), ``PosteriorEncoder`` and the text side of ``Vits.inference`` (``TextEncoder``,
``StochasticDurationPredictor``, ``Vits``), on MI355X."""
from .glow_decoder import Decoder
from .glow_tts import Encoder, GlowTTS
from .vits_flow import PosteriorEncoder, ResidualCouplingBlocks
from .vits_text import DurationPredictor, StochasticDurationPredictor, TextEncoder, Vits
from .xtts_decoder import HifiDecoder

__all__ = ["Decoder", "DurationPredictor", "Encoder", "GlowTTS", "HifiDecoder", "PosteriorEncoder", "ResidualCouplingBlocks",
           "StochasticDurationPredictor", "TextEncoder", "Vits"]
