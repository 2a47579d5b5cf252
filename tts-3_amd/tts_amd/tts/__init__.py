"""Acoustic-model surface: the Glow-TTS ``Decoder`` (reverse flow on MI355X)."""
from .glow_decoder import Decoder

__all__ = ["Decoder"]
