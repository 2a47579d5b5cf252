"""Acoustic-model surface: the Glow-TTS ``Decoder`` and the VITS ``ResidualCouplingBlocks`` flow
(reverse flows on MI355X)."""
from .glow_decoder import Decoder
from .vits_flow import ResidualCouplingBlocks

__all__ = ["Decoder", "ResidualCouplingBlocks"]
