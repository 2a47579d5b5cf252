"""Vocoder surface: ``HifiganGenerator``, ``GAN`` (inference part) and ``setup_generator``
(``TTS/vocoder/models/__init__.py:34-41``)."""
from .gan import GAN, setup_generator
from .hifigan_generator import HifiganGenerator

__all__ = ["GAN", "HifiganGenerator", "setup_generator"]
