"""Checkpoint loading (mirrors ``TTS/utils/io.py:27-54`` ``load_fsspec``).

Checkpoints are read with ``torch.load(..., weights_only=True)``: nothing in the file is
executed.  Coqui checkpoints hold plain tensors/dicts/numbers under ``"model"``.
"""
from __future__ import annotations

from typing import Any

import torch


def load_fsspec(path: str, map_location: Any = None, cache: bool = False, **kwargs) -> Any:
    try:
        import fsspec

        with fsspec.open(path, "rb") as f:
            return torch.load(f, map_location=map_location, weights_only=True, **kwargs)
    except ImportError:  # local files only
        with open(path, "rb") as f:
            return torch.load(f, map_location=map_location, weights_only=True, **kwargs)
