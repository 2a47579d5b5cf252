"""Shared helpers for the parity tests: golden fixtures and tolerance metrics."""
from __future__ import annotations

import glob
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# fp32-faithful parity gates vs the fp64 reference.  The reference's own fp32 CPU forward is
# max 5.6e-7 / rel-RMS 1e-6 off fp64 on HiFiGAN; the worst errors measured on
# MI355X over the whole GPU suite (profiles/parity_errors_r03.jsonl, TTS_ERRLOG) are rel-RMS 1.2e-6
# and, on bounded waveforms, max 1.7e-6.  Gates: rel-RMS 5e-6 everywhere; max|d| 1e-5 on
# waveforms / latents (|y| <= 1 or O(1)), 1e-4 on single-op outputs of unbounded magnitude
# (Winograd op tests reach 2.3e-5 on |y| ~ 30).
FP32_MAX_ABS = 1e-4
FP32_REL_RMS = 5e-6
WAV_MAX_ABS = 1e-5
# bf16 math mode (TTS_MATH_BF16, configs 3 / 5): SURVEY.md §8c's bf16 gate; the reference's own
# bf16 CPU forward measured rel-RMS 1.3e-2 and max 6.2e-3 vs fp64.  max|d|: 5e-2 on waveforms and
# flow latents (the worst measured in the round-5 log is 0.027, profiles/parity_errors_r05.jsonl),
# 1e-1 on unbounded outputs (single ops, the posterior's z = m + eps * exp(logs): 0.060)
BF16_MAX_ABS = 5e-2
BF16_MAX_ABS_OP = 1e-1
BF16_REL_RMS = 3e-2


def tol(mode: str, op: bool = False) -> dict:
    """Parity gates of a math mode (every mode but bf16 is held to the fp32 gates); ``op``:
    a single conv's output (magnitude not bounded like a waveform's)."""
    if mode == "bf16":
        return dict(max_abs_tol=BF16_MAX_ABS_OP if op else BF16_MAX_ABS, rel_rms_tol=BF16_REL_RMS)
    return dict(max_abs_tol=FP32_MAX_ABS if op else WAV_MAX_ABS, rel_rms_tol=FP32_REL_RMS)


def goldens(kind: str):
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))):
        with np.load(p, allow_pickle=False) as z:
            meta = json.loads(str(z["meta"]))
            if meta["kind"] == kind:
                out.append((os.path.basename(p)[:-4], meta, {k: z[k] for k in z.files if k != "meta"}))
    return out


def rel_rms(a, b) -> float:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(np.sqrt(np.mean(b**2)), 1e-30))


def max_abs(a, b) -> float:
    return float(np.max(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64))))


def hifigan_ctor(cfg: dict) -> dict:
    keys = ["in_channels", "out_channels", "resblock_type", "resblock_dilation_sizes", "resblock_kernel_sizes",
            "upsample_kernel_sizes", "upsample_initial_channel", "upsample_factors", "inference_padding",
            "cond_channels", "conv_pre_weight_norm", "conv_post_weight_norm", "conv_post_bias"]
    return {k: cfg[k] for k in keys if k in cfg}


def log_error(what: str, ma: float, rr: float, max_abs_tol=None, rel_rms_tol=None) -> None:
    """TTS_ERRLOG=<path>: append every measured parity error (JSON lines) - the record the gates
    below are calibrated from (profiles/parity_errors_r03.jsonl)."""
    path = os.environ.get("TTS_ERRLOG")
    if path:
        with open(path, "a") as fh:
            fh.write(json.dumps({"what": what, "max_abs": ma, "rel_rms": rr, "max_abs_tol": max_abs_tol,
                                 "rel_rms_tol": rel_rms_tol}) + "\n")


def assert_close_fp32(out, ref64, what: str, max_abs_tol=FP32_MAX_ABS, rel_rms_tol=FP32_REL_RMS):
    out = out.detach().cpu().numpy() if isinstance(out, torch.Tensor) else out
    ref64 = ref64.detach().cpu().numpy() if isinstance(ref64, torch.Tensor) else ref64
    assert out.shape == ref64.shape, f"{what}: shape {out.shape} vs {ref64.shape}"
    assert np.isfinite(out).all(), f"{what}: non-finite output"
    ma, rr = max_abs(out, ref64), rel_rms(out, ref64)
    log_error(what, ma, rr, max_abs_tol, rel_rms_tol)
    assert ma <= max_abs_tol and rr <= rel_rms_tol, f"{what}: max|d|={ma:.3e} (tol {max_abs_tol}), rel-RMS={rr:.3e} (tol {rel_rms_tol})"
    return ma, rr
