"""Drop-in VITS ``ResidualCouplingBlocks`` whose reverse (inference) flow runs in ``libtts_mi355x.so``.

Mirrors ``TTS/tts/layers/vits/networks.py`` (Coqui TTS 0.22.0): same constructor (:169-202),
same parameter tree (``flows.{i}.pre``, ``flows.{i}.enc.in_layers.*`` / ``res_skip_layers.*`` /
``cond_layer`` (weight-normed), ``flows.{i}.post``), so VITS checkpoints load unchanged.
``forward(x, x_mask, g=None, reverse=True)`` returns the flowed tensor like the reference
(:217-232, called by ``Vits.inference`` at vits.py:1156); the training direction raises.

VITS never removes its weight norm (vits.py has no remove_weight_norm call), so the reference
evaluates ``g * v / ||v||`` every forward in the module dtype; the wrapper folds it once with
PyTorch's own ``_weight_norm`` in fp32 (bit-identical to the fp32 module) and rebuilds the handle
when a parameter changes.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import numpy as np
import torch
from torch import nn

from .. import _native as N
from .glow_decoder import WN, _t


def _folded(m: nn.Module) -> np.ndarray:
    with torch.no_grad():
        return np.ascontiguousarray(m.weight.detach().to("cpu", torch.float32).numpy())


class ResidualCouplingBlock(nn.Module):
    """networks.py:103-166 (parameters only; mean_only=True as VITS builds it, :213)."""

    def __init__(self, channels, hidden_channels, kernel_size, dilation_rate, num_layers, dropout_p=0,
                 cond_channels=0, mean_only=False):
        assert channels % 2 == 0, "channels should be divisible by 2"
        super().__init__()
        self.half_channels = channels // 2
        self.mean_only = mean_only
        self.pre = nn.Conv1d(self.half_channels, hidden_channels, 1)
        self.enc = WN(hidden_channels, hidden_channels, kernel_size, dilation_rate, num_layers, dropout_p=dropout_p,
                      c_in_channels=cond_channels)
        self.post = nn.Conv1d(hidden_channels, self.half_channels * (2 - mean_only), 1)
        self.post.weight.data.zero_()
        self.post.bias.data.zero_()


class ResidualCouplingBlocks(nn.Module):
    def __init__(self, channels: int, hidden_channels: int, kernel_size: int, dilation_rate: int, num_layers: int,
                 num_flows=4, cond_channels=0, math_mode: Optional[str] = None):
        super().__init__()
        if math_mode is None:
            math_mode = N.default_math_mode()
        if math_mode not in N.MATH_MODES:
            raise ValueError(f"math_mode must be one of {sorted(N.MATH_MODES)}")
        self.math_mode = math_mode
        self.channels = channels
        self.hidden_channels = hidden_channels
        self.kernel_size = kernel_size
        self.dilation_rate = dilation_rate
        self.num_layers = num_layers
        self.num_flows = num_flows
        self.cond_channels = cond_channels
        self.flows = nn.ModuleList()
        for _ in range(num_flows):
            self.flows.append(ResidualCouplingBlock(channels, hidden_channels, kernel_size, dilation_rate, num_layers,
                                                    cond_channels=cond_channels, mean_only=True))
        c = N.TtsVitsFlowCfg()
        c.channels = channels
        c.hidden_channels = hidden_channels
        c.kernel_size = kernel_size
        c.dilation_rate = dilation_rate
        c.num_layers = num_layers
        c.num_flows = num_flows
        c.cond_channels = cond_channels
        c.math_mode = N.MATH_MODES[math_mode]
        self._cfg = c
        self._handle = None
        self._handle_key = None
        n = N.lib().tts_vits_flow_num_weights(ctypes.byref(c))
        if n < 0:
            N.check("tts_vits_flow_num_weights", -n)

    # ------------------------------------------------------------------ native handle
    def _weight_list(self) -> List[np.ndarray]:
        ws: List[np.ndarray] = []
        for fl in self.flows:
            ws += [_folded(fl.pre).reshape(-1), _t(fl.pre.bias)]
            for l in range(self.num_layers):
                ws += [_folded(fl.enc.in_layers[l]), _t(fl.enc.in_layers[l].bias)]
            for l in range(self.num_layers):
                ws += [_folded(fl.enc.res_skip_layers[l]), _t(fl.enc.res_skip_layers[l].bias)]
            if self.cond_channels > 0:
                ws += [_folded(fl.enc.cond_layer), _t(fl.enc.cond_layer.bias)]
            ws += [_folded(fl.post).reshape(-1), _t(fl.post.bias)]
        return [np.ascontiguousarray(w, dtype=np.float32) for w in ws]

    def _param_key(self):
        return tuple((p.data_ptr(), p._version, p.device) for p in self.parameters())

    def _device(self) -> torch.device:
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("ResidualCouplingBlocks (tts_amd) runs only on a ROCm device: move it with .to('cuda')")
        return dev

    def _native_handle(self):
        key = self._param_key()
        if self._handle is not None and key == self._handle_key:
            return self._handle
        self._release()
        dev = self._device()
        ws = self._weight_list()
        lib = N.lib()
        for i, w in enumerate(ws):
            n = lib.tts_vits_flow_weight_numel(ctypes.byref(self._cfg), i)
            if n != w.size:
                raise ValueError(f"weight {i} has {w.size} elements, expected {n}")
        arr = (ctypes.c_void_p * len(ws))(*[w.ctypes.data for w in ws])
        h = ctypes.c_void_p()
        N.call("tts_vits_flow_create", ctypes.byref(self._cfg), arr, dev.index or 0, ctypes.byref(h))
        self._handle, self._handle_key = h, key
        return h

    def _release(self):
        if getattr(self, "_handle", None) is not None:
            N.lib().tts_vits_flow_destroy(self._handle)
            self._handle = None
            self._handle_key = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    def _apply(self, fn, *args, **kwargs):
        self._release()
        return super()._apply(fn, *args, **kwargs)

    def _inputs(self, x, x_mask, g):
        dev = self._device()
        x = x.to(device=dev, dtype=torch.float32).contiguous()
        B, C, T = x.shape
        if x_mask is None:
            x_mask = torch.ones(B, 1, T, device=dev)
        m = x_mask.to(device=dev, dtype=torch.float32).reshape(B, T).contiguous()
        gg = None
        if self.cond_channels > 0:
            if g is None:
                raise ValueError("this flow is speaker-conditioned (cond_channels > 0): pass g [B, cond_channels, 1]")
            gg = g.to(device=dev, dtype=torch.float32).reshape(B, self.cond_channels).contiguous()
        return dev, x, m, gg

    # ------------------------------------------------------------------ reference API
    def forward(self, x: torch.Tensor, x_mask: torch.Tensor, g: Optional[torch.Tensor] = None, reverse: bool = False):
        """networks.py:217-232: reverse=True is the inference direction (vits.py:1155); reverse=False
        maps a posterior latent to the prior side (voice conversion, vits.py:1226)."""
        with torch.no_grad():
            h = self._native_handle()
            dev, x, m, gg = self._inputs(x, x_mask, g)
            B, C, T = x.shape
            y = torch.empty_like(x)
            N.call("tts_vits_flow_forward", h, N.ptr(x), N.ptr(m), N.ptr(gg), B, C, T, 1 if reverse else 0, N.ptr(y),
                   N.stream_ptr(dev))
        return y

    def profile(self, x: torch.Tensor, x_mask: torch.Tensor, g: Optional[torch.Tensor] = None, reverse: bool = True):
        """One pass with a hipEvent pair around every launch: (y, [{name, flops, bytes, ms}])."""
        h = self._native_handle()
        dev, x, m, gg = self._inputs(x, x_mask, g)
        B, C, T = x.shape
        y = torch.empty_like(x)
        cap = 1024
        recs = (N.TtsLaunchRecord * cap)()
        n = ctypes.c_int(0)
        N.call("tts_vits_flow_forward_profiled", h, N.ptr(x), N.ptr(m), N.ptr(gg), B, C, T, 1 if reverse else 0, N.ptr(y),
               N.stream_ptr(dev), recs, cap, ctypes.byref(n))
        rows = [{"name": recs[i].name.decode(), "flops": recs[i].flops, "bytes": recs[i].bytes, "ms": recs[i].ms}
                for i in range(min(n.value, cap))]
        return y, rows


class PosteriorEncoder(nn.Module):
    """``TTS/tts/layers/vits/networks.py:235-288`` on MI355X: pre (1x1) -> WN (weight-normed, speaker
    cond_layer optional) -> proj (1x1) -> split [m, logs] -> z = (m + eps * exp(logs)) * mask, one
    C-ABI call (``tts_vits_posterior_forward``).  Same constructor, parameter tree and state_dict keys
    as the reference.  ``forward(x, x_lengths, g=None, noise=None)`` returns ``(z, m, logs, x_mask)``;
    ``noise`` is the standard-normal sample the reference draws with ``torch.randn_like(mean)``
    (drawn the same way on the device when not given)."""

    def __init__(self, in_channels: int, out_channels: int, hidden_channels: int, kernel_size: int,
                 dilation_rate: int, num_layers: int, cond_channels=0, math_mode: Optional[str] = None):
        super().__init__()
        if math_mode is None:
            math_mode = N.default_math_mode()
        if math_mode not in N.MATH_MODES:
            raise ValueError(f"math_mode must be one of {sorted(N.MATH_MODES)}")
        self.math_mode = math_mode
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.hidden_channels = hidden_channels
        self.kernel_size = kernel_size
        self.dilation_rate = dilation_rate
        self.num_layers = num_layers
        self.cond_channels = cond_channels
        self.pre = nn.Conv1d(in_channels, hidden_channels, 1)
        self.enc = WN(hidden_channels, hidden_channels, kernel_size, dilation_rate, num_layers, c_in_channels=cond_channels)
        self.proj = nn.Conv1d(hidden_channels, out_channels * 2, 1)
        c = N.TtsVitsPosteriorCfg()
        c.in_channels, c.out_channels, c.hidden_channels = in_channels, out_channels, hidden_channels
        c.kernel_size, c.dilation_rate, c.num_layers = kernel_size, dilation_rate, num_layers
        c.cond_channels = cond_channels
        c.math_mode = N.MATH_MODES[math_mode]
        self._cfg = c
        self._handle = None
        self._handle_key = None
        n = N.lib().tts_vits_posterior_num_weights(ctypes.byref(c))
        if n < 0:
            N.check("tts_vits_posterior_num_weights", -n)

    def _weight_list(self) -> List[np.ndarray]:
        ws = [_folded(self.pre).reshape(-1), _t(self.pre.bias)]
        for l in range(self.num_layers):
            ws += [_folded(self.enc.in_layers[l]), _t(self.enc.in_layers[l].bias)]
        for l in range(self.num_layers):
            ws += [_folded(self.enc.res_skip_layers[l]), _t(self.enc.res_skip_layers[l].bias)]
        if self.cond_channels > 0:
            ws += [_folded(self.enc.cond_layer), _t(self.enc.cond_layer.bias)]
        ws += [_folded(self.proj).reshape(-1), _t(self.proj.bias)]
        return [np.ascontiguousarray(w, dtype=np.float32) for w in ws]

    def _param_key(self):
        return tuple((p.data_ptr(), p._version, p.device) for p in self.parameters())

    def _device(self) -> torch.device:
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("PosteriorEncoder (tts_amd) runs only on a ROCm device: move it with .to('cuda')")
        return dev

    def _native_handle(self):
        key = self._param_key()
        if self._handle is not None and key == self._handle_key:
            return self._handle
        self._release()
        dev = self._device()
        ws = self._weight_list()
        lib = N.lib()
        for i, w in enumerate(ws):
            n = lib.tts_vits_posterior_weight_numel(ctypes.byref(self._cfg), i)
            if n != w.size:
                raise ValueError(f"weight {i} has {w.size} elements, expected {n}")
        arr = (ctypes.c_void_p * len(ws))(*[w.ctypes.data for w in ws])
        h = ctypes.c_void_p()
        N.call("tts_vits_posterior_create", ctypes.byref(self._cfg), arr, dev.index or 0, ctypes.byref(h))
        self._handle, self._handle_key = h, key
        return h

    def _release(self):
        if getattr(self, "_handle", None) is not None:
            N.lib().tts_vits_posterior_destroy(self._handle)
            self._handle = None
            self._handle_key = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    def _apply(self, fn, *args, **kwargs):
        self._release()
        return super()._apply(fn, *args, **kwargs)

    def _io(self, x, x_lengths, g, noise):
        dev = self._device()
        x = x.to(device=dev, dtype=torch.float32).contiguous()
        B, C, T = x.shape
        if C != self.in_channels:
            raise ValueError(f"x has {C} channels, expected {self.in_channels}")
        lens = torch.as_tensor(x_lengths, device=dev).reshape(B)
        x_mask = (torch.arange(T, device=dev)[None, :] < lens[:, None]).to(torch.float32).unsqueeze(1)  # sequence_mask
        gg = None
        if self.cond_channels > 0:
            if g is None:
                raise ValueError("this encoder is speaker-conditioned (cond_channels > 0): pass g [B, cond_channels, 1]")
            gg = g.to(device=dev, dtype=torch.float32).reshape(B, self.cond_channels).contiguous()
        elif g is not None:
            raise ValueError("g given to a PosteriorEncoder built with cond_channels=0")
        if noise is None:
            noise = torch.randn(B, self.out_channels, T, device=dev, dtype=torch.float32)  # torch.randn_like(mean)
        noise = noise.to(device=dev, dtype=torch.float32).contiguous()
        if noise.shape != (B, self.out_channels, T):
            raise ValueError(f"noise has shape {tuple(noise.shape)}, expected {(B, self.out_channels, T)}")
        return dev, x, x_mask, gg, noise

    def forward(self, x: torch.Tensor, x_lengths: torch.Tensor, g: Optional[torch.Tensor] = None,
                noise: Optional[torch.Tensor] = None):
        with torch.no_grad():
            h = self._native_handle()
            dev, x, x_mask, gg, noise = self._io(x, x_lengths, g, noise)
            B, C, T = x.shape
            z = torch.empty(B, self.out_channels, T, device=dev)
            m = torch.empty_like(z)
            logs = torch.empty_like(z)
            N.call("tts_vits_posterior_forward", h, N.ptr(x), N.ptr(x_mask), N.ptr(gg), N.ptr(noise), B, C, T,
                   N.ptr(z), N.ptr(m), N.ptr(logs), N.stream_ptr(dev))
        return z, m, logs, x_mask

    def profile(self, x, x_lengths, g=None, noise=None):
        """One pass with a hipEvent pair around every launch: (z, [{name, flops, bytes, ms}])."""
        h = self._native_handle()
        dev, x, x_mask, gg, noise = self._io(x, x_lengths, g, noise)
        B, C, T = x.shape
        z = torch.empty(B, self.out_channels, T, device=dev)
        cap = 1024
        recs = (N.TtsLaunchRecord * cap)()
        n = ctypes.c_int(0)
        N.call("tts_vits_posterior_forward_profiled", h, N.ptr(x), N.ptr(x_mask), N.ptr(gg), N.ptr(noise), B, C, T,
               N.ptr(z), None, None, N.stream_ptr(dev), recs, cap, ctypes.byref(n))
        rows = [{"name": recs[i].name.decode(), "flops": recs[i].flops, "bytes": recs[i].bytes, "ms": recs[i].ms}
                for i in range(min(n.value, cap))]
        return z, rows
