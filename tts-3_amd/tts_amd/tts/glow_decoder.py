"""Drop-in Glow-TTS ``Decoder`` whose reverse (inference) flow runs in ``libtts_mi355x.so``.

Mirrors ``TTS/tts/layers/glow_tts/decoder.py`` (Coqui TTS 0.22.0): same constructor
(:68-81), same parameter tree (``flows.{3b}`` ActNorm ``logs``/``bias``, ``flows.{3b+1}``
InvConvNear ``weight`` (+``weight_inv`` after ``store_inverse``), ``flows.{3b+2}`` CouplingBlock
``start`` (weight-normed), ``end``, ``wn.in_layers.*`` / ``wn.res_skip_layers.*``, and
``wn.cond_layer`` when ``c_in_channels > 0``), so reference checkpoints load unchanged.
``forward(x, x_mask, g=None, reverse=True)`` returns ``(y, None)`` like the reference (:113-137);
``g`` ([B, c_in_channels, 1]) is the speaker vector every flow's WN projects with its own
``cond_layer`` and adds to its in_layer outputs (wavenet.py:98-107).  The training direction
(``reverse=False``, log-determinants) is out of scope and raises.

The nn modules below only hold parameters.  Weight norm is folded with PyTorch's own
``_weight_norm`` and InvConvNear's inverse is ``torch.inverse(weight.float())`` exactly as
``store_inverse`` (glow.py:139-141) computes it; both are handed to
``tts_glow_decoder_create`` once and the handle is rebuilt when any parameter changes.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import numpy as np
import torch
from torch import nn
from torch.nn.utils.parametrizations import weight_norm
from torch.nn.utils.parametrize import is_parametrized, remove_parametrizations

from .. import _native as N


class ActNorm(nn.Module):
    """normalization.py:66-123 (parameters only)."""

    def __init__(self, channels: int, ddi: bool = False, **kwargs):
        super().__init__()
        self.channels = channels
        self.initialized = not ddi
        self.logs = nn.Parameter(torch.zeros(1, channels, 1))
        self.bias = nn.Parameter(torch.zeros(1, channels, 1))

    def store_inverse(self):
        pass


class InvConvNear(nn.Module):
    """glow.py:70-141 (parameters only)."""

    def __init__(self, channels: int, num_splits: int = 4, no_jacobian: bool = False, **kwargs):
        super().__init__()
        assert num_splits % 2 == 0
        self.channels = channels
        self.num_splits = num_splits
        self.no_jacobian = no_jacobian
        self.weight_inv = None
        w_init = torch.linalg.qr(torch.FloatTensor(num_splits, num_splits).normal_(), "complete")[0]
        if torch.det(w_init) < 0:
            w_init[:, 0] = -1 * w_init[:, 0]
        self.weight = nn.Parameter(w_init)

    def inverse_weight(self) -> torch.Tensor:
        if self.weight_inv is not None:
            return self.weight_inv
        return torch.inverse(self.weight.float()).to(dtype=self.weight.dtype)  # glow.py:123

    def store_inverse(self):  # glow.py:139-141
        weight_inv = torch.inverse(self.weight.float()).to(dtype=self.weight.dtype)
        self.weight_inv = nn.Parameter(weight_inv, requires_grad=False)


class WN(nn.Module):
    """wavenet.py:16-123 (parameters only).  ``cond_layer`` (c_in_channels > 0) is registered after
    ``dropout`` as in the reference, so state_dict keys and order match."""

    def __init__(self, in_channels, hidden_channels, kernel_size, dilation_rate, num_layers, c_in_channels=0,
                 dropout_p=0, weight_norm_=True):
        super().__init__()
        assert kernel_size % 2 == 1
        assert hidden_channels % 2 == 0
        self.in_channels = in_channels
        self.hidden_channels = hidden_channels
        self.kernel_size = kernel_size
        self.dilation_rate = dilation_rate
        self.num_layers = num_layers
        self.c_in_channels = c_in_channels
        self.dropout_p = dropout_p
        self.in_layers = nn.ModuleList()
        self.res_skip_layers = nn.ModuleList()
        self.dropout = nn.Dropout(dropout_p)
        if c_in_channels > 0:
            self.cond_layer = weight_norm(nn.Conv1d(c_in_channels, 2 * hidden_channels * num_layers, 1), name="weight")
        for i in range(num_layers):
            dilation = dilation_rate**i
            padding = int((kernel_size * dilation - dilation) / 2)
            cin = in_channels if i == 0 else hidden_channels
            self.in_layers.append(weight_norm(nn.Conv1d(cin, 2 * hidden_channels, kernel_size, dilation=dilation,
                                                        padding=padding), name="weight"))
            rsc = 2 * hidden_channels if i < num_layers - 1 else hidden_channels
            self.res_skip_layers.append(weight_norm(nn.Conv1d(hidden_channels, rsc, 1), name="weight"))

    def remove_weight_norm(self):  # wavenet.py:117-123
        extra = [self.cond_layer] if self.c_in_channels > 0 else []
        for l in extra + list(self.in_layers) + list(self.res_skip_layers):
            if is_parametrized(l, "weight"):
                remove_parametrizations(l, "weight")


class CouplingBlock(nn.Module):
    """glow.py:144-233 (parameters only)."""

    def __init__(self, in_channels, hidden_channels, kernel_size, dilation_rate, num_layers, c_in_channels=0,
                 dropout_p=0, sigmoid_scale=False):
        super().__init__()
        self.in_channels = in_channels
        self.hidden_channels = hidden_channels
        self.sigmoid_scale = sigmoid_scale
        start = nn.Conv1d(in_channels // 2, hidden_channels, 1)
        self.start = weight_norm(start)
        end = nn.Conv1d(hidden_channels, in_channels, 1)
        end.weight.data.zero_()
        end.bias.data.zero_()
        self.end = end
        self.wn = WN(hidden_channels, hidden_channels, kernel_size, dilation_rate, num_layers, c_in_channels,
                     dropout_p)

    def store_inverse(self):  # glow.py:232-233 (start keeps its weight norm)
        self.wn.remove_weight_norm()


def _w(m: nn.Module) -> np.ndarray:
    with torch.no_grad():
        return np.ascontiguousarray(m.weight.detach().to("cpu", torch.float32).numpy())


def _t(t: torch.Tensor) -> np.ndarray:
    return np.ascontiguousarray(t.detach().to("cpu", torch.float32).numpy())


class Decoder(nn.Module):
    def __init__(self, in_channels, hidden_channels, kernel_size, dilation_rate, num_flow_blocks,
                 num_coupling_layers, dropout_p=0.0, num_splits=4, num_squeeze=2, sigmoid_scale=False,
                 c_in_channels=0, math_mode: Optional[str] = None):
        super().__init__()
        if math_mode is None:
            math_mode = N.default_math_mode()
        if math_mode not in N.MATH_MODES:
            raise ValueError(f"math_mode must be one of {sorted(N.MATH_MODES)}")
        self.math_mode = math_mode
        self.in_channels = in_channels
        self.hidden_channels = hidden_channels
        self.kernel_size = kernel_size
        self.dilation_rate = dilation_rate
        self.num_flow_blocks = num_flow_blocks
        self.num_coupling_layers = num_coupling_layers
        self.dropout_p = dropout_p
        self.num_splits = num_splits
        self.num_squeeze = num_squeeze
        self.sigmoid_scale = sigmoid_scale
        self.c_in_channels = c_in_channels
        self.flows = nn.ModuleList()
        for _ in range(num_flow_blocks):
            self.flows.append(ActNorm(channels=in_channels * num_squeeze))
            self.flows.append(InvConvNear(channels=in_channels * num_squeeze, num_splits=num_splits))
            self.flows.append(CouplingBlock(in_channels * num_squeeze, hidden_channels, kernel_size=kernel_size,
                                            dilation_rate=dilation_rate, num_layers=num_coupling_layers,
                                            c_in_channels=c_in_channels, dropout_p=dropout_p,
                                            sigmoid_scale=sigmoid_scale))
        c = N.TtsGlowDecoderCfg()
        c.in_channels = in_channels
        c.hidden_channels = hidden_channels
        c.kernel_size = kernel_size
        c.dilation_rate = dilation_rate
        c.num_flow_blocks = num_flow_blocks
        c.num_coupling_layers = num_coupling_layers
        c.num_splits = num_splits
        c.num_squeeze = num_squeeze
        c.sigmoid_scale = 1 if sigmoid_scale else 0
        c.c_in_channels = c_in_channels
        c.math_mode = N.MATH_MODES[math_mode]
        self._cfg = c
        self._handle = None
        self._handle_key = None
        n = N.lib().tts_glow_decoder_num_weights(ctypes.byref(c))
        if n < 0:
            N.check("tts_glow_decoder_num_weights", -n)

    # ------------------------------------------------------------------ native handle
    def _weight_list(self) -> List[np.ndarray]:
        ws: List[np.ndarray] = []
        for b in range(self.num_flow_blocks):
            an, ic, cb = self.flows[3 * b], self.flows[3 * b + 1], self.flows[3 * b + 2]
            ws += [_t(an.logs).reshape(-1), _t(an.bias).reshape(-1), _t(ic.inverse_weight()), _t(ic.weight)]
            ws += [_w(cb.start), _t(cb.start.bias)]
            if self.c_in_channels > 0:
                ws += [_w(cb.wn.cond_layer).reshape(-1), _t(cb.wn.cond_layer.bias)]
            for l in range(self.num_coupling_layers):
                ws += [_w(cb.wn.in_layers[l]), _t(cb.wn.in_layers[l].bias)]
                ws += [_w(cb.wn.res_skip_layers[l]), _t(cb.wn.res_skip_layers[l].bias)]
            ws += [_w(cb.end), _t(cb.end.bias)]
        return [np.ascontiguousarray(w) for w in ws]

    def _param_key(self):
        key = [(p.data_ptr(), p._version, p.device) for p in self.parameters()]
        return tuple(key)

    def _device(self) -> torch.device:
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("Decoder (tts_amd) runs only on a ROCm device: move it with .to('cuda') first")
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
            n = lib.tts_glow_decoder_weight_numel(ctypes.byref(self._cfg), i)
            if n != w.size:
                raise ValueError(f"weight {i} has {w.size} elements, expected {n}")
        arr = (ctypes.c_void_p * len(ws))(*[w.ctypes.data for w in ws])
        h = ctypes.c_void_p()
        N.call("tts_glow_decoder_create", ctypes.byref(self._cfg), arr, dev.index or 0, ctypes.byref(h))
        self._handle, self._handle_key = h, key
        return h

    def _release(self):
        if getattr(self, "_handle", None) is not None:
            N.lib().tts_glow_decoder_destroy(self._handle)
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

    # ------------------------------------------------------------------ reference API
    def _speaker(self, g: Optional[torch.Tensor], B: int, dev: torch.device) -> Optional[torch.Tensor]:
        """g [B, c_in, 1] (or [B, c_in]) -> contiguous fp32 [B, c_in] on the device; None when unconditioned."""
        if self.c_in_channels == 0:
            if g is not None:
                raise ValueError("g given to a Decoder built with c_in_channels=0 (it has no cond_layer)")
            return None
        if g is None:
            raise ValueError(f"this Decoder is speaker-conditioned (c_in_channels={self.c_in_channels}): pass g")
        g = g.to(device=dev, dtype=torch.float32).reshape(g.shape[0], -1).contiguous()
        if g.shape != (B, self.c_in_channels):
            raise ValueError(f"g has shape {tuple(g.shape)}, expected [{B}, {self.c_in_channels}, 1]")
        return g

    def forward(self, x: torch.Tensor, x_mask: torch.Tensor, g: Optional[torch.Tensor] = None, reverse: bool = False):
        """decoder.py:113-137: (y, None) for reverse=True (inference), (z, logdet [B]) for reverse=False
        (GlowTTS.decoder_inference's first pass, glow_tts.py:333)."""
        with torch.no_grad():
            h = self._native_handle()
            dev = self._device()
            x = x.to(device=dev, dtype=torch.float32).contiguous()
            B, C, T = x.shape
            if x_mask is None:
                x_mask = torch.ones(B, 1, T, device=dev)
            m = x_mask.to(device=dev, dtype=torch.float32).reshape(B, T).contiguous()
            gv = self._speaker(g, B, dev)
            Tq = (T // self.num_squeeze) * self.num_squeeze if self.num_squeeze > 1 else T
            y = torch.empty(B, C, Tq, device=dev, dtype=torch.float32)
            logdet = None if reverse else torch.empty(B, device=dev, dtype=torch.float32)
            N.call("tts_glow_decoder_forward", h, N.ptr(x), N.ptr(m), N.ptr(gv), B, C, T, 1 if reverse else 0,
                   N.ptr(y), N.ptr(logdet), N.stream_ptr(dev))
        return y, logdet

    def profile(self, x: torch.Tensor, x_mask: torch.Tensor, g: Optional[torch.Tensor] = None, reverse: bool = True):
        """One pass with a hipEvent pair around every launch: (y, [{name, flops, bytes, ms}])."""
        h = self._native_handle()
        dev = self._device()
        x = x.to(device=dev, dtype=torch.float32).contiguous()
        B, C, T = x.shape
        m = x_mask.to(device=dev, dtype=torch.float32).reshape(B, T).contiguous()
        gv = self._speaker(g, B, dev)
        Tq = (T // self.num_squeeze) * self.num_squeeze if self.num_squeeze > 1 else T
        y = torch.empty(B, C, Tq, device=dev)
        logdet = None if reverse else torch.empty(B, device=dev, dtype=torch.float32)
        cap = 2048
        recs = (N.TtsLaunchRecord * cap)()
        n = ctypes.c_int(0)
        N.call("tts_glow_decoder_forward_profiled", h, N.ptr(x), N.ptr(m), N.ptr(gv), B, C, T, 1 if reverse else 0,
               N.ptr(y), N.ptr(logdet), N.stream_ptr(dev), recs, cap, ctypes.byref(n))
        rows = [{"name": recs[i].name.decode(), "flops": recs[i].flops, "bytes": recs[i].bytes, "ms": recs[i].ms}
                for i in range(min(n.value, cap))]
        return y, rows

    def store_inverse(self):  # decoder.py:139-141
        for f in self.flows:
            f.store_inverse()
        self._release()
