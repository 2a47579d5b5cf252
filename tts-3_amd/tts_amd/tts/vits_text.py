"""Drop-in VITS text side whose inference runs in ``libtts_mi355x.so``.

* ``TextEncoder`` mirrors ``TTS/tts/layers/vits/networks.py:29-100`` (Coqui TTS 0.22.0): same
  constructor, same parameter tree (``emb``, ``encoder.*`` = RelativePositionTransformer with
  LayerNorm2 and window 4, ``proj``); ``forward(x, x_lengths)`` returns ``(x, m, logs, x_mask)``.
* ``StochasticDurationPredictor`` mirrors ``TTS/tts/layers/vits/stochastic_duration_predictor.py``
  (:150-282): every parameter of the reference (the training-only posterior side ``post_*``
  included, so checkpoints load unchanged); ``forward(..., reverse=True, noise_scale)`` returns
  ``logw`` like :273-282.  The reference draws its noise with ``torch.randn`` (:277); ``noise``
  passes that draw explicitly (drawn the same way on the device when not given).
* ``DurationPredictor`` mirrors ``TTS/tts/layers/glow_tts/duration_predictor.py`` as VITS builds it
  with ``use_sdp=False`` (vits.py:694-702): x + cond(g) + cond_lang(lang) -> 2 x (conv -> relu ->
  LayerNorm) -> proj.
* ``Vits`` is the inference surface of ``TTS/tts/models/vits.py``: ``inference(x, aux_input)``
  (:1088-1174) runs text encoder -> SDP (or the deterministic predictor) -> durations -> alignment
  expansion -> flow reverse -> (upsampling_z) -> waveform decoder on the device and returns the
  reference's output dict; the speaker / language embedding lookups, the d-vector normalisation,
  the given-durations branch and the masked slice are library kernels too.

Training (the SDP's forward direction, MAS, discriminators) is outside the MI355X path.
"""
from __future__ import annotations

import ctypes
import math
from typing import Dict, List, Optional

import numpy as np
import torch
from torch import nn

from .. import _native as N
from ..config import VITS_DECODER, VITS_FLOW, VITS_INFERENCE, VITS_SDP, VITS_TEXT_ENCODER
from ..vocoder.hifigan_generator import HifiganGenerator
from .glow_tts import LayerNorm, LayerNorm2, RelativePositionTransformer
from .vits_flow import ResidualCouplingBlocks


def _f32(t: torch.Tensor) -> np.ndarray:
    return np.ascontiguousarray(t.detach().to("cpu", torch.float32).numpy()).reshape(-1)


class _NativeModule(nn.Module):
    """Parameter-only module bound to one C-ABI handle (rebuilt when a parameter changes)."""

    _abi = ""  # entry-point prefix, e.g. "tts_vits_sdp"

    def _bind(self, cfg) -> None:
        self._cfg = cfg
        self._handle = None
        self._handle_key = None
        n = getattr(N.lib(), f"{self._abi}_num_weights")(ctypes.byref(cfg))
        if n < 0:
            N.check(f"{self._abi}_num_weights", -n)

    def _weight_list(self) -> List[np.ndarray]:
        raise NotImplementedError

    def _device(self) -> torch.device:
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError(f"{type(self).__name__} (tts_amd) runs only on a ROCm device: move it with .to('cuda')")
        return dev

    def _native_handle(self):
        key = tuple((p.data_ptr(), p._version, p.device) for p in self.parameters())
        if self._handle is not None and key == self._handle_key:
            return self._handle
        self._release()
        dev = self._device()
        ws = self._weight_list()
        numel = getattr(N.lib(), f"{self._abi}_weight_numel")
        for i, w in enumerate(ws):
            n = numel(ctypes.byref(self._cfg), i)
            if n != w.size:
                raise ValueError(f"weight {i} has {w.size} elements, expected {n}")
        arr = (ctypes.c_void_p * len(ws))(*[w.ctypes.data for w in ws])
        h = ctypes.c_void_p()
        N.call(f"{self._abi}_create", ctypes.byref(self._cfg), arr, dev.index or 0, ctypes.byref(h))
        self._handle, self._handle_key = h, key
        return h

    def _release(self):
        if getattr(self, "_handle", None) is not None:
            getattr(N.lib(), f"{self._abi}_destroy")(self._handle)
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


def _rows(recs, n):
    return [{"name": recs[i].name.decode(), "flops": recs[i].flops, "bytes": recs[i].bytes, "ms": recs[i].ms}
            for i in range(n)]


class TextEncoder(_NativeModule):
    """networks.py:29-100 on MI355X (one C-ABI call, ``tts_vits_text_encoder_forward``)."""

    _abi = "tts_vits_text_encoder"

    def __init__(self, n_vocab: int, out_channels: int, hidden_channels: int, hidden_channels_ffn: int, num_heads: int,
                 num_layers: int, kernel_size: int, dropout_p: float, language_emb_dim: int = None,
                 math_mode: str = "fp32x6"):
        super().__init__()
        if math_mode not in N.MATH_MODES:
            raise ValueError(f"math_mode must be one of {sorted(N.MATH_MODES)}")
        self.out_channels = out_channels
        self.hidden_channels = hidden_channels
        self.language_emb_dim = language_emb_dim or 0
        self.math_mode = math_mode
        self.emb = nn.Embedding(n_vocab, hidden_channels)
        nn.init.normal_(self.emb.weight, 0.0, hidden_channels**-0.5)
        if language_emb_dim:
            hidden_channels += language_emb_dim
        self.encoder = RelativePositionTransformer(hidden_channels, hidden_channels, hidden_channels,
                                                   hidden_channels_ffn, num_heads, num_layers, kernel_size=kernel_size,
                                                   dropout_p=dropout_p, layer_norm_type="2", rel_attn_window_size=4)
        self.proj = nn.Conv1d(hidden_channels, out_channels * 2, 1)
        c = N.TtsVitsTextEncoderCfg()
        c.n_vocab, c.out_channels, c.hidden_channels = n_vocab, out_channels, self.hidden_channels  # before + L
        c.hidden_channels_ffn, c.num_heads, c.num_layers = hidden_channels_ffn, num_heads, num_layers
        c.kernel_size = kernel_size
        c.language_emb_dim = language_emb_dim or 0
        c.math_mode = N.MATH_MODES[math_mode]
        self._bind(c)

    def _weight_list(self) -> List[np.ndarray]:
        ws = [_f32(self.emb.weight)]
        enc = self.encoder
        for l in range(enc.num_layers):
            a = enc.attn_layers[l]
            for m in (a.conv_q, a.conv_k, a.conv_v, a.conv_o):
                ws += [_f32(m.weight), _f32(m.bias)]
            if a.emb_rel_k.size(0) != 1:
                raise NotImplementedError("heads_share=False relative embeddings are not implemented")
            ws += [_f32(a.emb_rel_k), _f32(a.emb_rel_v)]
            ws += [_f32(enc.norm_layers_1[l].gamma), _f32(enc.norm_layers_1[l].beta)]
            f = enc.ffn_layers[l]
            ws += [_f32(f.conv_1.weight), _f32(f.conv_1.bias), _f32(f.conv_2.weight), _f32(f.conv_2.bias)]
            ws += [_f32(enc.norm_layers_2[l].gamma), _f32(enc.norm_layers_2[l].beta)]
        ws += [_f32(self.proj.weight), _f32(self.proj.bias)]
        return ws

    def _io(self, x, x_lengths):
        dev = self._device()
        tok = x.to(device=dev, dtype=torch.int64).contiguous()
        if tok.dim() != 2:
            raise ValueError("x must be token ids [B, T]")
        B, T = tok.shape
        if x_lengths.shape[0] != B:  # networks.py:89
            raise AssertionError("x and x_lengths batch sizes differ")
        lens = x_lengths.to(device=dev, dtype=torch.int64).contiguous()
        E, C = self.hidden_channels + self.language_emb_dim, self.out_channels
        out = (torch.empty(B, E, T, device=dev), torch.empty(B, C, T, device=dev), torch.empty(B, C, T, device=dev),
               torch.empty(B, 1, T, device=dev))
        return dev, tok, lens, out

    def _lang(self, lang_emb, B, dev):
        """lang_emb [B or 1, L, 1] (emb_l(lid).unsqueeze(-1)) -> [B, L] on the device (a batch of 1 is
        broadcast, as the reference's expand does); None without a language embedding."""
        L = self.language_emb_dim
        if not L:
            if lang_emb is not None:
                raise ValueError("lang_emb given to a TextEncoder built without language_emb_dim")
            return None
        if lang_emb is None:
            raise ValueError(f"this TextEncoder concatenates a language embedding (language_emb_dim={L}): "
                             "pass lang_emb [B, L, 1]")
        le = lang_emb.to(device=dev, dtype=torch.float32).reshape(lang_emb.shape[0], L)
        return le.expand(B, L).contiguous()

    def forward(self, x: torch.Tensor, x_lengths: torch.Tensor, lang_emb: Optional[torch.Tensor] = None):
        with torch.no_grad():
            h = self._native_handle()
            dev, tok, lens, (xo, m, logs, xm) = self._io(x, x_lengths)
            B, T = tok.shape
            le = self._lang(lang_emb, B, dev)
            N.call("tts_vits_text_encoder_forward", h, N.ptr(tok), N.ptr(lens), N.ptr(le), B, T, N.ptr(xo), N.ptr(m),
                   N.ptr(logs), N.ptr(xm), N.stream_ptr(dev))
        return xo, m, logs, xm

    def profile(self, x, x_lengths, lang_emb=None):
        h = self._native_handle()
        dev, tok, lens, (xo, m, logs, xm) = self._io(x, x_lengths)
        B, T = tok.shape
        le = self._lang(lang_emb, B, dev)
        cap = 1024
        recs = (N.TtsLaunchRecord * cap)()
        n = ctypes.c_int(0)
        N.call("tts_vits_text_encoder_forward_profiled", h, N.ptr(tok), N.ptr(lens), N.ptr(le), B, T, N.ptr(xo),
               N.ptr(m), N.ptr(logs), N.ptr(xm), N.stream_ptr(dev), recs, cap, ctypes.byref(n))
        return (xo, m, logs, xm), _rows(recs, min(n.value, cap))


class DilatedDepthSeparableConv(nn.Module):
    """stochastic_duration_predictor.py:11-44 (parameters only)."""

    def __init__(self, channels, kernel_size, num_layers, dropout_p=0.0):
        super().__init__()
        self.num_layers = num_layers
        self.convs_sep = nn.ModuleList()
        self.convs_1x1 = nn.ModuleList()
        self.norms_1 = nn.ModuleList()
        self.norms_2 = nn.ModuleList()
        for i in range(num_layers):
            dilation = kernel_size**i
            padding = (kernel_size * dilation - dilation) // 2
            self.convs_sep.append(nn.Conv1d(channels, channels, kernel_size, groups=channels, dilation=dilation,
                                            padding=padding))
            self.convs_1x1.append(nn.Conv1d(channels, channels, 1))
            self.norms_1.append(LayerNorm2(channels))
            self.norms_2.append(LayerNorm2(channels))


class ElementwiseAffine(nn.Module):
    """stochastic_duration_predictor.py:66-76 (parameters only)."""

    def __init__(self, channels):
        super().__init__()
        self.translation = nn.Parameter(torch.zeros(channels, 1))
        self.log_scale = nn.Parameter(torch.zeros(channels, 1))


class ConvFlow(nn.Module):
    """stochastic_duration_predictor.py:86-120 (parameters only)."""

    def __init__(self, in_channels, hidden_channels, kernel_size, num_layers, num_bins=10, tail_bound=5.0):
        super().__init__()
        self.num_bins = num_bins
        self.tail_bound = tail_bound
        self.hidden_channels = hidden_channels
        self.half_channels = in_channels // 2
        self.pre = nn.Conv1d(self.half_channels, hidden_channels, 1)
        self.convs = DilatedDepthSeparableConv(hidden_channels, kernel_size, num_layers, dropout_p=0.0)
        self.proj = nn.Conv1d(hidden_channels, self.half_channels * (num_bins * 3 - 1), 1)
        self.proj.weight.data.zero_()
        self.proj.bias.data.zero_()


class StochasticDurationPredictor(_NativeModule):
    """stochastic_duration_predictor.py:150-282 on MI355X, inference (reverse) direction."""

    _abi = "tts_vits_sdp"

    def __init__(self, in_channels: int, hidden_channels: int, kernel_size: int, dropout_p: float, num_flows=4,
                 cond_channels=0, language_emb_dim=0, math_mode: str = "fp32x6"):
        super().__init__()
        if math_mode not in N.MATH_MODES:
            raise ValueError(f"math_mode must be one of {sorted(N.MATH_MODES)}")
        if language_emb_dim:
            in_channels += language_emb_dim
        self.in_channels = in_channels
        self.hidden_channels = hidden_channels
        self.num_flows = num_flows
        self.cond_channels = cond_channels or 0
        self.language_emb_dim = language_emb_dim or 0
        self.math_mode = math_mode
        self.pre = nn.Conv1d(in_channels, hidden_channels, 1)
        self.convs = DilatedDepthSeparableConv(hidden_channels, kernel_size, num_layers=3, dropout_p=dropout_p)
        self.proj = nn.Conv1d(hidden_channels, hidden_channels, 1)
        self.flows = nn.ModuleList([ElementwiseAffine(2)])
        self.flows += [ConvFlow(2, hidden_channels, kernel_size, num_layers=3) for _ in range(num_flows)]
        self.post_pre = nn.Conv1d(1, hidden_channels, 1)
        self.post_convs = DilatedDepthSeparableConv(hidden_channels, kernel_size, num_layers=3, dropout_p=dropout_p)
        self.post_proj = nn.Conv1d(hidden_channels, hidden_channels, 1)
        self.post_flows = nn.ModuleList([ElementwiseAffine(2)])
        self.post_flows += [ConvFlow(2, hidden_channels, kernel_size, num_layers=3) for _ in range(num_flows)]
        if cond_channels:
            self.cond = nn.Conv1d(cond_channels, hidden_channels, 1)
        if language_emb_dim:
            self.cond_lang = nn.Conv1d(language_emb_dim, hidden_channels, 1)
        c = N.TtsVitsSdpCfg()
        c.in_channels, c.hidden_channels, c.kernel_size = in_channels, hidden_channels, kernel_size
        c.num_flows, c.cond_channels = num_flows, self.cond_channels
        c.language_emb_dim = language_emb_dim or 0
        c.math_mode = N.MATH_MODES[math_mode]
        self._bind(c)

    def _weight_list(self) -> List[np.ndarray]:
        def conv(m):
            return [_f32(m.weight), _f32(m.bias)]

        def dds(d):
            ws = []
            for i in range(3):
                ws += conv(d.convs_sep[i])
            for i in range(3):
                ws += conv(d.convs_1x1[i])
            for n in (d.norms_1, d.norms_2):
                for i in range(3):
                    ws += [_f32(n[i].gamma), _f32(n[i].beta)]
            return ws

        ws = conv(self.pre) + dds(self.convs) + conv(self.proj)
        ws += [_f32(self.flows[0].translation), _f32(self.flows[0].log_scale)]
        for f in self.flows[1:]:
            ws += conv(f.pre) + dds(f.convs) + conv(f.proj)
        if self.cond_channels:
            ws += conv(self.cond)
        if self.language_emb_dim:
            ws += conv(self.cond_lang)
        return ws

    def _io(self, x, x_mask, g, noise):
        dev = self._device()
        x = x.to(device=dev, dtype=torch.float32).contiguous()
        B, C, T = x.shape
        if C != self.in_channels:
            raise ValueError(f"x has {C} channels, expected {self.in_channels}")
        m = x_mask.to(device=dev, dtype=torch.float32).reshape(B, 1, T).contiguous()
        gg = None
        if g is not None:
            if not self.cond_channels:
                raise ValueError("g given to a StochasticDurationPredictor built with cond_channels=0")
            gg = g.to(device=dev, dtype=torch.float32).reshape(B, self.cond_channels).contiguous()
        if noise is None:
            noise = torch.randn(B, 2, T, device=dev, dtype=torch.float32)  # :277
        noise = noise.to(device=dev, dtype=torch.float32).contiguous()
        if noise.shape != (B, 2, T):
            raise ValueError(f"noise has shape {tuple(noise.shape)}, expected {(B, 2, T)}")
        return dev, x, m, gg, noise

    def forward(self, x, x_mask, dr=None, g=None, lang_emb=None, reverse=False, noise_scale=1.0,
                noise: Optional[torch.Tensor] = None):
        if not reverse:
            raise NotImplementedError("StochasticDurationPredictor: the training direction is not on the MI355X path")
        if self.cond_channels and g is None:
            raise ValueError("this predictor is speaker-conditioned (cond_channels > 0): pass g [B, cond, 1]")
        with torch.no_grad():
            h = self._native_handle()
            dev, x, m, gg, noise = self._io(x, x_mask, g, noise)
            B, _, T = x.shape
            le = _cond_rows(lang_emb, self.language_emb_dim, B, dev, "lang_emb", "cond_lang")
            logw = torch.empty(B, 1, T, device=dev)
            N.call("tts_vits_sdp_reverse", h, N.ptr(x), N.ptr(m), N.ptr(gg), N.ptr(le), N.ptr(noise),
                   float(noise_scale), B, T, N.ptr(logw), N.stream_ptr(dev))
        return logw

    def profile(self, x, x_mask, g=None, noise_scale=1.0, noise=None, lang_emb=None):
        h = self._native_handle()
        dev, x, m, gg, noise = self._io(x, x_mask, g, noise)
        B, _, T = x.shape
        le = _cond_rows(lang_emb, self.language_emb_dim, B, dev, "lang_emb", "cond_lang")
        logw = torch.empty(B, 1, T, device=dev)
        cap = 1024
        recs = (N.TtsLaunchRecord * cap)()
        n = ctypes.c_int(0)
        N.call("tts_vits_sdp_reverse_profiled", h, N.ptr(x), N.ptr(m), N.ptr(gg), N.ptr(le), N.ptr(noise),
               float(noise_scale), B, T, N.ptr(logw), N.stream_ptr(dev), recs, cap, ctypes.byref(n))
        return logw, _rows(recs, min(n.value, cap))


def _cond_rows(v, width, B, dev, what, layer):
    """A per-utterance conditioning vector [B or 1, width(, 1)] -> [B, width] on the device (None when
    the module has no such layer)."""
    if not width:
        if v is not None:
            raise ValueError(f"{what} given to a module without a {layer} layer")
        return None
    if v is None:
        raise ValueError(f"this module has a {layer} layer ({width} channels): pass {what} [B, {width}, 1]")
    v = v.to(device=dev, dtype=torch.float32).reshape(v.shape[0], width)
    return v.expand(B, width).contiguous()


class DurationPredictor(_NativeModule):
    """The deterministic duration predictor of VITS with ``use_sdp=False`` (vits.py:694-702):
    ``TTS/tts/layers/glow_tts/duration_predictor.py:6-68`` on MI355X (``tts_vits_dp_forward``).  Same
    constructor and parameter names; ``forward(x, x_mask, g=None, lang_emb=None)`` returns the log
    durations [B, 1, T] like :49-68."""

    _abi = "tts_vits_dp"

    def __init__(self, in_channels, hidden_channels, kernel_size, dropout_p, cond_channels=None, language_emb_dim=None,
                 math_mode: str = "fp32x6"):
        super().__init__()
        if math_mode not in N.MATH_MODES:
            raise ValueError(f"math_mode must be one of {sorted(N.MATH_MODES)}")
        L = language_emb_dim or 0
        I = in_channels + L  # :28-29
        self.in_channels = I
        self.filter_channels = hidden_channels
        self.kernel_size = kernel_size
        self.cond_channels = cond_channels or 0
        self.language_emb_dim = L
        self.math_mode = math_mode
        self.drop = nn.Dropout(dropout_p)
        self.conv_1 = nn.Conv1d(I, hidden_channels, kernel_size, padding=kernel_size // 2)
        self.norm_1 = LayerNorm(hidden_channels)
        self.conv_2 = nn.Conv1d(hidden_channels, hidden_channels, kernel_size, padding=kernel_size // 2)
        self.norm_2 = LayerNorm(hidden_channels)
        self.proj = nn.Conv1d(hidden_channels, 1, 1)
        if self.cond_channels:
            self.cond = nn.Conv1d(self.cond_channels, I, 1)
        if L:
            self.cond_lang = nn.Conv1d(L, I, 1)
        c = N.TtsVitsDpCfg()
        c.in_channels, c.hidden_channels, c.kernel_size = in_channels, hidden_channels, kernel_size
        c.cond_channels, c.language_emb_dim = self.cond_channels, L
        c.math_mode = N.MATH_MODES[math_mode]
        self._bind(c)

    def _weight_list(self) -> List[np.ndarray]:
        ws = [_f32(self.conv_1.weight), _f32(self.conv_1.bias), _f32(self.norm_1.gamma), _f32(self.norm_1.beta),
              _f32(self.conv_2.weight), _f32(self.conv_2.bias), _f32(self.norm_2.gamma), _f32(self.norm_2.beta),
              _f32(self.proj.weight), _f32(self.proj.bias)]
        if self.cond_channels:
            ws += [_f32(self.cond.weight), _f32(self.cond.bias)]
        if self.language_emb_dim:
            ws += [_f32(self.cond_lang.weight), _f32(self.cond_lang.bias)]
        return ws

    def _io(self, x, x_mask, g, lang_emb):
        dev = self._device()
        x = x.to(device=dev, dtype=torch.float32).contiguous()
        B, C, T = x.shape
        if C != self.in_channels:
            raise ValueError(f"x has {C} channels, expected {self.in_channels}")
        m = x_mask.to(device=dev, dtype=torch.float32).reshape(B, 1, T).contiguous()
        gg = _cond_rows(g, self.cond_channels, B, dev, "g", "cond") if g is not None else None
        le = _cond_rows(lang_emb, self.language_emb_dim, B, dev, "lang_emb", "cond_lang") if lang_emb is not None \
            else None
        return dev, x, m, gg, le

    def forward(self, x, x_mask, g=None, lang_emb=None):
        with torch.no_grad():
            h = self._native_handle()
            dev, x, m, gg, le = self._io(x, x_mask, g, lang_emb)
            B, _, T = x.shape
            logw = torch.empty(B, 1, T, device=dev)
            N.call("tts_vits_dp_forward", h, N.ptr(x), N.ptr(m), N.ptr(gg), N.ptr(le), B, T, N.ptr(logw),
                   N.stream_ptr(dev))
        return logw

    def profile(self, x, x_mask, g=None, lang_emb=None):
        h = self._native_handle()
        dev, x, m, gg, le = self._io(x, x_mask, g, lang_emb)
        B, _, T = x.shape
        logw = torch.empty(B, 1, T, device=dev)
        cap = 256
        recs = (N.TtsLaunchRecord * cap)()
        n = ctypes.c_int(0)
        N.call("tts_vits_dp_forward_profiled", h, N.ptr(x), N.ptr(m), N.ptr(gg), N.ptr(le), B, T, N.ptr(logw),
               N.stream_ptr(dev), recs, cap, ctypes.byref(n))
        return logw, _rows(recs, min(n.value, cap))


def vits_durations(logw: torch.Tensor, x_mask: torch.Tensor, length_scale: float = 1.0):
    """vits.py:1145-1148 on the device: (w_ceil [B,1,T_x], y_lengths [B] int64)."""
    B, _, Tx = logw.shape
    dev = logw.device
    w_ceil = torch.empty(B, 1, Tx, device=dev)
    y_len = torch.empty(B, dtype=torch.int64, device=dev)
    N.call("tts_vits_durations", N.ptr(logw.contiguous()), N.ptr(x_mask.contiguous()), B, Tx, float(length_scale),
           N.ptr(w_ceil), N.ptr(y_len), N.stream_ptr(dev))
    return w_ceil, y_len


def vits_expand(w_ceil, x_mask, y_lengths, m_p, logs_p, noise=None, noise_scale: float = 0.667, T_y: int = None,
                want_attn: bool = True):
    """vits.py:1147-1154 on the device: (z_p, y_mask, m_p', logs_p', attn)."""
    B, C, Tx = m_p.shape
    dev = m_p.device
    if T_y is None:
        T_y = int(y_lengths.max().item())  # sequence_mask(y_lengths, None)
    z_p = torch.empty(B, C, T_y, device=dev)
    y_mask = torch.empty(B, 1, T_y, device=dev)
    mp = torch.empty(B, C, T_y, device=dev)
    lp = torch.empty(B, C, T_y, device=dev)
    attn = torch.empty(B, Tx, T_y, device=dev) if want_attn else None
    if noise is None:
        noise = torch.randn(B, C, T_y, device=dev)  # torch.randn_like(m_p) (vits.py:1154)
    elif noise.dim() != 3 or noise.shape[0] != B or noise.shape[1] != C or noise.shape[2] < T_y:
        raise ValueError(f"noise has shape {tuple(noise.shape)}, expected [{B}, {C}, >= {T_y}]")
    noise = noise[:, :, :T_y].to(device=dev, dtype=torch.float32).contiguous()  # the first T_y frames
    N.call("tts_vits_expand", N.ptr(w_ceil), N.ptr(x_mask.contiguous()), N.ptr(y_lengths), N.ptr(m_p.contiguous()),
           N.ptr(logs_p.contiguous()), N.ptr(noise.contiguous()), float(noise_scale), B, C, Tx, T_y, N.ptr(z_p),
           N.ptr(y_mask), N.ptr(mp), N.ptr(lp), N.ptr(attn), N.stream_ptr(dev))
    return z_p, y_mask, mp, lp, attn


def vits_durations_given(durations: torch.Tensor, B: int, T_x: int, dev):
    """vits.py:1141-1146 with aux_input["durations"]: w = durations.unsqueeze(0), w_ceil = ceil(w) (no mask,
    no length_scale), y_lengths = clamp_min(sum(w_ceil), 1), on the device.  ``durations`` [T_x] / [1, T_x]
    is shared by every utterance, [B, T_x] gives one row each."""
    if durations.shape[-1] != T_x:  # :1142
        raise AssertionError("durations.shape[-1] != x.shape[-1]")
    d = durations.to(device=dev, dtype=torch.float32)
    if d.numel() == T_x:
        d, bstride = d.reshape(T_x).contiguous(), 0
    elif d.numel() == B * T_x:
        d, bstride = d.reshape(B, T_x).contiguous(), T_x
    else:
        raise ValueError(f"durations has shape {tuple(durations.shape)}: expected [T_x], [1, T_x] or [B, T_x]")
    w_ceil = torch.empty(B, 1, T_x, device=dev)
    y_len = torch.empty(B, dtype=torch.int64, device=dev)
    N.call("tts_vits_durations_given", N.ptr(d), bstride, B, T_x, N.ptr(w_ceil), N.ptr(y_len), N.stream_ptr(dev))
    return w_ceil, y_len


def vits_mask_slice(z: torch.Tensor, y_mask: torch.Tensor, T_out: Optional[int] = None) -> torch.Tensor:
    """(z * y_mask)[:, :, :T_out] (vits.py:1161) on the device."""
    B, C, T = z.shape
    T_out = T if T_out is None else min(int(T_out), T)
    if T_out < 1:
        raise ValueError("max_inference_len leaves no frames")
    z = z.contiguous()
    m = y_mask.to(device=z.device, dtype=torch.float32).reshape(B, 1, T).contiguous()
    out = torch.empty(B, C, T_out, device=z.device)
    N.call("tts_vits_mask_slice", N.ptr(z), N.ptr(m), B, C, T, T_out, N.ptr(out), N.stream_ptr(z.device))
    return out


def vits_upsample_z(z: torch.Tensor, y_lengths: torch.Tensor, factor: float):
    """upsampling_z (vits.py:944-959, encoder_sample_rate with interpolate_z) on the device:
    F.interpolate(z, scale_factor=[factor], mode="linear") and sequence_mask(y_lengths * factor).
    Returns (z2 [B, C, floor(T factor)], y_mask2 [B, 1, same])."""
    B, C, T = z.shape
    T2 = int(math.floor(float(T) * factor))  # F.interpolate's output size
    # the reference multiplies z2 by a mask of ceil(max(y_lengths) * factor) frames (fp32 product)
    Tm = int(math.ceil(float(np.float32(T) * np.float32(factor))))
    if T2 != Tm:
        raise RuntimeError(f"upsampling_z: z has {T2} frames after interpolation but the mask {Tm} (the reference's "
                           "z * y_mask fails the same way for this factor)")
    z2 = torch.empty(B, C, T2, device=z.device)
    m2 = torch.empty(B, 1, T2, device=z.device)
    yl = y_lengths.to(device=z.device, dtype=torch.int64).contiguous()
    N.call("tts_vits_upsample_z", N.ptr(z.contiguous()), N.ptr(yl), B, C, T, float(factor), T2, N.ptr(z2), N.ptr(m2),
           N.stream_ptr(z.device))
    return z2, m2


def embedding_rows(emb: nn.Embedding, ids: torch.Tensor) -> torch.Tensor:
    """emb(ids) for a batch of ids [B] (speaker / language embedding lookups, vits.py:1117, :1124) on the
    device; ids outside [0, num) are clamped (the reference raises IndexError)."""
    w = emb.weight
    if w.device.type != "cuda":
        raise RuntimeError("embedding tables run only on a ROCm device")
    ids = ids.to(device=w.device, dtype=torch.int64).reshape(-1).contiguous()
    B = ids.numel()
    out = torch.empty(B, w.shape[1], device=w.device)
    N.call("tts_embedding_rows", N.ptr(w.detach().float().contiguous()), w.shape[0], w.shape[1], N.ptr(ids), 1, B,
           N.ptr(out), N.stream_ptr(w.device))
    return out


def l2_normalize_rows(d: torch.Tensor, dev) -> torch.Tensor:
    """F.normalize(d) (dim 1, p 2, eps 1e-12) of [B, C] d-vectors on the device (vits.py:884-886)."""
    d = d.to(device=dev, dtype=torch.float32)
    if d.dim() == 1:
        d = d.unsqueeze(0)
    d = d.reshape(d.shape[0], -1).contiguous()
    out = torch.empty_like(d)
    N.call("tts_l2_normalize_rows", N.ptr(d), d.shape[0], d.shape[1], N.ptr(out), N.stream_ptr(dev))
    return out


class Vits(nn.Module):
    """The inference surface of ``TTS/tts/models/vits.py`` (``Vits.inference``, :1088-1174) on MI355X.

    ``args`` takes ``VitsArgs`` field names (vits.py:541-596; unset fields keep the reference
    defaults): num_chars, hidden_channels, the text encoder / flow / decoder / duration predictor
    fields, use_sdp, use_speaker_embedding + num_speakers + speaker_embedding_channels,
    use_d_vector_file + d_vector_dim, condition_dp_on_speaker, use_language_embedding +
    num_languages + embedded_language_dim (the reference takes num_languages from its language
    manager, vits.py:796-801), encoder_sample_rate + interpolate_z (with ``sample_rate``, the audio
    config's rate, vits.py:808-812), length_scale, inference_noise_scale(_dp), max_inference_len.
    Sub-modules keep the reference names (``text_encoder``, ``duration_predictor``, ``flow``,
    ``waveform_decoder``, ``emb_g``, ``emb_l``) so a Vits checkpoint's inference keys load unchanged
    (``load_state_dict(strict=False)`` skips the posterior encoder and discriminator)."""

    def __init__(self, args: Optional[Dict] = None, text_math_mode: str = "fp32x6",
                 flow_math_mode: Optional[str] = None, decoder_math_mode: Optional[str] = None):
        super().__init__()
        a = dict(num_chars=64, hidden_channels=192, use_sdp=True, use_speaker_embedding=False, num_speakers=0,
                 speaker_embedding_channels=256, use_d_vector_file=False, d_vector_dim=0,
                 condition_dp_on_speaker=True, use_language_embedding=False, num_languages=0,
                 embedded_language_dim=4, encoder_sample_rate=None, interpolate_z=True, sample_rate=22050,
                 max_inference_len=None, dropout_p_duration_predictor=0.5,
                 num_layers_text_encoder=VITS_TEXT_ENCODER["num_layers"],
                 hidden_channels_ffn_text_encoder=VITS_TEXT_ENCODER["hidden_channels_ffn"],
                 num_heads_text_encoder=VITS_TEXT_ENCODER["num_heads"],
                 kernel_size_text_encoder=VITS_TEXT_ENCODER["kernel_size"],
                 kernel_size_flow=VITS_FLOW["kernel_size"], dilation_rate_flow=VITS_FLOW["dilation_rate"],
                 num_layers_flow=VITS_FLOW["num_layers"],
                 resblock_type_decoder=VITS_DECODER["resblock_type"],
                 resblock_dilation_sizes_decoder=VITS_DECODER["resblock_dilation_sizes"],
                 resblock_kernel_sizes_decoder=VITS_DECODER["resblock_kernel_sizes"],
                 upsample_kernel_sizes_decoder=VITS_DECODER["upsample_kernel_sizes"],
                 upsample_initial_channel_decoder=VITS_DECODER["upsample_initial_channel"],
                 upsample_rates_decoder=VITS_DECODER["upsample_factors"],
                 length_scale=VITS_INFERENCE["length_scale"],
                 inference_noise_scale=VITS_INFERENCE["inference_noise_scale"],
                 inference_noise_scale_dp=VITS_INFERENCE["inference_noise_scale_dp"])
        a.update(args or {})
        self.args = a
        self.length_scale = a["length_scale"]
        self.inference_noise_scale = a["inference_noise_scale"]
        self.inference_noise_scale_dp = a["inference_noise_scale_dp"]
        self.max_inference_len = a["max_inference_len"]
        self.interpolate_factor = None
        if a["encoder_sample_rate"]:  # init_upsampling (vits.py:806-812)
            self.interpolate_factor = a["sample_rate"] / a["encoder_sample_rate"]
        H = a["hidden_channels"]
        self.embedded_speaker_dim = 0  # vits.py:740-786
        if a["use_speaker_embedding"] and a["num_speakers"] > 0:
            self.embedded_speaker_dim = a["speaker_embedding_channels"]
            self.emb_g = nn.Embedding(a["num_speakers"], self.embedded_speaker_dim)
        elif a["use_d_vector_file"]:
            self.embedded_speaker_dim = a["d_vector_dim"]
        self.embedded_language_dim = 0  # init_multilingual (vits.py:788-804)
        if a["use_language_embedding"] and a["num_languages"] > 0:
            self.embedded_language_dim = a["embedded_language_dim"]
            self.emb_l = nn.Embedding(a["num_languages"], self.embedded_language_dim)
            torch.nn.init.xavier_uniform_(self.emb_l.weight)
        gin, L = self.embedded_speaker_dim, self.embedded_language_dim
        self.text_encoder = TextEncoder(a["num_chars"], H, H, a["hidden_channels_ffn_text_encoder"],
                                        a["num_heads_text_encoder"], a["num_layers_text_encoder"],
                                        a["kernel_size_text_encoder"], 0.1, language_emb_dim=L,
                                        math_mode=text_math_mode)
        self.flow = ResidualCouplingBlocks(H, H, kernel_size=a["kernel_size_flow"], dilation_rate=a["dilation_rate_flow"],
                                           num_layers=a["num_layers_flow"], cond_channels=gin, math_mode=flow_math_mode)
        if a["use_sdp"]:  # vits.py:684-702
            self.duration_predictor = StochasticDurationPredictor(
                H, 192, 3, a["dropout_p_duration_predictor"], 4,
                cond_channels=gin if a["condition_dp_on_speaker"] else 0, language_emb_dim=L,
                math_mode=text_math_mode)
        else:
            self.duration_predictor = DurationPredictor(H, 256, 3, a["dropout_p_duration_predictor"],
                                                        cond_channels=gin, language_emb_dim=L,
                                                        math_mode=text_math_mode)
        self.waveform_decoder = HifiganGenerator(
            H, 1, a["resblock_type_decoder"], a["resblock_dilation_sizes_decoder"], a["resblock_kernel_sizes_decoder"],
            a["upsample_kernel_sizes_decoder"], a["upsample_initial_channel_decoder"], a["upsample_rates_decoder"],
            inference_padding=0, cond_channels=gin, conv_pre_weight_norm=False, conv_post_weight_norm=False,
            conv_post_bias=False, math_mode=decoder_math_mode)

    def _dev(self) -> torch.device:
        return self.waveform_decoder.conv_pre.weight.device

    def _set_cond_input(self, aux_input: Dict):
        """vits.py:874-894: (sid, g, lid, durations); the d-vectors are normalised on the device."""
        sid = g = lid = None
        if aux_input.get("speaker_ids") is not None:
            sid = aux_input["speaker_ids"]
            if sid.ndim == 0:
                sid = sid.unsqueeze(0)
        if aux_input.get("d_vectors") is not None:
            d = aux_input["d_vectors"]
            g = l2_normalize_rows(d, self._dev()).unsqueeze(-1)  # F.normalize(d).unsqueeze(-1)
            if d.ndim == 1:  # g.ndim == 2 in the reference: unsqueeze_(0) -> [1, C, 1]
                g = g.reshape(1, -1, 1)
        if aux_input.get("language_ids") is not None:
            lid = aux_input["language_ids"]
            if lid.ndim == 0:
                lid = lid.unsqueeze(0)
        return sid, g, lid, aux_input.get("durations")

    @torch.no_grad()
    def inference(self, x, aux_input=None):
        """vits.py:1088-1174.  Extra aux_input keys (test hooks): ``noise_dp`` [B, 2, T_x] and ``noise_z``
        [B, hidden, >= T_y] (its first T_y frames are used), the two standard-normal draws the
        reference makes (:277 of the SDP and randn_like(m_p) at vits.py:1154); drawn on the device
        when absent."""
        aux_input = aux_input or {}
        sid, g, lid, durations = self._set_cond_input(aux_input)
        x_lengths = aux_input.get("x_lengths")
        if x_lengths is None:  # _set_x_lengths (:1083-1086)
            x_lengths = torch.tensor(x.shape[1:2]).to(x.device)
        if self.args["use_speaker_embedding"] and hasattr(self, "emb_g") and sid is not None:  # :1115-1117
            g = embedding_rows(self.emb_g, sid).unsqueeze(-1)
        lang_emb = None
        if self.args["use_language_embedding"] and hasattr(self, "emb_l") and lid is not None:  # :1120-1122
            lang_emb = embedding_rows(self.emb_l, lid).unsqueeze(-1)
        x, m_p, logs_p, x_mask = self.text_encoder(x, x_lengths, lang_emb=lang_emb)
        B, _, T_x = x.shape
        g_dp = g if self.args["condition_dp_on_speaker"] else None
        if durations is None:
            if self.args["use_sdp"]:  # :1127-1135
                logw = self.duration_predictor(x, x_mask, g=g_dp, reverse=True,
                                               noise_scale=self.inference_noise_scale_dp, lang_emb=lang_emb,
                                               noise=aux_input.get("noise_dp"))
            else:  # :1136-1139
                logw = self.duration_predictor(x, x_mask, g=g_dp, lang_emb=lang_emb)
            w_ceil, y_lengths = vits_durations(logw, x_mask, self.length_scale)
        else:  # w = durations.unsqueeze(0) (:1141-1143)
            w_ceil, y_lengths = vits_durations_given(durations, B, T_x, x.device)
        z_p, y_mask, m_p, logs_p, attn = vits_expand(w_ceil, x_mask, y_lengths, m_p, logs_p,
                                                     noise=aux_input.get("noise_z"),
                                                     noise_scale=self.inference_noise_scale)
        z = self.flow(z_p, y_mask, g=g, reverse=True)
        if self.interpolate_factor is not None and self.args["interpolate_z"]:  # upsampling_z (:1159, :944-959)
            z, y_mask = vits_upsample_z(z, y_lengths, self.interpolate_factor)
        o = self.waveform_decoder(vits_mask_slice(z, y_mask, self.max_inference_len), g=g)
        return {"model_outputs": o, "alignments": attn, "durations": w_ceil, "z": z, "z_p": z_p, "m_p": m_p,
                "logs_p": logs_p, "y_mask": y_mask}
