"""Drop-in Glow-TTS text side whose inference runs in ``libtts_mi355x.so``.

* ``Encoder`` mirrors ``TTS/tts/layers/glow_tts/encoder.py`` (Coqui TTS 0.22.0) for every
  ``encoder_type`` (:97-123): ``rel_pos_transformer`` (the Glow-TTS default), ``gated_conv``,
  ``residual_conv_bn`` and ``time_depth_separable``; same constructor (:83-95), same parameter
  tree (``emb``, ``prenet.*``, ``encoder.*``, ``postnet.*``, ``proj_m``, ``proj_s``,
  ``duration_predictor.*``) so reference checkpoints load unchanged; ``forward(x, x_lengths,
  g=None)`` returns ``(x_m, x_logs, logw, x_mask)`` like :143-179.
* ``GlowTTS`` is the inference surface of ``TTS/tts/models/glow_tts.py``: ``inference(x,
  aux_input)`` (:342-374) runs encoder -> durations -> alignment expansion -> decoder reverse
  on the device and returns the reference's output dict.  ``load_checkpoint`` (:522-530) reads
  the ``model`` state dict with ``torch.load(weights_only=True)``.

The nn modules below only hold parameters; the handle is rebuilt when any parameter changes.
Multi-speaker models (``use_speaker_embedding`` / ``use_d_vector_file``, glow_tts.py:107-191)
condition the duration predictor and the decoder flows on ``g``.  Training (``forward``, MAS)
is outside the MI355X path.
"""
from __future__ import annotations

import ctypes
import math
from types import SimpleNamespace
from typing import Dict, List, Optional

import numpy as np
import torch
from torch import nn
from torch.nn import functional as F

from .. import _native as N
from ..config import GLOW_TTS_DECODER, GLOW_TTS_ENCODER, GLOW_TTS_INFERENCE
from .glow_decoder import Decoder


class LayerNorm(nn.Module):
    """normalization.py:5-28 (parameters only)."""

    def __init__(self, channels: int, eps: float = 1e-4):
        super().__init__()
        self.channels = channels
        self.eps = eps
        self.gamma = nn.Parameter(torch.ones(1, channels, 1) * 0.1)
        self.beta = nn.Parameter(torch.zeros(1, channels, 1))


class LayerNorm2(nn.Module):
    """normalization.py:31-53 (parameters only): F.layer_norm over the channels, eps 1e-5."""

    def __init__(self, channels: int, eps: float = 1e-5):
        super().__init__()
        self.channels = channels
        self.eps = eps
        self.gamma = nn.Parameter(torch.ones(channels))
        self.beta = nn.Parameter(torch.zeros(channels))


class ResidualConv1dLayerNormBlock(nn.Module):
    """glow.py:11-67 (parameters only)."""

    def __init__(self, in_channels, hidden_channels, out_channels, kernel_size, num_layers, dropout_p):
        super().__init__()
        assert num_layers > 1 and kernel_size % 2 == 1
        self.kernel_size = kernel_size
        self.num_layers = num_layers
        self.conv_layers = nn.ModuleList(
            [nn.Conv1d(in_channels if i == 0 else hidden_channels, hidden_channels, kernel_size,
                       padding=kernel_size // 2) for i in range(num_layers)])
        self.norm_layers = nn.ModuleList([LayerNorm(hidden_channels) for _ in range(num_layers)])
        self.proj = nn.Conv1d(hidden_channels, out_channels, 1)


class RelativePositionMultiHeadAttention(nn.Module):
    """transformer.py:10-115 (parameters only)."""

    def __init__(self, channels, out_channels, num_heads, rel_attn_window_size=None, heads_share=True,
                 dropout_p=0.0, input_length=None, proximal_bias=False, proximal_init=False):
        super().__init__()
        assert channels % num_heads == 0, " [!] channels should be divisible by num_heads."
        self.num_heads = num_heads
        self.rel_attn_window_size = rel_attn_window_size
        self.input_length = input_length
        self.k_channels = channels // num_heads
        self.conv_q = nn.Conv1d(channels, channels, 1)
        self.conv_k = nn.Conv1d(channels, channels, 1)
        self.conv_v = nn.Conv1d(channels, channels, 1)
        self.conv_o = nn.Conv1d(channels, out_channels, 1)
        if rel_attn_window_size is not None:
            n_heads_rel = 1 if heads_share else num_heads
            std = self.k_channels**-0.5
            self.emb_rel_k = nn.Parameter(torch.randn(n_heads_rel, rel_attn_window_size * 2 + 1, self.k_channels) * std)
            self.emb_rel_v = nn.Parameter(torch.randn(n_heads_rel, rel_attn_window_size * 2 + 1, self.k_channels) * std)


class FeedForwardNetwork(nn.Module):
    """transformer.py:285-341 (parameters only)."""

    def __init__(self, in_channels, out_channels, hidden_channels, kernel_size, dropout_p=0.0, causal=False):
        super().__init__()
        self.conv_1 = nn.Conv1d(in_channels, hidden_channels, kernel_size)
        self.conv_2 = nn.Conv1d(hidden_channels, out_channels, kernel_size)


class RelativePositionTransformer(nn.Module):
    """transformer.py:344-432 (parameters only; in = out = hidden as Encoder builds it)."""

    def __init__(self, in_channels, out_channels, hidden_channels, hidden_channels_ffn, num_heads, num_layers,
                 kernel_size=1, dropout_p=0.0, rel_attn_window_size=None, input_length=None, layer_norm_type="1"):
        super().__init__()
        if layer_norm_type not in ("1", "2"):
            raise ValueError(" [!] Unknown layer norm type")  # transformer.py:388-389
        self.layer_norm_type = layer_norm_type
        self.input_length = input_length
        self.num_layers = num_layers
        self.attn_layers = nn.ModuleList()
        self.norm_layers_1 = nn.ModuleList()
        self.ffn_layers = nn.ModuleList()
        self.norm_layers_2 = nn.ModuleList()
        for idx in range(num_layers):
            self.attn_layers.append(RelativePositionMultiHeadAttention(
                hidden_channels if idx != 0 else in_channels, hidden_channels, num_heads,
                rel_attn_window_size=rel_attn_window_size, dropout_p=dropout_p, input_length=input_length))
            Norm = LayerNorm if layer_norm_type == "1" else LayerNorm2
            self.norm_layers_1.append(Norm(hidden_channels))
            last = (idx + 1) == num_layers
            self.ffn_layers.append(FeedForwardNetwork(hidden_channels, out_channels if last else hidden_channels,
                                                      hidden_channels_ffn, kernel_size, dropout_p=dropout_p))
            self.norm_layers_2.append(Norm(out_channels if last else hidden_channels))


class GatedConvBlock(nn.Module):
    """generic/gated_conv.py:6-25 (parameters only)."""

    def __init__(self, in_out_channels, kernel_size, dropout_p, num_layers):
        super().__init__()
        self.dropout_p = dropout_p
        self.num_layers = num_layers
        self.kernel_size = kernel_size
        self.conv_layers = nn.ModuleList()
        self.norm_layers = nn.ModuleList()
        self.layers = nn.ModuleList()
        for _ in range(num_layers):
            self.conv_layers += [nn.Conv1d(in_out_channels, 2 * in_out_channels, kernel_size,
                                           padding=kernel_size // 2)]
            self.norm_layers += [LayerNorm(2 * in_out_channels)]


class Conv1dBN(nn.Module):
    """generic/res_conv_bn.py:19-44 (parameters only): conv (no padding) -> zero pad -> relu -> BN."""

    def __init__(self, in_channels, out_channels, kernel_size, dilation):
        super().__init__()
        self.conv1d = nn.Conv1d(in_channels, out_channels, kernel_size, dilation=dilation)
        self.norm = nn.BatchNorm1d(out_channels)


class Conv1dBNBlock(nn.Module):
    """generic/res_conv_bn.py:47-83 (parameters only)."""

    def __init__(self, in_channels, out_channels, hidden_channels, kernel_size, dilation, num_conv_blocks=2):
        super().__init__()
        self.conv_bn_blocks = nn.Sequential(*[
            Conv1dBN(in_channels if idx == 0 else hidden_channels,
                     out_channels if idx == (num_conv_blocks - 1) else hidden_channels, kernel_size, dilation)
            for idx in range(num_conv_blocks)])


class ResidualConv1dBNBlock(nn.Module):
    """generic/res_conv_bn.py:86-127 (parameters only)."""

    def __init__(self, in_channels, out_channels, hidden_channels, kernel_size, dilations, num_res_blocks=13,
                 num_conv_blocks=2):
        super().__init__()
        assert len(dilations) == num_res_blocks
        self.kernel_size = kernel_size
        self.dilations = list(dilations)
        self.num_conv_blocks = num_conv_blocks
        self.res_blocks = nn.ModuleList([
            Conv1dBNBlock(in_channels if idx == 0 else hidden_channels,
                          out_channels if (idx + 1) == len(dilations) else hidden_channels, hidden_channels,
                          kernel_size, dilation, num_conv_blocks)
            for idx, dilation in enumerate(dilations)])


class TimeDepthSeparableConv(nn.Module):
    """generic/time_depth_sep_conv.py:5-56 (parameters only)."""

    def __init__(self, in_channels, hid_channels, out_channels, kernel_size, bias=True):
        super().__init__()
        self.time_conv = nn.Conv1d(in_channels, 2 * hid_channels, kernel_size=1, stride=1, padding=0, bias=bias)
        self.norm1 = nn.BatchNorm1d(2 * hid_channels)
        self.depth_conv = nn.Conv1d(hid_channels, hid_channels, kernel_size, stride=1,
                                    padding=(kernel_size - 1) // 2, groups=hid_channels, bias=bias)
        self.norm2 = nn.BatchNorm1d(hid_channels)
        self.time_conv2 = nn.Conv1d(hid_channels, out_channels, kernel_size=1, stride=1, padding=0, bias=bias)
        self.norm3 = nn.BatchNorm1d(out_channels)


class TimeDepthSeparableConvBlock(nn.Module):
    """generic/time_depth_sep_conv.py:59-84 (parameters only)."""

    def __init__(self, in_channels, hid_channels, out_channels, num_layers, kernel_size, bias=True):
        super().__init__()
        assert (kernel_size - 1) % 2 == 0
        assert num_layers > 1
        self.kernel_size = kernel_size
        self.layers = nn.ModuleList()
        self.layers.append(TimeDepthSeparableConv(in_channels, hid_channels,
                                                  out_channels if num_layers == 1 else hid_channels, kernel_size,
                                                  bias))
        for idx in range(num_layers - 1):
            self.layers.append(TimeDepthSeparableConv(
                hid_channels, hid_channels, out_channels if (idx + 1) == (num_layers - 1) else hid_channels,
                kernel_size, bias))


class DurationPredictor(nn.Module):
    """duration_predictor.py:7-73 (parameters only)."""

    def __init__(self, in_channels, hidden_channels, kernel_size, dropout_p, cond_channels=None, language_emb_dim=None):
        super().__init__()
        self.conv_1 = nn.Conv1d(in_channels, hidden_channels, kernel_size, padding=kernel_size // 2)
        self.norm_1 = LayerNorm(hidden_channels)
        self.conv_2 = nn.Conv1d(hidden_channels, hidden_channels, kernel_size, padding=kernel_size // 2)
        self.norm_2 = LayerNorm(hidden_channels)
        self.proj = nn.Conv1d(hidden_channels, 1, 1)


def _f32(t: torch.Tensor) -> np.ndarray:
    return np.ascontiguousarray(t.detach().to("cpu", torch.float32).numpy())


class Encoder(nn.Module):
    def __init__(self, num_chars, out_channels, hidden_channels, hidden_channels_dp, encoder_type, encoder_params,
                 dropout_p_dp=0.1, mean_only=False, use_prenet=True, c_in_channels=0, math_mode: str = "fp32x6"):
        super().__init__()
        et = encoder_type.lower()
        if et not in N.ENCODER_TYPES:
            raise ValueError(" [!] Unkown encoder type.")  # encoder.py:123
        if math_mode not in N.MATH_MODES:
            raise ValueError(f"math_mode must be one of {sorted(N.MATH_MODES)}")
        self.num_chars = num_chars
        self.out_channels = out_channels
        self.hidden_channels = hidden_channels
        self.hidden_channels_dp = hidden_channels_dp
        self.mean_only = mean_only
        self.use_prenet = use_prenet
        self.c_in_channels = c_in_channels
        self.encoder_type = encoder_type
        self.encoder_params = dict(encoder_params)
        self.math_mode = math_mode
        self.emb = nn.Embedding(num_chars, hidden_channels)
        nn.init.normal_(self.emb.weight, 0.0, hidden_channels**-0.5)
        H = hidden_channels
        if et == "rel_pos_transformer":  # encoder.py:104-111
            if use_prenet:
                self.prenet = ResidualConv1dLayerNormBlock(H, H, H, kernel_size=5, num_layers=3, dropout_p=0.5)
            self.encoder = RelativePositionTransformer(H, H, H, **encoder_params)
        elif et == "gated_conv":  # :112-113
            self.encoder = GatedConvBlock(H, **encoder_params)
        elif et == "residual_conv_bn":  # :114-120
            if use_prenet:
                self.prenet = nn.Sequential(nn.Conv1d(H, H, 1), nn.ReLU())
            self.encoder = ResidualConv1dBNBlock(H, H, H, **encoder_params)
            self.postnet = nn.Sequential(nn.Conv1d(H, H, 1), nn.BatchNorm1d(H))
        else:  # time_depth_separable, :121-127
            if use_prenet:
                self.prenet = ResidualConv1dLayerNormBlock(H, H, H, kernel_size=5, num_layers=3, dropout_p=0.5)
            self.encoder = TimeDepthSeparableConvBlock(H, H, H, **encoder_params)
        self.proj_m = nn.Conv1d(hidden_channels, out_channels, 1)
        if not mean_only:
            self.proj_s = nn.Conv1d(hidden_channels, out_channels, 1)
        self.duration_predictor = DurationPredictor(hidden_channels + c_in_channels, hidden_channels_dp, 3,
                                                    dropout_p_dp)
        ep = self.encoder_params
        c = N.TtsGlowEncoderCfg()
        c.num_chars = num_chars
        c.out_channels = out_channels
        c.hidden_channels = hidden_channels
        c.hidden_channels_dp = hidden_channels_dp
        c.encoder_type = N.ENCODER_TYPES[et]
        c.kernel_size = self.encoder.kernel_size if et != "rel_pos_transformer" else ep.get("kernel_size", 1)
        if et == "rel_pos_transformer":
            c.hidden_channels_ffn = ep["hidden_channels_ffn"]
            c.num_heads = ep["num_heads"]
            c.num_layers = ep["num_layers"]
            c.rel_attn_window_size = ep.get("rel_attn_window_size") or 0
            c.layer_norm_type = 2 if self.encoder.layer_norm_type == "2" else 1
            if self.encoder.input_length is not None:
                c.has_input_length, c.input_length = 1, int(self.encoder.input_length)
        elif et == "residual_conv_bn":
            d = self.encoder.dilations
            if len(d) > 32:
                raise NotImplementedError("residual_conv_bn: more than 32 residual blocks")
            c.num_res_blocks = len(d)
            c.num_conv_blocks = self.encoder.num_conv_blocks
            for i, v in enumerate(d):
                c.dilations[i] = int(v)
        else:
            c.num_layers = len(self.encoder.layers) if et == "time_depth_separable" else self.encoder.num_layers
        c.mean_only = 1 if mean_only else 0
        # residual_conv_bn: the reference calls its nn.Sequential prenet with (x, x_mask) and raises
        # TypeError in forward (encoder.py:158); this module raises the same there
        self._prenet_typeerror = et == "residual_conv_bn" and use_prenet
        c.use_prenet = 1 if (use_prenet and not self._prenet_typeerror) else 0
        c.c_in_channels = c_in_channels
        c.math_mode = N.MATH_MODES[math_mode]
        self._cfg = c
        self._handle = None
        self._handle_key = None
        n = N.lib().tts_glow_encoder_num_weights(ctypes.byref(c))
        if n < 0:
            N.check("tts_glow_encoder_num_weights", -n)

    # ------------------------------------------------------------------ native handle
    def _weight_list(self) -> List[np.ndarray]:
        ws: List[np.ndarray] = [_f32(self.emb.weight)]

        def conv(m):
            ws.extend([_f32(m.weight), _f32(m.bias)])

        def norm(m):
            ws.extend([_f32(m.gamma).reshape(-1), _f32(m.beta).reshape(-1)])

        def bn(m):
            ws.extend([_f32(m.weight), _f32(m.bias), _f32(m.running_mean), _f32(m.running_var)])

        et = self.encoder_type.lower()
        if self.use_prenet and et in ("rel_pos_transformer", "time_depth_separable"):
            for l in range(3):
                conv(self.prenet.conv_layers[l])
                norm(self.prenet.norm_layers[l])
            conv(self.prenet.proj)
        enc = self.encoder
        if et == "gated_conv":
            for l in range(enc.num_layers):
                conv(enc.conv_layers[l])
                norm(enc.norm_layers[l])
        elif et == "residual_conv_bn":
            for blk in enc.res_blocks:
                for cb in blk.conv_bn_blocks:
                    conv(cb.conv1d)
                    bn(cb.norm)
            conv(self.postnet[0])
            bn(self.postnet[1])
        elif et == "time_depth_separable":
            for L in enc.layers:
                conv(L.time_conv)
                bn(L.norm1)
                conv(L.depth_conv)
                bn(L.norm2)
                conv(L.time_conv2)
                bn(L.norm3)
        for l in range(enc.num_layers if et == "rel_pos_transformer" else 0):
            a = enc.attn_layers[l]
            for m in (a.conv_q, a.conv_k, a.conv_v, a.conv_o):
                conv(m)
            if a.rel_attn_window_size is not None:
                if a.emb_rel_k.size(0) != 1:
                    raise NotImplementedError("heads_share=False relative embeddings are not implemented")
                ws.extend([_f32(a.emb_rel_k), _f32(a.emb_rel_v)])
            norm(enc.norm_layers_1[l])
            conv(enc.ffn_layers[l].conv_1)
            conv(enc.ffn_layers[l].conv_2)
            norm(enc.norm_layers_2[l])
        conv(self.proj_m)
        if not self.mean_only:
            conv(self.proj_s)
        dp = self.duration_predictor
        conv(dp.conv_1)
        norm(dp.norm_1)
        conv(dp.conv_2)
        norm(dp.norm_2)
        conv(dp.proj)
        return [np.ascontiguousarray(w) for w in ws]

    def _device(self) -> torch.device:
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("Encoder (tts_amd) runs only on a ROCm device: move it with .to('cuda') first")
        return dev

    def _native_handle(self):
        # BatchNorm running statistics are buffers: part of the key too
        key = tuple((p.data_ptr(), p._version, p.device) for p in list(self.parameters()) + list(self.buffers()))
        if self._handle is not None and key == self._handle_key:
            return self._handle
        self._release()
        dev = self._device()
        ws = self._weight_list()
        lib = N.lib()
        for i, w in enumerate(ws):
            n = lib.tts_glow_encoder_weight_numel(ctypes.byref(self._cfg), i)
            if n != w.size:
                raise ValueError(f"weight {i} has {w.size} elements, expected {n}")
        arr = (ctypes.c_void_p * len(ws))(*[w.ctypes.data for w in ws])
        h = ctypes.c_void_p()
        N.call("tts_glow_encoder_create", ctypes.byref(self._cfg), arr, dev.index or 0, ctypes.byref(h))
        self._handle, self._handle_key = h, key
        return h

    def _release(self):
        if getattr(self, "_handle", None) is not None:
            N.lib().tts_glow_encoder_destroy(self._handle)
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

    def _speaker(self, g: Optional[torch.Tensor], B: int, dev: torch.device) -> Optional[torch.Tensor]:
        """g [B, c_in, 1] (encoder.py:166-168 expands it over time) -> contiguous fp32 [B, c_in]."""
        if not self.c_in_channels:
            if g is not None:
                raise ValueError("g given to an encoder built with c_in_channels=0")
            return None
        if g is None:
            raise ValueError(f"this encoder is speaker-conditioned: g [B, {self.c_in_channels}, 1] is required")
        if g.dim() == 3 and g.shape[-1] == 1:
            g = g[..., 0]
        if g.shape != (B, self.c_in_channels):
            raise ValueError(f"g must be [{B}, {self.c_in_channels}, 1], got {tuple(g.shape)}")
        return g.to(device=dev, dtype=torch.float32).contiguous()

    def _io(self, x, x_lengths, g=None):
        dev = self._device()
        tok = x.to(device=dev, dtype=torch.int64).contiguous()
        lens = x_lengths.to(device=dev, dtype=torch.int64).contiguous()
        B, T = tok.shape
        if lens.shape != (B,):
            raise ValueError(f"x_lengths must be [B] = [{B}], got {tuple(lens.shape)}")
        gv = self._speaker(g, B, dev)
        x_m = torch.empty(B, self.out_channels, T, device=dev)
        x_logs = torch.empty_like(x_m)
        logw = torch.empty(B, 1, T, device=dev)
        x_mask = torch.empty(B, 1, T, device=dev)
        return dev, tok, lens, gv, (x_m, x_logs, logw, x_mask)

    # ------------------------------------------------------------------ reference API
    def forward(self, x: torch.Tensor, x_lengths: torch.Tensor, g: Optional[torch.Tensor] = None):
        """encoder.py:143-179: x [B, T] token ids, x_lengths [B], g [B, c_in, 1] (speaker vector of a
        c_in_channels > 0 encoder, concatenated to the duration predictor's input, :166-168)
        -> (x_m, x_logs, logw, x_mask)."""
        if self._prenet_typeerror:
            raise TypeError("Sequential.forward() takes 2 positional arguments but 3 were given")
        with torch.no_grad():
            h = self._native_handle()
            dev, tok, lens, gv, outs = self._io(x, x_lengths, g)
            B, T = tok.shape
            N.call("tts_glow_encoder_forward", h, N.ptr(tok), N.ptr(lens), N.ptr(gv), B, T,
                   *[N.ptr(o) for o in outs], N.stream_ptr(dev))
        return outs

    def profile(self, x: torch.Tensor, x_lengths: torch.Tensor, g: Optional[torch.Tensor] = None):
        """One forward with a hipEvent pair around every launch: (outputs, [{name, flops, bytes, ms}])."""
        h = self._native_handle()
        dev, tok, lens, gv, outs = self._io(x, x_lengths, g)
        B, T = tok.shape
        cap = 1024
        recs = (N.TtsLaunchRecord * cap)()
        n = ctypes.c_int(0)
        N.call("tts_glow_encoder_forward_profiled", h, N.ptr(tok), N.ptr(lens), N.ptr(gv), B, T,
               *[N.ptr(o) for o in outs], N.stream_ptr(dev), recs, cap, ctypes.byref(n))
        rows = [{"name": recs[i].name.decode(), "flops": recs[i].flops, "bytes": recs[i].bytes, "ms": recs[i].ms}
                for i in range(min(n.value, cap))]
        return outs, rows


def _cfg_get(config, key, default):
    if config is None:
        return default
    if isinstance(config, dict):
        return config.get(key, default)
    return getattr(config, key, default)


class GlowTTS(nn.Module):
    """Inference surface of ``TTS/tts/models/glow_tts.py`` (GlowTTS, :22-530) on the MI355X path.

    ``config`` is a ``GlowTTSConfig``-like object or dict with the reference's field names
    (glow_tts_config.py:103-152); missing fields take the reference defaults.  ``num_chars`` is
    required (the reference takes it from the tokenizer, glow_tts.py:63-66).
    ``math_mode`` / ``decoder_math_mode`` select the conv arithmetic.  The encoder's durations are
    ceil()-quantised, so it runs an fp32-faithful mode: ``"fp32x6"`` by default (bf16x6 split, as
    accurate as fp32 against the fp64 reference) or ``"fp32"``; the decoder defaults to the same."""

    def __init__(self, config=None, math_mode: str = "fp32x6", decoder_math_mode: Optional[str] = None, **overrides):
        super().__init__()
        cfg = dict(overrides)

        def get(key, default):
            return cfg[key] if key in cfg else _cfg_get(config, key, default)

        self.num_chars = get("num_chars", None)
        if self.num_chars is None:
            raise ValueError("num_chars is required")
        self.out_channels = get("out_channels", GLOW_TTS_ENCODER["out_channels"])
        self.encoder_type = get("encoder_type", GLOW_TTS_ENCODER["encoder_type"])
        self.encoder_params = dict(get("encoder_params", GLOW_TTS_ENCODER["encoder_params"]))
        self.encoder_params.pop("dropout_p", None)
        if self.encoder_params.get("input_length", None) is None:
            self.encoder_params.pop("input_length", None)
        self.hidden_channels_enc = get("hidden_channels_enc", GLOW_TTS_ENCODER["hidden_channels"])
        self.hidden_channels_dec = get("hidden_channels_dec", GLOW_TTS_DECODER["hidden_channels"])
        self.hidden_channels_dp = get("hidden_channels_dp", GLOW_TTS_ENCODER["hidden_channels_dp"])
        self.mean_only = get("mean_only", GLOW_TTS_ENCODER["mean_only"])
        self.use_encoder_prenet = get("use_encoder_prenet", GLOW_TTS_ENCODER["use_prenet"])
        self.num_flow_blocks_dec = get("num_flow_blocks_dec", GLOW_TTS_DECODER["num_flow_blocks"])
        self.kernel_size_dec = get("kernel_size_dec", GLOW_TTS_DECODER["kernel_size"])
        self.dilation_rate = get("dilation_rate", GLOW_TTS_DECODER["dilation_rate"])
        self.num_block_layers = get("num_block_layers", GLOW_TTS_DECODER["num_coupling_layers"])
        self.num_splits = get("num_splits", GLOW_TTS_DECODER["num_splits"])
        self.num_squeeze = get("num_squeeze", GLOW_TTS_DECODER["num_squeeze"])
        self.sigmoid_scale = get("sigmoid_scale", GLOW_TTS_DECODER["sigmoid_scale"])
        self.inference_noise_scale = get("inference_noise_scale", GLOW_TTS_INFERENCE["inference_noise_scale"])
        self.length_scale = get("length_scale", GLOW_TTS_INFERENCE["length_scale"])
        # init_multispeaker (glow_tts.py:107-135): emb_g is registered before the encoder, as there
        self.num_speakers = get("num_speakers", 0)
        self.use_speaker_embedding = get("use_speaker_embedding", False)
        self.use_d_vector_file = get("use_d_vector_file", False)
        self.embedded_speaker_dim = 0
        if self.use_d_vector_file:
            d = get("d_vector_dim", None)
            self.embedded_speaker_dim = d if d is not None else 512
        if self.use_speaker_embedding and not self.use_d_vector_file:
            self.embedded_speaker_dim = self.hidden_channels_enc
            self.emb_g = nn.Embedding(self.num_speakers, self.hidden_channels_enc)
            nn.init.uniform_(self.emb_g.weight, -0.1, 0.1)
        self.c_in_channels = self.embedded_speaker_dim
        self.encoder = Encoder(self.num_chars, out_channels=self.out_channels,
                               hidden_channels=self.hidden_channels_enc, hidden_channels_dp=self.hidden_channels_dp,
                               encoder_type=self.encoder_type, encoder_params=self.encoder_params,
                               mean_only=self.mean_only, use_prenet=self.use_encoder_prenet,
                               dropout_p_dp=get("dropout_p_dp", 0.1), c_in_channels=self.c_in_channels,
                               math_mode=math_mode)
        self.decoder = Decoder(self.out_channels, self.hidden_channels_dec, self.kernel_size_dec, self.dilation_rate,
                               self.num_flow_blocks_dec, self.num_block_layers,
                               dropout_p=get("dropout_p_dec", 0.05), num_splits=self.num_splits,
                               num_squeeze=self.num_squeeze, sigmoid_scale=self.sigmoid_scale,
                               c_in_channels=self.c_in_channels,
                               math_mode=decoder_math_mode or math_mode)

    def _device(self) -> torch.device:
        return self.encoder._device()

    def _set_speaker_input(self, aux_input: Optional[Dict]):  # glow_tts.py:162-177
        d_vectors = None if aux_input is None else aux_input.get("d_vectors", None)
        speaker_ids = None if aux_input is None else aux_input.get("speaker_ids", None)
        if d_vectors is not None and speaker_ids is not None:
            raise ValueError("[!] Cannot use d-vectors and speaker-ids together.")
        if speaker_ids is not None and not hasattr(self, "emb_g"):
            raise ValueError("[!] Cannot use speaker-ids without enabling speaker embedding.")
        return speaker_ids if speaker_ids is not None else d_vectors

    def _speaker_embedding(self, aux_input: Optional[Dict]) -> Optional[torch.Tensor]:  # glow_tts.py:179-191
        """speaker ids -> F.normalize(emb_g(ids)) or d-vectors -> F.normalize(d): [B, c_in, 1].
        A few hundred floats: the lookup and the normalisation stay in torch on the device."""
        g = self._set_speaker_input(aux_input)
        if g is None:
            return None
        if not self.c_in_channels:
            raise ValueError("d_vectors given to a single-speaker model (use_d_vector_file=False)")
        dev = self._device()
        if hasattr(self, "emb_g"):
            g = g.to(dev)
            if not g.size():
                g = g.unsqueeze(0)
            return F.normalize(self.emb_g(g)).unsqueeze(-1)
        return F.normalize(g.to(device=dev, dtype=torch.float32)).unsqueeze(-1)

    @torch.no_grad()
    def inference(self, x, aux_input={"x_lengths": None, "d_vectors": None, "speaker_ids": None}):  # noqa: B006
        """glow_tts.py:342-374.  ``aux_input["noise"]`` (optional, [B, out, T_y]) replaces
        ``torch.randn_like(y_mean)`` so that a caller can pin the sampling noise.  ``speaker_ids``
        or ``d_vectors`` condition a multi-speaker model (both encoder and decoder, :346-365)."""
        x_lengths = aux_input["x_lengths"]
        g = self._speaker_embedding(aux_input)
        if self.c_in_channels and g is None:
            raise ValueError("multi-speaker Glow-TTS: pass aux_input speaker_ids or d_vectors")
        dev = self._device()
        o_mean, o_log_scale, o_dur_log, x_mask = self.encoder(x, x_lengths, g=g)
        B, C, T_x = o_mean.shape
        w_ceil = torch.empty(B, 1, T_x, device=dev)
        y_lengths = torch.empty(B, dtype=torch.int64, device=dev)
        o_attn_dur = torch.empty(B, 1, T_x, device=dev)
        stream = N.stream_ptr(dev)
        N.call("tts_glow_durations", N.ptr(o_dur_log), N.ptr(x_mask), B, T_x, float(self.length_scale),
               N.ptr(w_ceil), N.ptr(y_lengths), N.ptr(o_attn_dur), stream)
        T_y = int(y_lengths.max().item())  # sequence_mask(y_lengths, None) (glow_tts.py:353)
        noise = aux_input.get("noise")
        if noise is not None:
            noise = noise.to(device=dev, dtype=torch.float32).contiguous()
            if noise.shape != (B, C, T_y):
                raise ValueError(f"noise must be [{B}, {C}, {T_y}], got {tuple(noise.shape)}")
        elif self.inference_noise_scale != 0:
            noise = torch.randn(B, C, T_y, device=dev)
        z = torch.empty(B, C, T_y, device=dev)
        y_mask = torch.empty(B, 1, T_y, device=dev)
        y_mean = torch.empty(B, C, T_y, device=dev)
        y_log_scale = torch.empty(B, C, T_y, device=dev)
        attn = torch.empty(B, T_x, T_y, device=dev)
        N.call("tts_glow_expand", N.ptr(w_ceil), N.ptr(x_mask), N.ptr(y_lengths), N.ptr(o_mean),
               N.ptr(None if self.mean_only else o_log_scale), N.ptr(noise), float(self.inference_noise_scale),
               B, C, T_x, T_y, N.ptr(z), N.ptr(y_mask), N.ptr(y_mean), N.ptr(y_log_scale), N.ptr(attn), stream)
        y, logdet = self.decoder(z, y_mask, g=g, reverse=True)
        return {
            "model_outputs": y.transpose(1, 2),
            "logdet": logdet,
            "y_mean": y_mean.transpose(1, 2),
            "y_log_scale": y_log_scale.transpose(1, 2),
            "alignments": attn.permute(0, 2, 1),
            "durations_log": o_dur_log.transpose(1, 2),
            "total_durations_log": o_attn_dur.transpose(1, 2),
        }

    @torch.no_grad()
    def decoder_inference(self, y, y_lengths=None, aux_input={"d_vectors": None, "speaker_ids": None}):  # noqa: B006
        """glow_tts.py:319-339: the decoder forward (mel -> z, reverse=False) then reverse (z -> mel),
        y: [B, T, C] mel frames, y_lengths: [B].  Returns {"model_outputs": [B, T', C], "logdet": None}
        (the reverse pass's logdet, as the reference's)."""
        dev = self._device()
        y = y.to(device=dev, dtype=torch.float32).transpose(1, 2)
        B, _, T = y.shape
        g = self._speaker_embedding(aux_input)
        if self.c_in_channels and g is None:
            raise ValueError("multi-speaker Glow-TTS: pass aux_input speaker_ids or d_vectors")
        if y_lengths is None:
            y_lengths = torch.full((B,), T, device=dev)
        lens = torch.as_tensor(y_lengths, device=dev).reshape(B)
        y_mask = (torch.arange(T, device=dev)[None, :] < lens[:, None]).to(torch.float32).unsqueeze(1)  # :331
        z, logdet = self.decoder(y, y_mask, g=g, reverse=False)  # :333
        y, logdet = self.decoder(z, y_mask[:, :, : z.shape[2]], g=g, reverse=True)  # :335
        return {"model_outputs": y.transpose(1, 2), "logdet": logdet}

    def store_inverse(self):  # glow_tts.py:519-520
        self.decoder.store_inverse()

    def load_checkpoint(self, config, checkpoint_path, eval=False, cache=False):  # glow_tts.py:522-530
        state = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        self.load_state_dict(state["model"] if "model" in state else state)
        if eval:
            self.eval()
            self.store_inverse()
            assert not self.training


__all__ = ["Encoder", "GlowTTS"]
