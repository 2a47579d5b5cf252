"""Drop-in ``HifiganGenerator`` whose compute runs in ``libtts_mi355x.so`` on MI355X.

Mirrors ``TTS/vocoder/models/hifigan_generator.py`` (Coqui TTS 0.22.0):

* same constructor arguments (:163-178) and the same parameter tree, so reference checkpoints
  load with identical ``state_dict`` keys, weight-norm parametrized (``…parametrizations.weight
  .original0/1``) or folded;
* ``forward(x, g=None)`` (:236-265), ``inference(c)`` (:267-282, replicate pad of
  ``inference_padding`` frames), ``remove_weight_norm()`` (:284-291) and
  ``load_checkpoint(config, path, eval)`` (:293-301) behave like the reference.

The ``torch.nn`` conv modules below only hold parameters; their ``forward`` is never called.
The first call on a ROCm device folds weight norm with PyTorch's own ``_weight_norm`` (the
values ``remove_weight_norm`` would store), hands the folded fp32 weights to
``tts_hifigan_create`` which packs them into the MFMA kernel layout in HBM, and every call
after that is one C-ABI call on the current stream.  The handle is rebuilt automatically
when any parameter changes (data pointer or in-place version counter).

There is no CPU path: inputs must be on (or are moved to) the parameters' ROCm device, and
a module whose parameters are on the CPU raises instead of silently computing elsewhere.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np
import torch
from torch import nn
from torch.nn import Conv1d, ConvTranspose1d
from torch.nn.utils.parametrizations import weight_norm
from torch.nn.utils.parametrize import is_parametrized, remove_parametrizations

from .. import _native as N

LRELU_SLOPE = 0.1  # hifigan_generator.py:11


def get_padding(k: int, d: int) -> int:  # :14-15
    return int((k * d - d) / 2)


class ResBlock1(nn.Module):
    """Parameter container of ResBlock1 (:18-105): convs1 (dilated) and convs2 (dilation 1)."""

    def __init__(self, channels: int, kernel_size: int = 3, dilation=(1, 3, 5)):
        super().__init__()
        self.convs1 = nn.ModuleList(
            [weight_norm(Conv1d(channels, channels, kernel_size, 1, dilation=d, padding=get_padding(kernel_size, d)))
             for d in dilation[:3]]
        )
        self.convs2 = nn.ModuleList(
            [weight_norm(Conv1d(channels, channels, kernel_size, 1, dilation=1, padding=get_padding(kernel_size, 1)))
             for _ in range(3)]
        )

    def conv_order(self) -> List[nn.Module]:
        return list(self.convs1) + list(self.convs2)

    def remove_weight_norm(self):
        for l in self.conv_order():
            if is_parametrized(l, "weight"):
                remove_parametrizations(l, "weight")


class ResBlock2(nn.Module):
    """Parameter container of ResBlock2 (:108-159)."""

    def __init__(self, channels: int, kernel_size: int = 3, dilation=(1, 3)):
        super().__init__()
        self.convs = nn.ModuleList(
            [weight_norm(Conv1d(channels, channels, kernel_size, 1, dilation=d, padding=get_padding(kernel_size, d)))
             for d in dilation[:2]]
        )

    def conv_order(self) -> List[nn.Module]:
        return list(self.convs)

    def remove_weight_norm(self):
        for l in self.convs:
            if is_parametrized(l, "weight"):
                remove_parametrizations(l, "weight")


def _effective_weight(m: nn.Module) -> np.ndarray:
    # For a parametrized module ``m.weight`` evaluates torch._weight_norm(v, g, 0): the same
    # values remove_parametrizations(m, "weight") would store (hifigan_generator.py:284-291).
    with torch.no_grad():
        return np.ascontiguousarray(m.weight.detach().to("cpu", torch.float32).numpy())


def _host(t: Optional[torch.Tensor]) -> np.ndarray:
    return np.ascontiguousarray(t.detach().to("cpu", torch.float32).numpy())


class HifiganGenerator(nn.Module):
    def __init__(
        self,
        in_channels: int,
        out_channels: int,
        resblock_type: str,
        resblock_dilation_sizes: Sequence[Sequence[int]],
        resblock_kernel_sizes: Sequence[int],
        upsample_kernel_sizes: Sequence[int],
        upsample_initial_channel: int,
        upsample_factors: Sequence[int],
        inference_padding: int = 5,
        cond_channels: int = 0,
        conv_pre_weight_norm: bool = True,
        conv_post_weight_norm: bool = True,
        conv_post_bias: bool = True,
        math_mode: Optional[str] = None,
        cond_in_each_up_layer: bool = False,
    ):
        """Arguments as the reference (:163-178).  ``math_mode`` selects how the conv contractions
        run on MI355X (all take and return fp32; include/tts_mi355x.h TTS_MATH_*):

        * ``"f16x3"`` (the default, unless ``$TTS_MI355X_MATH_MODE`` names another): each fp32
          operand scaled by an exact power of two and split into fp16 hi + lo, the three products
          hi*hi + hi*lo + lo*hi accumulated in fp32 on the fp16 matrix cores.  Its error against the
          fp64 oracle is at or below the exact-fp32 mode's at 3x the speed.
        * ``"fp32"``: v_mfma_f32_32x32x2_f32, exact fp32 products.
        * ``"fp32x6"``: 3 exact bf16 pieces per operand, the 6 leading cross products.
        * ``"bf16"``: bf16 operands, fp32 accumulation (lower precision; VITS / Glow-TTS configs).

        ``cond_in_each_up_layer`` is the XTTS
        generator's option (TTS/tts/layers/xtts/hifigan_decoder.py:199, :240-244, :276-279):
        ``o = ups[i](o) + conds[i](g)`` after every upsampling."""
        super().__init__()
        if math_mode is None:
            math_mode = N.default_math_mode()
        if math_mode not in N.MATH_MODES:
            raise ValueError(f"math_mode must be one of {sorted(N.MATH_MODES)}")
        self.math_mode = math_mode
        self.inference_padding = inference_padding
        self.num_kernels = len(resblock_kernel_sizes)
        self.num_upsamples = len(upsample_factors)
        self.resblock_type = str(resblock_type)
        self._cfg = N.TtsHifiganCfg()
        c = self._cfg
        c.in_channels = in_channels
        c.out_channels = out_channels
        c.resblock_type = 1 if self.resblock_type == "1" else 2
        if len(resblock_kernel_sizes) > N.MAX_KERNELS or len(upsample_factors) > N.MAX_UPSAMPLES:
            raise ValueError("too many resblocks / upsample layers for the native configuration")
        c.num_kernels = len(resblock_kernel_sizes)
        for j, k in enumerate(resblock_kernel_sizes):
            c.resblock_kernel_sizes[j] = int(k)
        nd = len(resblock_dilation_sizes[0]) if len(resblock_dilation_sizes) else 0
        c.num_dilations = min(nd, N.MAX_DILATIONS)
        for j, ds in enumerate(resblock_dilation_sizes[: N.MAX_KERNELS]):
            for m, d in enumerate(list(ds)[: N.MAX_DILATIONS]):
                c.resblock_dilation_sizes[j][m] = int(d)
        c.num_upsamples = len(upsample_factors)
        for i, (u, k) in enumerate(zip(upsample_factors, upsample_kernel_sizes)):
            c.upsample_factors[i] = int(u)
            c.upsample_kernel_sizes[i] = int(k)
        c.upsample_initial_channel = upsample_initial_channel
        c.inference_padding = inference_padding
        c.cond_channels = cond_channels
        c.conv_post_bias = 1 if conv_post_bias else 0
        c.math_mode = N.MATH_MODES[math_mode]
        c.cond_in_each_up_layer = 1 if cond_in_each_up_layer else 0
        self.cond_in_each_up_layer = cond_in_each_up_layer
        self.hop_length = int(np.prod(upsample_factors))

        # parameter tree identical to the reference (:203-234)
        self.conv_pre = weight_norm(Conv1d(in_channels, upsample_initial_channel, 7, 1, padding=3))
        resblock = ResBlock1 if self.resblock_type == "1" else ResBlock2
        self.ups = nn.ModuleList()
        for i, (u, k) in enumerate(zip(upsample_factors, upsample_kernel_sizes)):
            self.ups.append(
                weight_norm(
                    ConvTranspose1d(
                        upsample_initial_channel // (2**i),
                        upsample_initial_channel // (2 ** (i + 1)),
                        k,
                        u,
                        padding=(k - u) // 2,
                    )
                )
            )
        self.resblocks = nn.ModuleList()
        for i in range(len(self.ups)):
            ch = upsample_initial_channel // (2 ** (i + 1))
            for k, d in zip(resblock_kernel_sizes, resblock_dilation_sizes):
                self.resblocks.append(resblock(ch, k, d))
        self.conv_post = weight_norm(Conv1d(ch, out_channels, 7, 1, padding=3, bias=conv_post_bias))
        if cond_channels > 0:
            self.cond_layer = nn.Conv1d(cond_channels, upsample_initial_channel, 1)
        if not conv_pre_weight_norm:
            remove_parametrizations(self.conv_pre, "weight")
        if not conv_post_weight_norm:
            remove_parametrizations(self.conv_post, "weight")
        if cond_in_each_up_layer:  # xtts/hifigan_decoder.py:240-244
            self.conds = nn.ModuleList()
            for i in range(len(self.ups)):
                ch = upsample_initial_channel // (2 ** (i + 1))
                self.conds.append(nn.Conv1d(cond_channels, ch, 1))

        self._handle = None
        self._handle_key = None
        # fail at construction for configurations the native path cannot run
        n = N.lib().tts_hifigan_num_weights(ctypes.byref(self._cfg))
        if n < 0:
            N.check("tts_hifigan_num_weights", -n)

    # ------------------------------------------------------------------ native handle
    def _weight_list(self) -> List[np.ndarray]:
        """Folded fp32 weights in the C-ABI order (include/tts_mi355x.h)."""
        ws: List[np.ndarray] = [_effective_weight(self.conv_pre), _host(self.conv_pre.bias)]
        for u in self.ups:
            ws += [_effective_weight(u), _host(u.bias)]
        for rb in self.resblocks:
            for cv in rb.conv_order():
                ws += [_effective_weight(cv), _host(cv.bias)]
        ws.append(_effective_weight(self.conv_post))
        if self.conv_post.bias is not None:
            ws.append(_host(self.conv_post.bias))
        if hasattr(self, "cond_layer"):
            ws += [_effective_weight(self.cond_layer), _host(self.cond_layer.bias)]
        if self.cond_in_each_up_layer:
            for cv in self.conds:
                ws += [_effective_weight(cv), _host(cv.bias)]
        return ws

    def _param_key(self):
        return tuple((p.data_ptr(), p._version, p.device) for p in self.parameters())

    def _device(self) -> torch.device:
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError(
                "HifiganGenerator (tts_amd) runs only on a ROCm device: move the module with "
                ".to('cuda') first (there is no CPU fallback)"
            )
        return dev

    def _native_handle(self):
        key = self._param_key()
        if self._handle is not None and key == self._handle_key:
            return self._handle
        self._release()
        dev = self._device()
        ws = self._weight_list()
        lib = N.lib()
        expected = lib.tts_hifigan_num_weights(ctypes.byref(self._cfg))
        if expected < 0:
            N.check("tts_hifigan_num_weights", -expected)
        if expected != len(ws):
            raise RuntimeError(f"internal: {len(ws)} weight tensors, library expects {expected}")
        for i, w in enumerate(ws):
            n = lib.tts_hifigan_weight_numel(ctypes.byref(self._cfg), i)
            if n != w.size:
                raise ValueError(f"weight {i} has {w.size} elements, expected {n}")
        arr = (ctypes.c_void_p * len(ws))(*[w.ctypes.data for w in ws])
        h = ctypes.c_void_p()
        N.call("tts_hifigan_create", ctypes.byref(self._cfg), arr, dev.index or 0, ctypes.byref(h))
        self._handle, self._handle_key = h, key
        return h

    def _release(self):
        if getattr(self, "_handle", None) is not None:
            N.lib().tts_hifigan_destroy(self._handle)
            self._handle = None
            self._handle_key = None

    def __del__(self):
        try:
            self._release()
        except Exception:  # interpreter shutdown
            pass

    # ------------------------------------------------------------------ reference API
    def _run(self, x: torch.Tensor, pad: int, g: Optional[torch.Tensor]) -> torch.Tensor:
        h = self._native_handle()
        dev = self._device()
        if x.dim() != 3:
            raise ValueError(f"expected [B, C, T] input, got shape {tuple(x.shape)}")
        x = x.to(device=dev, dtype=torch.float32).contiguous()
        B, C, T = x.shape
        if C != self._cfg.in_channels:
            raise ValueError(f"input has {C} channels, generator expects {self._cfg.in_channels}")
        gv = None
        if self._cfg.cond_channels > 0:
            if g is None:
                raise ValueError("this generator has cond_channels > 0: pass g")
            gv = g.to(device=dev, dtype=torch.float32).reshape(B, self._cfg.cond_channels).contiguous()
        out = torch.empty(B, self._cfg.out_channels, self.hop_length * (T + 2 * pad), device=dev,
                          dtype=torch.float32)
        N.call("tts_hifigan_forward", h, N.ptr(x), B, C, T, pad, N.ptr(gv), N.ptr(out), N.stream_ptr(dev))
        return out

    def forward(self, x: torch.Tensor, g: Optional[torch.Tensor] = None) -> torch.Tensor:
        """hifigan_generator.py:236-265 (no inference padding).  Inference only."""
        with torch.no_grad():
            return self._run(x, 0, g)

    @torch.no_grad()
    def inference(self, c: torch.Tensor, g: Optional[torch.Tensor] = None) -> torch.Tensor:
        """hifigan_generator.py:267-282: move to the weight device, replicate-pad, forward."""
        return self._run(c, self.inference_padding, g)

    def profile(self, c: torch.Tensor, pad: Optional[int] = None, g: Optional[torch.Tensor] = None):
        """One forward with a hipEvent pair around every kernel launch (g: the conditioning vector of a
        cond_channels > 0 generator).  Returns (wav, [ {name, flops, bytes, ms}, ... ])."""
        h = self._native_handle()
        dev = self._device()
        pad = self.inference_padding if pad is None else pad
        x = c.to(device=dev, dtype=torch.float32).contiguous()
        B, C, T = x.shape
        gg = None
        if g is not None:
            gg = g.to(device=dev, dtype=torch.float32).reshape(B, -1).contiguous()
        out = torch.empty(B, self._cfg.out_channels, self.hop_length * (T + 2 * pad), device=dev)
        cap = 4096  # windowed long utterances run ~80 launches per window
        recs = (N.TtsLaunchRecord * cap)()
        n = ctypes.c_int(0)
        N.call("tts_hifigan_forward_profiled", h, N.ptr(x), B, C, T, pad, N.ptr(gg), N.ptr(out),
               N.stream_ptr(dev), recs, cap, ctypes.byref(n))
        rows = [
            {"name": recs[i].name.decode(), "flops": recs[i].flops, "bytes": recs[i].bytes, "ms": recs[i].ms}
            for i in range(min(n.value, cap))
        ]
        return out, rows

    def reserve(self, batch: int, frames: int, pad: Optional[int] = None) -> None:
        """Pre-allocate the activation workspace for [batch, C, frames] inputs."""
        pad = self.inference_padding if pad is None else pad
        N.call("tts_hifigan_reserve", self._native_handle(), batch, frames, pad)

    def remove_weight_norm(self):
        """hifigan_generator.py:284-291 (idempotent here)."""
        print("Removing weight norm...")
        for l in self.ups:
            if is_parametrized(l, "weight"):
                remove_parametrizations(l, "weight")
        for l in self.resblocks:
            l.remove_weight_norm()
        for l in (self.conv_pre, self.conv_post):
            if is_parametrized(l, "weight"):
                remove_parametrizations(l, "weight")
        self._release()

    def load_checkpoint(self, config, checkpoint_path, eval=False, cache=False):  # noqa: A002
        """hifigan_generator.py:293-301.  Checkpoints are read with weights_only=True."""
        from ..io import load_fsspec

        state = load_fsspec(checkpoint_path, map_location=torch.device("cpu"), cache=cache)
        self.load_state_dict(state["model"])
        if eval:
            self.eval()
            assert not self.training
            self.remove_weight_norm()

    def _apply(self, fn, *args, **kwargs):
        self._release()
        return super()._apply(fn, *args, **kwargs)
