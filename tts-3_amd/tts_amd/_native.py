"""ctypes binding of ``libtts_mi355x.so`` (the C-ABI in ``include/tts_mi355x.h``).

The library is the only compute path of this package: there is no CPU or PyTorch fallback.
If the shared object is missing or fails to load, every entry point raises.

``torch`` is imported before the library is opened so that the library's ``DT_NEEDED``
``libamdhip64.so.7`` binds to the HIP runtime PyTorch already loaded (one runtime per process:
device pointers and streams from PyTorch are then valid inside the library).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_char, c_char_p, c_double, c_float, c_int, c_int64, c_void_p

import torch  # noqa: F401  (load order: see module docstring)

_LIB_NAME = "libtts_mi355x.so"
_LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
LIB_PATH = os.environ.get("TTS_MI355X_LIB", os.path.join(_LIB_DIR, _LIB_NAME))

TTS_OK = 0
TTS_ERR_INVALID = 1
TTS_ERR_HIP = 2
TTS_ERR_UNSUPPORTED = 3
TTS_ERR_OOM = 4

# math modes (TTS_MATH_* in tts_mi355x.h)
MATH_MODES = {"fp32": 0, "fp32x6": 1, "f16x3": 2, "bf16": 3}

# the C-ABI revision these bindings were written for (tts_abi_version() in csrc/abi.cpp)
ABI_VERSION = 115


def default_math_mode(fp32_faithful_only: bool = True) -> str:
    """Math mode of a module built without an explicit ``math_mode``: ``$TTS_MI355X_MATH_MODE`` if
    set, else ``"f16x3"`` (fp32 in / fp32 out, measured at or below the exact-fp32 MFMA mode's error
    against the fp64 oracle, DESIGN.md section 3, and 3x its speed).  ``bf16`` is a lower-precision
    mode and is only taken from the environment when the caller allows it."""
    m = os.environ.get("TTS_MI355X_MATH_MODE", "f16x3")
    if m not in MATH_MODES:
        raise ValueError(f"TTS_MI355X_MATH_MODE={m!r}: must be one of {sorted(MATH_MODES)}")
    if fp32_faithful_only and m == "bf16":
        raise ValueError("TTS_MI355X_MATH_MODE=bf16 is not fp32-faithful; pass math_mode='bf16' explicitly")
    return m

MAX_UPSAMPLES = 8
MAX_KERNELS = 4
MAX_DILATIONS = 4


class TtsHifiganCfg(Structure):
    _fields_ = [
        ("in_channels", c_int),
        ("out_channels", c_int),
        ("resblock_type", c_int),
        ("num_kernels", c_int),
        ("resblock_kernel_sizes", c_int * MAX_KERNELS),
        ("num_dilations", c_int),
        ("resblock_dilation_sizes", (c_int * MAX_DILATIONS) * MAX_KERNELS),
        ("num_upsamples", c_int),
        ("upsample_factors", c_int * MAX_UPSAMPLES),
        ("upsample_kernel_sizes", c_int * MAX_UPSAMPLES),
        ("upsample_initial_channel", c_int),
        ("inference_padding", c_int),
        ("cond_channels", c_int),
        ("conv_post_bias", c_int),
        ("math_mode", c_int),
        ("cond_in_each_up_layer", c_int),
    ]


class TtsGlowDecoderCfg(Structure):
    _fields_ = [
        ("in_channels", c_int),
        ("hidden_channels", c_int),
        ("kernel_size", c_int),
        ("dilation_rate", c_int),
        ("num_flow_blocks", c_int),
        ("num_coupling_layers", c_int),
        ("num_splits", c_int),
        ("num_squeeze", c_int),
        ("sigmoid_scale", c_int),
        ("c_in_channels", c_int),
        ("math_mode", c_int),
    ]


class TtsGlowEncoderCfg(Structure):
    _fields_ = [
        ("num_chars", c_int),
        ("out_channels", c_int),
        ("hidden_channels", c_int),
        ("hidden_channels_dp", c_int),
        ("hidden_channels_ffn", c_int),
        ("num_heads", c_int),
        ("num_layers", c_int),
        ("kernel_size", c_int),
        ("rel_attn_window_size", c_int),
        ("mean_only", c_int),
        ("use_prenet", c_int),
        ("c_in_channels", c_int),
        ("math_mode", c_int),
        ("encoder_type", c_int),
        ("num_conv_blocks", c_int),
        ("num_res_blocks", c_int),
        ("dilations", c_int * 32),
        ("layer_norm_type", c_int),
        ("has_input_length", c_int),
        ("input_length", c_int),
    ]


# TtsGlowEncoderCfg.encoder_type (include/tts_mi355x.h TTS_ENC_*)
ENCODER_TYPES = {"rel_pos_transformer": 0, "gated_conv": 1, "residual_conv_bn": 2, "time_depth_separable": 3}


class TtsAudioNormCfg(Structure):
    _fields_ = [
        ("signal_norm", c_int),
        ("symmetric_norm", c_int),
        ("clip_norm", c_int),
        ("max_norm", c_double),
        ("min_level_db", c_double),
        ("ref_level_db", c_double),
        ("d_mel_mean", c_void_p),
        ("d_mel_scale", c_void_p),
    ]


class TtsVitsFlowCfg(Structure):
    _fields_ = [
        ("channels", c_int),
        ("hidden_channels", c_int),
        ("kernel_size", c_int),
        ("dilation_rate", c_int),
        ("num_layers", c_int),
        ("num_flows", c_int),
        ("cond_channels", c_int),
        ("math_mode", c_int),
    ]


class TtsVitsPosteriorCfg(Structure):
    _fields_ = [
        ("in_channels", c_int),
        ("out_channels", c_int),
        ("hidden_channels", c_int),
        ("kernel_size", c_int),
        ("dilation_rate", c_int),
        ("num_layers", c_int),
        ("cond_channels", c_int),
        ("math_mode", c_int),
    ]


class TtsVitsTextEncoderCfg(Structure):
    _fields_ = [
        ("n_vocab", c_int),
        ("out_channels", c_int),
        ("hidden_channels", c_int),
        ("hidden_channels_ffn", c_int),
        ("num_heads", c_int),
        ("num_layers", c_int),
        ("kernel_size", c_int),
        ("language_emb_dim", c_int),
        ("math_mode", c_int),
    ]


class TtsVitsSdpCfg(Structure):
    _fields_ = [
        ("in_channels", c_int),
        ("hidden_channels", c_int),
        ("kernel_size", c_int),
        ("num_flows", c_int),
        ("cond_channels", c_int),
        ("language_emb_dim", c_int),
        ("math_mode", c_int),
    ]


class TtsVitsDpCfg(Structure):
    _fields_ = [
        ("in_channels", c_int),
        ("hidden_channels", c_int),
        ("kernel_size", c_int),
        ("cond_channels", c_int),
        ("language_emb_dim", c_int),
        ("math_mode", c_int),
    ]


class TtsLaunchRecord(Structure):
    _fields_ = [("name", c_char * 48), ("flops", c_double), ("bytes", c_double), ("ms", c_float)]


class TtsConv1dDesc(Structure):
    _fields_ = [
        ("B", c_int),
        ("Cin", c_int),
        ("Cout", c_int),
        ("Tin", c_int),
        ("K", c_int),
        ("dil", c_int),
        ("rep_pad", c_int),
        ("in_slope", c_float),
        ("out_slope", c_float),
        ("zmode", c_int),
        ("zdiv", c_float),
        ("math_mode", c_int),
    ]


# name -> (restype, argtypes); must list every function declared in include/tts_mi355x.h
SIGNATURES = {
    "tts_last_error": (c_char_p, []),
    "tts_abi_version": (c_int, []),
    "tts_build_target": (c_char_p, []),
    "tts_build_info": (c_char_p, []),
    "tts_hifigan_num_weights": (c_int, [POINTER(TtsHifiganCfg)]),
    "tts_hifigan_weight_numel": (c_int64, [POINTER(TtsHifiganCfg), c_int]),
    "tts_hifigan_create": (c_int, [POINTER(TtsHifiganCfg), POINTER(c_void_p), c_int, POINTER(c_void_p)]),
    "tts_hifigan_destroy": (c_int, [c_void_p]),
    "tts_hifigan_output_length": (c_int64, [c_void_p, c_int, c_int]),
    "tts_hifigan_workspace_bytes": (c_int64, [c_void_p, c_int, c_int, c_int]),
    "tts_hifigan_reserve": (c_int, [c_void_p, c_int, c_int, c_int]),
    "tts_hifigan_forward": (
        c_int,
        [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    ),
    "tts_hifigan_forward_profiled": (
        c_int,
        [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
         POINTER(TtsLaunchRecord), c_int, POINTER(c_int)],
    ),
    "tts_glow_decoder_num_weights": (c_int, [POINTER(TtsGlowDecoderCfg)]),
    "tts_glow_decoder_weight_numel": (c_int64, [POINTER(TtsGlowDecoderCfg), c_int]),
    "tts_glow_decoder_create": (
        c_int, [POINTER(TtsGlowDecoderCfg), POINTER(c_void_p), c_int, POINTER(c_void_p)]
    ),
    "tts_glow_decoder_destroy": (c_int, [c_void_p]),
    "tts_glow_decoder_forward": (
        c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]
    ),
    "tts_glow_decoder_forward_profiled": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
         POINTER(TtsLaunchRecord), c_int, POINTER(c_int)],
    ),
    "tts_glow_encoder_num_weights": (c_int, [POINTER(TtsGlowEncoderCfg)]),
    "tts_glow_encoder_weight_numel": (c_int64, [POINTER(TtsGlowEncoderCfg), c_int]),
    "tts_glow_encoder_create": (
        c_int, [POINTER(TtsGlowEncoderCfg), POINTER(c_void_p), c_int, POINTER(c_void_p)]
    ),
    "tts_glow_encoder_destroy": (c_int, [c_void_p]),
    "tts_glow_encoder_forward": (
        c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    ),
    "tts_glow_encoder_forward_profiled": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         POINTER(TtsLaunchRecord), c_int, POINTER(c_int)],
    ),
    "tts_glow_durations": (
        c_int, [c_void_p, c_void_p, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p]
    ),
    "tts_glow_expand": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int, c_int, c_int, c_int,
         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "tts_mel_handoff": (
        c_int,
        [c_void_p, c_int, c_int, c_int, c_int, POINTER(TtsAudioNormCfg), POINTER(TtsAudioNormCfg), c_int, c_float,
         c_void_p, c_void_p],
    ),
    "tts_wav_to_int16": (c_int, [c_void_p, c_int, c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "tts_vits_flow_num_weights": (c_int, [POINTER(TtsVitsFlowCfg)]),
    "tts_vits_flow_weight_numel": (c_int64, [POINTER(TtsVitsFlowCfg), c_int]),
    "tts_vits_flow_create": (c_int, [POINTER(TtsVitsFlowCfg), POINTER(c_void_p), c_int, POINTER(c_void_p)]),
    "tts_vits_flow_destroy": (c_int, [c_void_p]),
    "tts_vits_flow_forward": (
        c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]
    ),
    "tts_vits_flow_forward_profiled": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
         POINTER(TtsLaunchRecord), c_int, POINTER(c_int)],
    ),
    "tts_vits_posterior_num_weights": (c_int, [POINTER(TtsVitsPosteriorCfg)]),
    "tts_vits_posterior_weight_numel": (c_int64, [POINTER(TtsVitsPosteriorCfg), c_int]),
    "tts_vits_posterior_create": (c_int, [POINTER(TtsVitsPosteriorCfg), POINTER(c_void_p), c_int, POINTER(c_void_p)]),
    "tts_vits_posterior_destroy": (c_int, [c_void_p]),
    "tts_vits_posterior_forward": (
        c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                c_void_p]
    ),
    "tts_vits_posterior_forward_profiled": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
         c_void_p, POINTER(TtsLaunchRecord), c_int, POINTER(c_int)],
    ),
    "tts_vits_text_encoder_num_weights": (c_int, [POINTER(TtsVitsTextEncoderCfg)]),
    "tts_vits_text_encoder_weight_numel": (c_int64, [POINTER(TtsVitsTextEncoderCfg), c_int]),
    "tts_vits_text_encoder_create": (
        c_int, [POINTER(TtsVitsTextEncoderCfg), POINTER(c_void_p), c_int, POINTER(c_void_p)]
    ),
    "tts_vits_text_encoder_destroy": (c_int, [c_void_p]),
    "tts_vits_text_encoder_forward": (
        c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                c_void_p]
    ),
    "tts_vits_text_encoder_forward_profiled": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         POINTER(TtsLaunchRecord), c_int, POINTER(c_int)],
    ),
    "tts_vits_sdp_num_weights": (c_int, [POINTER(TtsVitsSdpCfg)]),
    "tts_vits_sdp_weight_numel": (c_int64, [POINTER(TtsVitsSdpCfg), c_int]),
    "tts_vits_sdp_create": (c_int, [POINTER(TtsVitsSdpCfg), POINTER(c_void_p), c_int, POINTER(c_void_p)]),
    "tts_vits_sdp_destroy": (c_int, [c_void_p]),
    "tts_vits_sdp_reverse": (
        c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int, c_int, c_void_p,
                c_void_p]
    ),
    "tts_vits_sdp_reverse_profiled": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int, c_int, c_void_p, c_void_p,
         POINTER(TtsLaunchRecord), c_int, POINTER(c_int)],
    ),
    "tts_vits_dp_num_weights": (c_int, [POINTER(TtsVitsDpCfg)]),
    "tts_vits_dp_weight_numel": (c_int64, [POINTER(TtsVitsDpCfg), c_int]),
    "tts_vits_dp_create": (c_int, [POINTER(TtsVitsDpCfg), POINTER(c_void_p), c_int, POINTER(c_void_p)]),
    "tts_vits_dp_destroy": (c_int, [c_void_p]),
    "tts_vits_dp_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "tts_vits_dp_forward_profiled": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
         POINTER(TtsLaunchRecord), c_int, POINTER(c_int)],
    ),
    "tts_vits_durations": (c_int, [c_void_p, c_void_p, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p]),
    "tts_vits_expand": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int, c_int, c_int, c_int,
         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "tts_vits_durations_given": (c_int, [c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "tts_vits_mask_slice": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "tts_vits_upsample_z": (
        c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_double, c_int, c_void_p, c_void_p, c_void_p]
    ),
    "tts_embedding_rows": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int64, c_int, c_void_p, c_void_p]),
    "tts_l2_normalize_rows": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "tts_op_conv1d": (
        c_int, [POINTER(TtsConv1dDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    ),
    "tts_op_conv1d_bench": (
        c_int,
        [POINTER(TtsConv1dDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
         POINTER(c_float), c_void_p],
    ),
    "tts_op_conv1d_num_tiles": (c_int, [c_int]),
    "tts_op_conv_transpose1d": (
        c_int,
        [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_int, c_void_p, c_void_p],
    ),
    "tts_op_conv_post": (
        c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_void_p]
    ),
}

_lib = None

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # tts-3_amd/


def source_hash(pkg_dir: str = _PKG_DIR) -> str:
    """The src= stamp tts_build_info() should carry for the sources in ``pkg_dir`` (the Makefile's
    HASHED list: SRCS, csrc/*.hpp, ../include/tts_mi355x.h and the Makefile, sorted by path)."""
    import glob
    import hashlib
    import re

    mk = open(os.path.join(pkg_dir, "Makefile")).read()
    srcs = re.search(r"^SRCS := (.*)$", mk, re.M).group(1).split()
    hdrs = [os.path.relpath(p, pkg_dir) for p in glob.glob(os.path.join(pkg_dir, "csrc", "*.hpp"))]
    files = sorted(set(srcs + hdrs + ["../include/tts_mi355x.h", "Makefile"]))
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(pkg_dir, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_info_fields(handle) -> dict:
    """``tts_build_info()`` parsed: target=, src= (source hash) and defs= (build-option macros)."""
    handle.tts_build_info.restype = c_char_p
    handle.tts_build_info.argtypes = []
    return dict(kv.split("=", 1) for kv in handle.tts_build_info().decode().split())


def build_info() -> dict:
    """Provenance of the loaded library: its stamped source hash, the build-option macros it was
    compiled with, and the file's own sha256."""
    import hashlib

    fields = build_info_fields(lib())
    with open(LIB_PATH, "rb") as fh:
        fields["lib_sha256"] = hashlib.sha256(fh.read()).hexdigest()[:16]
    fields["lib_path"] = LIB_PATH
    return fields


class NativeError(RuntimeError):
    """A C-ABI call returned a non-zero status."""

    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed (status {code}): {msg}")
        self.code = code


def lib() -> ctypes.CDLL:
    """Open the library (once).  Raises if it is missing: there is no fallback path."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{_LIB_NAME} not found at {LIB_PATH}: build it with `make -C tts-3_amd` "
            "(or __graft_entry__.build()); the MI355X path has no CPU fallback"
        )
    handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    handle.tts_abi_version.restype = c_int
    handle.tts_abi_version.argtypes = []
    abi = handle.tts_abi_version()
    if abi != ABI_VERSION:
        # argument lists differ between revisions: binding them to another revision passes
        # pointers where the library expects sizes (garbage or a GPU fault), so refuse to load
        raise RuntimeError(f"{LIB_PATH} implements C-ABI {abi}, these bindings need {ABI_VERSION}: "
                           "rebuild it with `make -C tts-3_amd`")
    for name, (res, args) in SIGNATURES.items():
        try:
            fn = getattr(handle, name)
        except AttributeError:  # a call to it raises the same error (tests check every symbol is exported)
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = handle
    stamp = build_info_fields(handle).get("src")
    if stamp is not None and os.path.exists(os.path.join(_PKG_DIR, "Makefile")):
        try:
            want = source_hash()
        except OSError:
            want = None
        if want is not None and stamp != want:
            import warnings

            warnings.warn(f"{LIB_PATH} was built from other sources (src={stamp}, tree={want}); "
                          "rebuild it with `make -C tts-3_amd`", RuntimeWarning, stacklevel=2)
    return _lib


def check(fn_name: str, status: int) -> None:
    if status != TTS_OK:
        msg = lib().tts_last_error().decode(errors="replace")
        raise NativeError(fn_name, status, msg)


def call(fn_name: str, *args) -> int:
    """Call a status-returning entry point and raise on failure."""
    st = getattr(lib(), fn_name)(*args)
    check(fn_name, st)
    return st


def ptr(t) -> c_void_p:
    """Raw device/host pointer of a tensor or numpy array (None -> NULL)."""
    if t is None:
        return c_void_p(0)
    if hasattr(t, "data_ptr"):
        return c_void_p(t.data_ptr())
    return c_void_p(t.ctypes.data)


def stream_ptr(device: torch.device) -> c_void_p:
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device_tensor(t: torch.Tensor, what: str) -> None:
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise RuntimeError(
            f"{what} must be a ROCm device tensor: the tts_amd path runs only on MI355X (no CPU fallback)"
        )
