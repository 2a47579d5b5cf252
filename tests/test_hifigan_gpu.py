"""HiFiGAN parity on MI355X through the C-ABI (libtts_mi355x.so).

* single kernels (tts_op_*) vs torch.nn.functional fp64 on the CPU, over the shapes of
  HiFiGAN v1/v3, ragged channel counts, edge lengths, every epilogue mode;
* the whole generator vs the reference's own outputs (tests/golden, fp64 anchor);
* at the benchmark size (B=32 x 1024 frames) the size-independent properties: finite,
  |y| <= 1, batch-invariance (each utterance bit-identical to running it alone),
  run-to-run determinism, and four utterances vs the fp64 CPU oracle.

fp32-faithful gates (tests/_util.py): rel-RMS <= 5e-6 and max|d| <= 1e-5 on waveforms (1e-4 on
single-op outputs) against the fp64 reference; bf16: SURVEY.md §8c's 3e-2.
"""
import ctypes
import functools

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from _util import assert_close_fp32, goldens, hifigan_ctor, log_error, max_abs, rel_rms, tol
from oracle import hifigan_ref
from tts_amd import _native as N
from tts_amd import synthetic
from tts_amd.config import HIFIGAN_V1
from tts_amd.vocoder import HifiganGenerator

pytestmark = pytest.mark.gpu
V1 = dict(in_channels=80, out_channels=1, **HIFIGAN_V1)


def _rng(seed):
    return torch.Generator().manual_seed(seed)


# ----------------------------------------------------------------------------- conv1d
MODES = ["fp32", "fp32x6", "f16x3", "bf16"]  # TTS_MATH_* (f16x3: HiFiGAN executor and the conv op only)

CONV_CASES = [
    # B, Cin, Cout, T, K, dil, rep, in_slope, out_slope, res, zmode
    (2, 80, 512, 37, 7, 1, 5, 1.0, 1.0, False, 0),     # conv_pre with replicate padding
    (2, 256, 256, 300, 11, 5, 0, 0.1, 0.1, False, 0),  # MRF convs1, stage 1
    (1, 256, 256, 129, 3, 1, 0, 1.0, 1.0, True, 0),    # convs2 + residual
    (1, 128, 128, 1000, 7, 3, 0, 0.1, 0.1, False, 0),
    (2, 64, 64, 777, 3, 1, 0, 1.0, 1.0, True, 1),      # z init
    (1, 64, 64, 600, 11, 1, 0, 1.0, 1.0, True, 2),     # z accumulate
    (1, 32, 32, 1100, 11, 5, 0, 1.0, 1.0, True, 3),    # z final (/3)
    (3, 33, 17, 50, 5, 2, 0, 0.1, 1.0, False, 0),      # ragged channels
    (1, 24, 40, 97, 7, 12, 0, 0.1, 1.0, True, 0),      # HiFiGAN-v3 dilation 12 (wide halo)
    (2, 192, 384, 61, 5, 1, 0, 1.0, 1.0, False, 0),    # Glow WN in_layer
    (1, 80, 192, 33, 1, 1, 0, 1.0, 1.0, False, 0),     # 1x1
    (1, 16, 16, 1, 11, 5, 0, 0.1, 0.1, False, 0),      # single frame
    (1, 80, 512, 1, 7, 1, 5, 1.0, 1.0, False, 0),      # single mel frame + replicate pad
]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("case", CONV_CASES, ids=[f"c{i}" for i in range(len(CONV_CASES))])
def test_op_conv1d(cuda_device, case, mode):
    B, Cin, Cout, T, K, dil, rep, s_in, s_out, use_res, zmode = case
    g = _rng(hash(case) & 0xFFFF)
    x = torch.randn(B, Cin, T, generator=g)
    w = torch.randn(Cout, Cin, K, generator=g) / np.sqrt(Cin * K)
    b = torch.randn(Cout, generator=g) * 0.1
    To = T + 2 * rep
    res = torch.randn(B, Cout, To, generator=g) if use_res else None
    z0 = torch.randn(B, Cout, To, generator=g)
    # fp64 reference
    xp = F.pad(x.double(), (rep, rep), "replicate") if rep else x.double()
    v = F.conv1d(F.leaky_relu(xp, s_in), w.double(), b.double(), dilation=dil, padding=dil * (K - 1) // 2)
    v = F.leaky_relu(v, s_out)
    if res is not None:
        v = v + res.double()
    ref = {0: v, 1: v, 2: z0.double() + v, 3: (z0.double() + v) / 3.0}[zmode]
    d = N.TtsConv1dDesc(B, Cin, Cout, T, K, dil, rep, s_in, s_out, zmode, 3.0, N.MATH_MODES[mode])
    xd = x.to(cuda_device)
    resd = res.to(cuda_device) if res is not None else None
    y = torch.full((B, Cout, To), float("nan"), device=cuda_device)
    z = z0.to(cuda_device)
    wn, bn = w.numpy().copy(), b.numpy().copy()
    N.call("tts_op_conv1d", ctypes.byref(d), N.ptr(xd), N.ptr(wn), N.ptr(bn), N.ptr(resd), N.ptr(y), N.ptr(z),
           N.stream_ptr(cuda_device))
    out = y if zmode == 0 else z
    assert_close_fp32(out.cpu(), ref, f"conv1d {case}", **tol(mode, op=True))


WINO_TILE = 21  # kSplitWinoTile (common.hpp): Winograd F(4,4), f16x3
WINO_CASES = [
    # B, Cin, Cout, T, K, dil, in_slope, out_slope, res, zmode
    (2, 256, 256, 300, 11, 5, 0.1, 0.1, False, 0),   # stage-1 convs1
    (1, 128, 128, 1000, 7, 3, 0.1, 0.1, False, 0),   # stage-2 convs1
    (1, 128, 128, 777, 11, 1, 1.0, 1.0, True, 2),    # convs2 + residual, z accumulate
    (2, 256, 256, 129, 7, 1, 1.0, 1.0, True, 3),     # z final (/3)
    (1, 128, 128, 1, 11, 5, 0.1, 0.1, False, 0),     # single frame
    (2, 128, 128, 9, 7, 5, 0.1, 0.1, True, 1),       # shorter than the halo
    (3, 144, 256, 263, 11, 3, 0.1, 1.0, True, 0),    # Cin != Cout, 9 channel chunks
    (1, 128, 384, 1283, 11, 1, 0.1, 0.1, False, 0),  # 3 row blocks, ragged last workgroup
    # T % 4 == 0: the 8-wave form (LDS-DMA input windows)
    (2, 128, 128, 1028, 11, 5, 0.1, 0.1, False, 0),
    (1, 128, 128, 2048, 11, 3, 1.0, 1.0, True, 2),
    (2, 256, 256, 516, 7, 1, 1.0, 1.0, True, 3),
    (1, 128, 128, 8, 7, 5, 0.1, 0.1, True, 1),      # shorter than the halo
    (3, 144, 128, 252, 11, 1, 0.1, 0.1, False, 0),  # 9 channel chunks (odd)
    (1, 16, 128, 64, 11, 1, 0.1, 0.1, False, 0),    # one channel chunk
    (2, 32, 256, 300, 7, 3, 0.1, 1.0, True, 0),     # two channel chunks, 2 row blocks
    # kernel 3 (one chunk of 4 taps, the 4th zero)
    (2, 128, 128, 1024, 3, 5, 0.1, 0.1, False, 0),
    (1, 256, 256, 516, 3, 1, 1.0, 1.0, True, 3),
    (1, 128, 128, 777, 3, 3, 0.1, 0.1, True, 2),    # 4-wave form (T % 4 != 0)
    (1, 128, 128, 4, 3, 1, 1.0, 1.0, True, 1),
]


@pytest.mark.parametrize("case", WINO_CASES, ids=[f"w{i}" for i in range(len(WINO_CASES))])
def test_op_conv1d_winograd(cuda_device, case):
    """The Winograd F(4,4) conv (wino_kernel.hpp) against fp64 at the fp32 gates, every epilogue
    mode, every dilation, lengths around its 256 / 252 / 240-sample workgroups."""
    B, Cin, Cout, T, K, dil, s_in, s_out, use_res, zmode = case
    g = _rng(hash(case) & 0xFFFF)
    x = torch.randn(B, Cin, T, generator=g) * 2
    w = torch.randn(Cout, Cin, K, generator=g) / np.sqrt(Cin * K)
    b = torch.randn(Cout, generator=g) * 0.1
    res = torch.randn(B, Cout, T, generator=g) if use_res else None
    z0 = torch.randn(B, Cout, T, generator=g)
    v = F.conv1d(F.leaky_relu(x.double(), s_in), w.double(), b.double(), dilation=dil, padding=dil * (K - 1) // 2)
    v = F.leaky_relu(v, s_out)
    if res is not None:
        v = v + res.double()
    ref = {0: v, 1: v, 2: z0.double() + v, 3: (z0.double() + v) / 3.0}[zmode]
    d = N.TtsConv1dDesc(B, Cin, Cout, T, K, dil, 0, s_in, s_out, zmode, 3.0, N.MATH_MODES["f16x3"])
    y = torch.full((B, Cout, T), float("nan"), device=cuda_device)
    z = z0.to(cuda_device)
    resd = res.to(cuda_device) if res is not None else None
    wn, bn = w.numpy().copy(), b.numpy().copy()
    N.call("tts_op_conv1d_bench", ctypes.byref(d), N.ptr(x.to(cuda_device)), N.ptr(wn), N.ptr(bn), N.ptr(resd),
           N.ptr(y), N.ptr(z), WINO_TILE, 0, None, N.stream_ptr(cuda_device))
    out = y if zmode == 0 else z
    ma, rr = assert_close_fp32(out.cpu(), ref, f"winograd conv1d {case}")
    assert rr < 3e-6, rr  # ~3x the direct f16x3 conv's error, far inside the gate


def test_op_conv1d_winograd_rejects_unsupported(cuda_device):
    x = torch.zeros(1, 120, 16, device=cuda_device)
    y = torch.zeros(1, 128, 16, device=cuda_device)
    w, b = np.zeros((128, 120, 11), np.float32), np.zeros(128, np.float32)
    d = N.TtsConv1dDesc(1, 120, 128, 16, 11, 1, 0, 1.0, 1.0, 0, 1.0, N.MATH_MODES["f16x3"])  # Cin % 16 != 0
    with pytest.raises(N.NativeError):
        N.call("tts_op_conv1d_bench", ctypes.byref(d), N.ptr(x), N.ptr(w), N.ptr(b), None, N.ptr(y), None,
               WINO_TILE, 0, None, N.stream_ptr(cuda_device))


# ----------------------------------------------------------------------------- conv_transpose1d
CONVT_CASES = [
    # B, Cin, Cout, T, U
    (2, 512, 256, 37, 8),
    (1, 256, 128, 100, 8),
    (2, 128, 64, 129, 2),
    (1, 64, 32, 300, 2),
    (1, 256, 128, 1, 8),
    (2, 64, 32, 50, 4),
    (1, 48, 24, 17, 2),   # ragged
    (3, 40, 20, 9, 8),    # ragged
    (2, 128, 64, 70, 8),  # window-resident x8 form at 128 input channels (2 passes of 256 rows)
    (3, 256, 128, 129, 8),  # window-resident x8 form: frames across two 64-frame tiles + the pad frame
    (2, 512, 256, 130, 8),  # x8, 512 channels: 3 windows, each window's 8 passes over 4 workgroups
    (1, 256, 128, 260, 8),  # x8, 256 channels: windows across a 128-frame boundary too
    (2, 64, 32, 513, 2),    # x2 window form, 64 channels: 514 frames over 128-frame windows
]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("case", CONVT_CASES, ids=[f"t{i}" for i in range(len(CONVT_CASES))])
def test_op_conv_transpose1d(cuda_device, case, mode):
    B, Cin, Cout, T, U = case
    K = 2 * U
    g = _rng(1000 + T)
    x = torch.randn(B, Cin, T, generator=g)
    w = torch.randn(Cin, Cout, K, generator=g) / np.sqrt(Cin * 2)
    b = torch.randn(Cout, generator=g) * 0.1
    ref = F.conv_transpose1d(F.leaky_relu(x.double(), 0.1), w.double(), b.double(), stride=U, padding=(K - U) // 2)
    y = torch.full((B, Cout, U * T), float("nan"), device=cuda_device)
    wn, bn = w.numpy().copy(), b.numpy().copy()
    N.call("tts_op_conv_transpose1d", N.ptr(x.to(cuda_device)), B, Cin, T, N.ptr(wn), N.ptr(bn), Cout, K, U, 0.1,
           N.MATH_MODES[mode], N.ptr(y), N.stream_ptr(cuda_device))
    assert_close_fp32(y.cpu(), ref, f"convT {case}", **tol(mode, op=True))


@pytest.mark.parametrize("B,Cin,T", [(2, 32, 1000), (1, 32, 1), (3, 8, 513), (2, 64, 3001), (1, 20, 1024), (2, 32, 2052), (1, 13, 4)])
def test_op_conv_post(cuda_device, B, Cin, T):
    g = _rng(T)
    z = torch.randn(B, Cin, T, generator=g)
    w = torch.randn(1, Cin, 7, generator=g) / np.sqrt(Cin * 7)
    b = torch.randn(1, generator=g) * 0.1
    ref = torch.tanh(F.conv1d(F.leaky_relu(z.double(), 0.01), w.double(), b.double(), padding=3))
    y = torch.full((B, 1, T), float("nan"), device=cuda_device)
    wn, bn = w.numpy().copy(), b.numpy().copy()
    N.call("tts_op_conv_post", N.ptr(z.to(cuda_device)), B, Cin, T, N.ptr(wn), N.ptr(bn), 0.01, N.ptr(y),
           N.stream_ptr(cuda_device))
    assert_close_fp32(y.cpu(), ref, "conv_post")


# ----------------------------------------------------------------------------- whole generator
HIFI = goldens("hifigan")


def build(cfg, seed, device, math_mode="fp32"):
    g = HifiganGenerator(**hifigan_ctor(cfg), math_mode=math_mode)
    g.load_state_dict(synthetic.hifigan_state_dict(**cfg, seed=seed, weight_norm=True))
    g.eval()
    if cfg.get("conv_pre_weight_norm", True):
        g.remove_weight_norm()
    return g.to(device)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("name,meta,arr", HIFI, ids=[h[0] for h in HIFI])
def test_generator_vs_reference_goldens(cuda_device, name, meta, arr, mode):
    cfg = meta["config"]
    g = build(cfg, meta["seed"], cuda_device, mode)
    mel = torch.from_numpy(arr["mel"]).to(cuda_device)
    gv = torch.from_numpy(arr["g"]).to(cuda_device) if "g" in arr else None
    out = g.inference(mel, gv) if gv is not None else g.inference(mel)
    assert_close_fp32(out.cpu(), arr["out_ref_fp64"], f"{name} inference", **tol(mode))
    # and as close to the reference fp32 CPU forward as that forward is to fp64
    assert max_abs(out.cpu().numpy(), arr["out_ref_fp32"]) < tol(mode)["max_abs_tol"]
    if "fwd_ref_fp64" in arr:
        fwd = g(mel, gv) if gv is not None else g(mel)
        assert_close_fp32(fwd.cpu(), arr["fwd_ref_fp64"], f"{name} forward", **tol(mode))


def test_generator_stage_parity(cuda_device):
    """conv_pre / ups outputs via the op entry points on the reference's own intermediates."""
    name, meta, arr = [h for h in HIFI if "stage_conv_pre" in h[2]][0]
    cfg = meta["config"]
    sd = hifigan_ref.fold_weight_norm(synthetic.hifigan_state_dict(**cfg, seed=meta["seed"]), torch.float32)
    mel = torch.from_numpy(arr["stage_mel"])
    B, C, T = mel.shape
    P = meta["pad"]
    d = N.TtsConv1dDesc(B, C, 512, T, 7, 1, P, 1.0, 1.0, 0, 1.0)
    y = torch.empty(B, 512, T + 2 * P, device=cuda_device)
    w, b = sd["conv_pre.weight"].float().numpy().copy(), sd["conv_pre.bias"].float().numpy().copy()
    N.call("tts_op_conv1d", ctypes.byref(d), N.ptr(mel.to(cuda_device)), N.ptr(w), N.ptr(b), None, N.ptr(y), None,
           N.stream_ptr(cuda_device))
    assert_close_fp32(y.cpu(), arr["stage_conv_pre"], "conv_pre stage", max_abs_tol=1e-5)


@pytest.mark.parametrize("mode", ["fp32", "fp32x6", "f16x3"])
def test_generator_edge_lengths_vs_oracle(cuda_device, mode):
    """Short and ragged lengths through every kernel family: the fused resblock kernels of the split
    modes (pair tiles of 256 - (K-1) / 192 - (K-1) columns at C=32 / C=64, whole-block tiles of 232
    columns at C=32 and 104 at C=64 / C=128), the Winograd convs and the streaming conv_post."""
    sd = synthetic.hifigan_state_dict(seed=31, weight_norm=False)
    g = HifiganGenerator(**V1, math_mode=mode)
    g.remove_weight_norm()
    g.load_state_dict(sd)
    g = g.to(cuda_device)
    for B, T, pad in [(1, 1, 0), (2, 3, 0), (1, 2, 5), (3, 67, 5), (2, 101, 0)]:
        mel = synthetic.mel(B, T, seed=T)
        out = g._run(mel.to(cuda_device), pad, None)
        ref = hifigan_ref.hifigan_forward(sd, mel, pad=pad, dtype=torch.float64, **V1)
        assert_close_fp32(out.cpu(), ref, f"B={B} T={T} pad={pad}", **tol(mode))


def test_input_validation(cuda_device):
    g = HifiganGenerator(**V1).to(cuda_device)
    with pytest.raises(ValueError):
        g.inference(torch.zeros(1, 81, 4, device=cuda_device))
    with pytest.raises(ValueError):
        g.inference(torch.zeros(80, 4, device=cuda_device))


def test_profiled_forward_records(cuda_device):
    g = build(dict(V1, inference_padding=5), 1234, cuda_device)
    mel = synthetic.mel(2, 16).to(cuda_device)
    out, rows = g.profile(mel)
    assert len(rows) == 1 + 4 + 4 * 3 * 6 + 1  # conv_pre, ups, 72 MRF convs, conv_post
    assert all(r["ms"] > 0 for r in rows)
    flops = sum(r["flops"] for r in rows)
    # 614.1 MFLOP per padded frame, minus the conv zero-padding waste at T'=26
    assert 0.9 * 614.1e6 * 2 * 26 < flops <= 614.2e6 * 2 * 26
    assert torch.equal(out, g.inference(mel))


@pytest.mark.slow
@pytest.mark.parametrize("mode", MODES)
def test_benchmark_size_properties(cuda_device, mode):
    """Config 2 of BASELINE.json: B=32 x 1024 frames, HiFiGAN-v1, fp32."""
    sd = synthetic.hifigan_state_dict(seed=1234, weight_norm=False)
    g = HifiganGenerator(**V1, math_mode=mode)
    g.remove_weight_norm()
    g.load_state_dict(sd)
    g = g.to(cuda_device)
    mel = synthetic.mel(32, 1024, seed=0).to(cuda_device)
    out = g.inference(mel)
    assert out.shape == (32, 1, 256 * 1034)
    assert torch.isfinite(out).all() and out.abs().max() <= 1.0
    assert out.std() > 0.05  # not collapsed
    again = g.inference(mel)
    assert torch.equal(out, again), "run-to-run determinism"
    for i in (0, 17, 31):
        single = g.inference(mel[i : i + 1])
        assert torch.equal(single[0], out[i]), f"batch invariance, item {i}"
    # f16x3 takes a power-of-two scale per utterance and plane, so each row's arithmetic differs:
    # four rows (first, two inner, last) against the fp64 oracle, computed once for all modes
    for i in BENCH_ORACLE_ROWS:
        assert_close_fp32(out[i : i + 1].cpu(), _bench_row_oracle(i), f"B=32 item {i} vs fp64 oracle", **tol(mode))


BENCH_ORACLE_ROWS = (0, 9, 17, 31)


@functools.lru_cache(maxsize=None)
def _config1_case():
    sd = synthetic.hifigan_state_dict(seed=1234, weight_norm=False)
    mel = synthetic.mel(1, 256, seed=0)
    return sd, mel, hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **V1)


@pytest.mark.parametrize("mode", MODES)
def test_config1_single_mel_vs_oracle(cuda_device, mode):
    """BASELINE.json configs[0]: HiFiGAN-v1 on one 80 x 256 mel through the drop-in
    ``HifiganGenerator.inference`` (hifigan_generator.py:267-282, replicate pad 5), here on the HIP
    path in every math mode against the fp64 oracle.  (The reference runs this config on the CPU;
    the product has no CPU path by design, so the CPU side of config 1 is the oracle itself.)"""
    sd, mel, ref = _config1_case()
    g = HifiganGenerator(**V1, math_mode=mode)
    g.remove_weight_norm()
    g.load_state_dict(sd)
    g = g.to(cuda_device)
    out = g.inference(mel.to(cuda_device))
    assert out.shape == (1, 1, 256 * 266)
    assert torch.isfinite(out).all() and out.abs().max() <= 1.0
    assert_close_fp32(out.cpu(), ref, f"config 1 [1,80,256] ({mode})", **tol(mode))


@functools.lru_cache(maxsize=None)
def _bench_row_oracle(i):
    sd = synthetic.hifigan_state_dict(seed=1234, weight_norm=False)
    mel = synthetic.mel(32, 1024, seed=0)[i : i + 1]
    return hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **V1)


def test_split_modes_accuracy_not_worse_than_fp32(cuda_device, monkeypatch):
    """The bf16x6 and scaled fp16 hi/lo splits are fp32-faithful: their error vs the fp64
    reference matches exact-fp32 MFMA (and the reference's own fp32 CPU forward).  The Winograd
    F(4,4) form of the >= 128-channel MRF convs (f16x3 default) stays within 4x of it."""
    name, meta, arr = [h for h in HIFI if h[0] == "hifigan_v1_b2_t32"][0]
    errs = {}
    for mode, wino in (("fp32", "0"), ("fp32x6", "0"), ("f16x3", "0"), ("f16x3_wino", "1")):
        monkeypatch.setenv("TTS_MI355X_WINO", wino)
        g = build(meta["config"], meta["seed"], cuda_device, mode.split("_")[0])
        out = g.inference(torch.from_numpy(arr["mel"]).to(cuda_device)).cpu().numpy()
        errs[mode] = (max_abs(out, arr["out_ref_fp64"]), rel_rms(out, arr["out_ref_fp64"]))
    ref32 = (max_abs(arr["out_ref_fp32"], arr["out_ref_fp64"]), rel_rms(arr["out_ref_fp32"], arr["out_ref_fp64"]))
    print("max|d|, rel-RMS vs fp64:", errs, "reference fp32 CPU:", ref32)
    for mode in ("fp32x6", "f16x3"):
        assert errs[mode][1] <= 2.0 * max(errs["fp32"][1], ref32[1]), mode
        assert errs[mode][0] <= 2.0 * max(errs["fp32"][0], ref32[0]), mode
    assert errs["f16x3_wino"][1] <= 4.0 * max(errs["fp32"][1], ref32[1])
    assert errs["f16x3_wino"][0] <= 4.0 * max(errs["fp32"][0], ref32[0])


def _dynamic_range_mel(T=240, seed=21):
    """One utterance with a realistic log-mel dynamic range: a stretch at the log floor
    (ln(1e-5) = -11.5, what AudioProcessor emits for silence), loud speech-like frames, a
    near-silent stretch just above the floor, and isolated outlier bins."""
    g = _rng(seed)
    mel = torch.empty(1, 80, T)
    mel[:, :, 0:60] = -11.5 + 0.01 * torch.randn(1, 80, 60, generator=g)            # floor
    mel[:, :, 60:120] = 1.0 + 2.0 * torch.randn(1, 80, 60, generator=g)             # loud
    mel[:, :, 120:180] = -9.0 + 0.3 * torch.randn(1, 80, 60, generator=g)           # near silent
    mel[:, :, 180:T] = -4.0 + 1.5 * torch.randn(1, 80, T - 180, generator=g)        # speech
    mel[0, 7, 70], mel[0, 40, 200], mel[0, 63, 150] = 9.0, -16.0, 6.0              # outliers
    return mel


@pytest.mark.parametrize("wino", ["0", "1"])
def test_f16x3_realistic_dynamic_range(cuda_device, monkeypatch, wino):
    """f16x3 picks one power-of-two scale per utterance and plane from its max-abs: a quiet
    stretch next to loud frames keeps 22 bits relative to the loud max only.  Per segment of
    the output (floor / loud / near-silent / speech, 256 samples per frame), the f16x3 error
    against fp64 must stay within 2x of the exact-fp32 MFMA mode's (and the Winograd F(4,4)
    default within 2x as well)."""
    sd = synthetic.hifigan_state_dict(seed=1234, weight_norm=False)
    mel = _dynamic_range_mel()
    ref = hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **V1)[0, 0].numpy()
    monkeypatch.setenv("TTS_MI355X_WINO", wino)
    outs = {}
    for mode in ("fp32", "f16x3"):
        g = HifiganGenerator(**V1, math_mode=mode)
        g.remove_weight_norm()
        g.load_state_dict(sd)
        outs[mode] = g.to(cuda_device).inference(mel.to(cuda_device))[0, 0].cpu().numpy()
    segs = {"floor": (0, 60), "loud": (60, 120), "near_silent": (120, 180), "speech": (180, 240)}
    for seg, (f0, f1) in segs.items():
        sl = slice(256 * (f0 + 5), 256 * (f1 + 5))  # replicate pad 5 frames
        e = {m: (max_abs(o[sl], ref[sl]), rel_rms(o[sl], ref[sl])) for m, o in outs.items()}
        for m in e:
            log_error(f"dynamic range {seg} {m} wino={wino}", *e[m])
        # 5e-8 / 5e-7 floors: below them both modes sit at the fp32 rounding of tanh's output
        assert e["f16x3"][0] <= max(2.0 * e["fp32"][0], 5e-8), (seg, e)
        assert e["f16x3"][1] <= max(2.0 * e["fp32"][1], 5e-7), (seg, e)
        assert e["fp32"][1] <= 1e-5, (seg, e)


def test_winograd_generator_matches_direct(cuda_device, monkeypatch):
    """Whole HiFiGAN-v1 with and without the Winograd MRF convs (f16x3) at a multi-workgroup
    length: both within the fp32 gates of the fp64 oracle and of each other."""
    sd = synthetic.hifigan_state_dict(seed=77, weight_norm=False)
    mel = synthetic.mel(2, 61, seed=5)
    ref = hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **V1)
    outs = []
    for wino in ("1", "0"):  # Winograd for every supported MRF conv / none
        monkeypatch.setenv("TTS_MI355X_WINO", wino)
        g = HifiganGenerator(**V1, math_mode="f16x3")
        g.remove_weight_norm()
        g.load_state_dict(sd)
        g = g.to(cuda_device)
        outs.append(g.inference(mel.to(cuda_device)).cpu())
        assert_close_fp32(outs[-1], ref, f"wino={wino}")
    assert max_abs(outs[0].numpy(), outs[1].numpy()) < 2e-5


@pytest.mark.parametrize("mode", ["f16x3", "bf16"])
def test_whole_block_fusion_matches_unfused(cuda_device, monkeypatch, mode):
    """The kernel-3 ResBlock1 as one launch (resblock3_kernel: C=32, 64 and 128) against the
    per-iteration path (TTS_MI355X_RESBLOCK3=0) over several workgroups per utterance: both within
    the mode's gates of the fp64 oracle, and within the mode's own error of each other."""
    sd = synthetic.hifigan_state_dict(seed=41, weight_norm=False)
    mel = synthetic.mel(2, 45, seed=3)
    ref = hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **V1)
    outs = []
    for policy in ("all", "0"):
        monkeypatch.setenv("TTS_MI355X_RESBLOCK3", policy)
        g = HifiganGenerator(**V1, math_mode=mode)
        g.remove_weight_norm()
        g.load_state_dict(sd)
        g = g.to(cuda_device)
        outs.append(g.inference(mel.to(cuda_device)).cpu())
        assert_close_fp32(outs[-1], ref, f"{mode} resblock3={policy}", **tol(mode))
    assert max_abs(outs[0].numpy(), outs[1].numpy()) <= 2 * tol(mode).get("max_abs_tol", 1e-4)


# ResBlock2 topologies at channel widths the whole-block kernel takes (32 / 64 / 128):
# YourTTS's decoder form (VITS kernels 3, 7, 11 with ResBlock2 dilations (1, 3),
# recipes/vctk/yourtts/train_yourtts.py:134) and HiFiGAN-v3's kernels / dilations
RB2_YOURTTS = dict(in_channels=80, out_channels=1, resblock_type="2",
                   resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], resblock_kernel_sizes=[3, 7, 11],
                   upsample_kernel_sizes=[16, 16, 4, 4], upsample_initial_channel=256, upsample_factors=[8, 8, 2, 2],
                   inference_padding=5)
RB2_V3 = dict(in_channels=80, out_channels=1, resblock_type="2",
              resblock_dilation_sizes=[[1, 2], [2, 6], [3, 12]], resblock_kernel_sizes=[3, 5, 7],
              upsample_kernel_sizes=[16, 16, 8], upsample_initial_channel=256, upsample_factors=[8, 8, 4],
              inference_padding=5)


@pytest.mark.parametrize("mode", ["f16x3", "bf16", "fp32x6"])
@pytest.mark.parametrize("topo", ["yourtts", "v3"])
def test_resblock2_whole_block_matches_unfused(cuda_device, monkeypatch, mode, topo):
    """ResBlock2 (hifigan_generator.py:108-159) as one launch per block (resblock_block.hpp, kernels
    3 / 5 / 7 / 11) against the per-conv path (TTS_MI355X_RESBLOCK3=0), both within the mode's gates
    of the fp64 oracle over several workgroups per utterance, and the fused launches really used."""
    cfg = RB2_YOURTTS if topo == "yourtts" else RB2_V3
    sd = synthetic.hifigan_state_dict(seed=43, weight_norm=False, **cfg)
    mel = synthetic.mel(2, 23, seed=7)
    ref = hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **cfg)
    outs = []
    for policy in ("all", "0"):
        monkeypatch.setenv("TTS_MI355X_RESBLOCK3", policy)
        g = HifiganGenerator(**cfg, math_mode=mode)
        g.remove_weight_norm()
        g.load_state_dict(sd)
        g = g.to(cuda_device)
        outs.append(g.inference(mel.to(cuda_device)).cpu())
        names = [r["name"] for r in g.profile(mel.to(cuda_device))[1]]
        fused = [n for n in names if n.startswith("mrf_block2_")]
        if policy == "0":
            assert not fused
        else:
            # x6 has no 128-channel form; kernel 7 at dilation 12 (v3) stays per conv
            # f16x3 / x6 keep kernel 11 at 64 channels per conv (resblock2_preferred)
            expect = {"yourtts": {"f16x3": 6, "bf16": 7, "fp32x6": 5}, "v3": {"f16x3": 6, "bf16": 6, "fp32x6": 4}}
            assert len(fused) == expect[topo][mode], names
        assert_close_fp32(outs[-1], ref, f"{topo} {mode} whole-block={policy}", **tol(mode))
    assert max_abs(outs[0].numpy(), outs[1].numpy()) <= 2 * tol(mode).get("max_abs_tol", 1e-4)


@pytest.mark.parametrize("geo64", ["0", "1"])
def test_resblock2_long_ragged_vs_oracle(cuda_device, monkeypatch, geo64):
    """The ResBlock2 whole-block kernels at a length spanning many tiles per utterance (and a tile
    edge that is not a multiple of the column tile) against the fp64 oracle, both 64-channel
    geometries, every supported block fused (TTS_MI355X_RB2_ALL)."""
    monkeypatch.setenv("TTS_MI355X_RB2_GEO64", geo64)
    monkeypatch.setenv("TTS_MI355X_RB2_ALL", "1")
    cfg = RB2_YOURTTS
    sd = synthetic.hifigan_state_dict(seed=44, weight_norm=False, **cfg)
    mel = synthetic.mel(1, 61, seed=8)
    ref = hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **cfg)
    g = HifiganGenerator(**cfg, math_mode="f16x3")
    g.remove_weight_norm()
    g.load_state_dict(sd)
    g = g.to(cuda_device)
    out = g.inference(mel.to(cuda_device)).cpu()
    assert_close_fp32(out, ref, f"rb2 geo64={geo64}")
    names = [r["name"] for r in g.profile(mel.to(cuda_device))[1]]
    assert sum(n.startswith("mrf_block2_") and n.endswith("_c64") for n in names) == 3, names


def _padded_slice(mel, pad, a, b):
    """Frames [a, b) of the replicate-padded mel (hifigan_generator.py:281), clamped indices."""
    T = mel.shape[2]
    idx = (torch.arange(a, b) - pad).clamp(0, T - 1)
    return mel[:, :, idx]


@pytest.mark.parametrize("mode", ["fp32", "f16x3", "bf16"])
def test_windowed_forward_matches_plain(cuda_device, monkeypatch, mode):
    """Long-utterance path at an ordinary length: TTS_MI355X_WINDOW_FRAMES forces 37-frame payloads
    with the receptive-field halo on each side.  The payload samples of every window equal the
    plain forward's (fp32: bit for bit, the same sums in the same order; the split modes take a
    per-window power-of-two scale, so within the gates of the fp64 oracle)."""
    sd = synthetic.hifigan_state_dict(seed=91, weight_norm=False)
    mel = synthetic.mel(2, 150, seed=92)
    outs = {}
    for frames in ("0", "37"):
        monkeypatch.setenv("TTS_MI355X_WINDOW_FRAMES", frames)
        g = HifiganGenerator(**V1, math_mode=mode)
        g.remove_weight_norm()
        g.load_state_dict(sd)
        g = g.to(cuda_device)
        outs[frames] = g.inference(mel.to(cuda_device)).cpu()
        if frames == "37":
            names = [r["name"] for r in g.profile(mel.to(cuda_device))[1]]
            assert names.count("mel_window") == 5  # ceil(160 / 37) windows
    if mode == "fp32":
        assert torch.equal(outs["0"], outs["37"])
    ref = hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **V1)
    assert_close_fp32(outs["37"], ref, f"windowed ({mode})", **tol(mode))


@pytest.mark.parametrize("name", ["hifigan_small_rb2_b2_t16"])
def test_windowed_halo_other_topologies(cuda_device, monkeypatch, name):
    """The window halo (Hifigan::window_halo, the generator's receptive-field radius) for the
    other golden topology (v3-like: ResBlock2, x8 x8 x4 upsampling, dilation up to 12): 7-frame payloads
    must give the plain forward's output bit for bit in fp32, which only holds when every payload
    sample's whole receptive field lies inside its window."""
    hit = [h for h in HIFI if h[0] == name]
    if not hit:
        pytest.skip(f"golden {name} absent")
    _, meta, _ = hit[0]
    cfg = meta["config"]
    mel = synthetic.mel(2, 57, channels=cfg.get("in_channels", 80), seed=95)
    outs = {}
    for frames in ("0", "7"):
        monkeypatch.setenv("TTS_MI355X_WINDOW_FRAMES", frames)
        g = build(cfg, meta["seed"], cuda_device, "fp32")
        outs[frames] = g.inference(mel.to(cuda_device)).cpu()
    assert torch.equal(outs["0"], outs["7"])


@pytest.mark.slow
@pytest.mark.parametrize("mode", ["f16x3", "fp32"])
def test_long_utterance_beyond_plane_cap(cuda_device, mode):
    """An utterance whose 128-channel plane passes 2 GiB (T' = 65540 padded frames > 65535, the
    kernels' 32-bit range): windowed automatically.  Checked against the fp64 oracle on frame
    ranges at the start, across the window seam and at the end (each oracle run sees its
    range plus 32 frames of context: more than the 16-frame receptive field)."""
    sd = synthetic.hifigan_state_dict(seed=93, weight_norm=False)
    T, pad = 65530, 5
    mel = synthetic.mel(1, T, seed=94)
    g = HifiganGenerator(**V1, math_mode=mode)
    g.remove_weight_norm()
    g.load_state_dict(sd)
    g = g.to(cuda_device)
    y = g.inference(mel.to(cuda_device))
    L = T + 2 * pad
    assert y.shape == (1, 1, 256 * L)
    assert torch.isfinite(y).all() and y.abs().max() <= 1.0
    y = y.cpu()
    ctx = 32
    for a, b in [(0, 24), (65490, 65520), (L - 24, L)]:
        lo, hi = max(0, a - ctx), min(L, b + ctx)
        ref = hifigan_ref.hifigan_forward(sd, _padded_slice(mel, pad, lo, hi), pad=0, dtype=torch.float64, **V1)
        ref = ref[:, :, 256 * (a - lo):256 * (b - lo)]
        assert_close_fp32(y[:, :, 256 * a:256 * b], ref, f"long utterance frames [{a},{b}) ({mode})", **tol(mode))


@pytest.mark.parametrize("mode", ["f16x3", "fp32x6", "bf16"])
def test_conv_post_fusion_bitwise(cuda_device, monkeypatch, mode):
    """conv_post inside the last MRF pair launch (ResPairArgs::post_w: tiles overlapping by conv_post's
    3-sample halo, the final z kept in LDS) against the separate conv_post launch
    (TTS_MI355X_POST_FUSION=0): the same fp32 operations in the same order, so bitwise equal, at
    lengths that end inside, exactly on and just past a tile (240-sample stride at k11 / c32)."""
    sd = synthetic.hifigan_state_dict(seed=51, weight_norm=False)
    for B, T in [(2, 37), (1, 15), (3, 61)]:
        mel = synthetic.mel(B, T, seed=T).to(cuda_device)
        outs = {}
        for fused in ("1", "0"):
            monkeypatch.setenv("TTS_MI355X_POST_FUSION", fused)
            g = HifiganGenerator(**V1, math_mode=mode)
            g.remove_weight_norm()
            g.load_state_dict(sd)
            g = g.to(cuda_device)
            outs[fused] = g.inference(mel)
            names = [r["name"] for r in g.profile(mel)[1]]
            assert ("conv_post" in names) == (fused == "0"), names[-3:]
        assert torch.equal(outs["1"], outs["0"]), (B, T, (outs["1"] - outs["0"]).abs().max().item())


@pytest.mark.parametrize("mode", ["fp32", "f16x3"])
def test_concurrent_schedules_bitwise(cuda_device, monkeypatch, mode):
    """Execution lanes (Hifigan::forward): the MRF branches on 1, 2 or 3 streams
    (TTS_MI355X_MRF_STREAMS) and the batch split into sub-batches on concurrent lanes
    (TTS_MI355X_SUBBATCH, uneven at B = 5) compute every utterance with the same kernels in the
    same order, so the waveforms are bitwise those of the one-stream forward; and the result is
    still the reference generator's (fp64 oracle, the mode's gate)."""
    sd = synthetic.hifigan_state_dict(seed=71, weight_norm=False)
    mel = synthetic.mel(5, 40, seed=72)
    outs = {}
    for streams, sub in (("1", "1"), (None, None), ("3", "1"), ("2", "2"), ("3", "3"), ("3", "8")):
        for var, val in (("TTS_MI355X_MRF_STREAMS", streams), ("TTS_MI355X_SUBBATCH", sub)):
            if val is None:
                monkeypatch.delenv(var, raising=False)  # the defaults
            else:
                monkeypatch.setenv(var, val)
        g = HifiganGenerator(**V1, math_mode=mode)
        g.remove_weight_norm()
        g.load_state_dict(sd)
        g = g.to(cuda_device)
        outs[(streams, sub)] = g.inference(mel.to(cuda_device)).cpu()
        outs[(streams, sub, 2)] = g.inference(mel.to(cuda_device)).cpu()  # reused lanes / events
    base = outs[("1", "1")]
    for k, v in outs.items():
        assert torch.equal(v, base), f"schedule {k} differs from the one-stream forward ({mode})"
    ref = hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **V1)
    assert_close_fp32(base, ref, f"concurrent schedules ({mode})", **tol(mode))


@pytest.mark.parametrize("mode", ["f16x3", "bf16", "fp32x6"])
def test_whole_block_k7_k11_matches_pairs(cuda_device, monkeypatch, mode):
    """Kernel-7 / 11 ResBlock1 as one launch at 32 and 64 channels (resblock3_kernel with K = 7 / 11,
    TTS_MI355X_RB1_WHOLE_K) against the pair path, over several workgroups per utterance and a
    ragged tail: both within the mode's gates of the fp64 oracle and of each other; the profiled
    launch names show the whole-block launches."""
    sd = synthetic.hifigan_state_dict(seed=43, weight_norm=False)
    mel = synthetic.mel(2, 47, seed=5)
    ref = hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **V1)
    outs = []
    for wk in ("7,11", ""):
        monkeypatch.setenv("TTS_MI355X_RB1_WHOLE_K", wk)
        g = HifiganGenerator(**V1, math_mode=mode)
        g.remove_weight_norm()
        g.load_state_dict(sd)
        g = g.to(cuda_device)
        outs.append(g.inference(mel.to(cuda_device)).cpu())
        assert_close_fp32(outs[-1], ref, f"{mode} whole k={wk!r}", **tol(mode))
        names = [r["name"] for r in g.profile(mel.to(cuda_device))[1]]
        if wk:
            for nm in ("mrf_block_k7_c32", "mrf_block_k11_c32", "mrf_block_k7_c64", "mrf_block_k11_c64"):
                assert names.count(nm) == 1, (nm, names)
    assert max_abs(outs[0].numpy(), outs[1].numpy()) <= 2 * tol(mode).get("max_abs_tol", 1e-4)


@pytest.mark.parametrize("mode", ["fp32", "f16x3"])
def test_nonfinite_mel_stays_in_its_utterance(cuda_device, mode):
    """A NaN / inf mel value is outside the generator's contract (the kernels build without NaN
    semantics, include/tts_mi355x.h), but it must not leak: every other utterance of the batch is
    bitwise the clean run's (per-utterance planes and f16x3 statistics, split over lanes)."""
    sd = synthetic.hifigan_state_dict(seed=1234, weight_norm=False)
    g = HifiganGenerator(**V1, math_mode=mode)
    g.remove_weight_norm()
    g.load_state_dict(sd)
    g = g.to(cuda_device)
    mel = synthetic.mel(3, 40, seed=5).to(cuda_device)
    clean = g.inference(mel)
    for bad_value in (float("nan"), float("inf")):
        bad = mel.clone()
        bad[1, 7, 20] = bad_value
        out = g.inference(bad)
        assert torch.equal(out[0], clean[0]) and torch.equal(out[2], clean[2]), bad_value
