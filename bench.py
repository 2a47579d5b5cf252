#!/usr/bin/env python3
"""Benchmark: HiFiGAN-v1 mel->waveform on MI355X (BASELINE.json metric / config 2).

One "step" = ``HifiganGenerator.inference`` on a resident [32, 80, 1024] fp32 mel batch
(replicate pad 5 -> 1034 frames -> 32 x 264,704 output samples), through the C-ABI library.
One process per GPU; with N GPUs every rank vocodes its own 32-utterance shard (weak
scaling, config 4's 256 utterances at N=8, no exchange step on the data path).

Prints ONE JSON line (rank 0) with the driver contract fields plus:
  roofline     : the dominant kernel family's algorithmic FLOP/s (hipEvent-timed inside one
                 profiled forward, on the stream the kernels run on) vs the 157.3 TF fp32 peak
  cpu_baseline : the CPU oracle (oracle/hifigan_ref.py, torch.nn.functional fp32, the same
                 ATen kernels as the reference) on a bounded sample, rank 0 at N=1 only
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "tts-3_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_PEAK_TFLOPS = 157.3  # MI355X fp32 (vector = matrix), MI355X_MICROARCH.md
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA
# ceiling of each math mode in algorithmic fp32 FLOP/s: fp32x6 issues 6 bf16 MFMA products
# per fp32 multiply-accumulate, f16x3 3 fp16 products (same MFMA rate as bf16); see
# include/tts_mi355x.h TTS_MATH_*
MODE_PEAK = {"fp32": FP32_PEAK_TFLOPS, "fp32x6": BF16_PEAK_TFLOPS / 6.0, "f16x3": BF16_PEAK_TFLOPS / 3.0,
             "bf16": BF16_PEAK_TFLOPS}
PEAK_BASIS = {
    "fp32": "fp32 MFMA 157.3 TF",
    "fp32x6": "bf16 dense MFMA 2.5 PF / 6 products per fp32 MAC",
    "f16x3": "fp16 dense MFMA 2.5 PF / 3 products per fp32 MAC",
    "bf16": "bf16 dense MFMA 2.5 PF",
}
DTYPE = {
    "fp32": "fp32",
    "fp32x6": "fp32 (bf16x6 split on bf16 MFMA, fp32 accumulate)",
    "f16x3": "fp32 (power-of-2 scaled fp16 hi/lo split on fp16 MFMA, fp32 accumulate)",
    "bf16": "bf16 (bf16 MFMA operands, fp32 accumulate, fp32 activations)",
}
HBM_PEAK_GBS = 8000.0
SAMPLE_RATE = 22050
METRIC = "audio samples/sec + RTF, HiFiGAN-v1 22.05kHz 80-mel, batch 32 @ 1/2/4/8 GPU"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=32, help="utterances per GPU")
    p.add_argument("--frames", type=int, default=1024)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    p.add_argument("--comm", action="store_true",
                   help="also time an RCCL scatter of mels / gather of wavs from rank 0 (reported separately)")
    p.add_argument("--math-mode", default="f16x3", choices=sorted(MODE_PEAK),
                   help="conv contraction arithmetic (see include/tts_mi355x.h TTS_MATH_*)")
    p.add_argument("--no-alt", action="store_true", help="skip the secondary run in the other math mode")
    p.add_argument("--no-glow", action="store_true", help="skip the Glow-TTS decoder measurement")
    p.add_argument("--no-e2e", action="store_true", help="skip the Glow-TTS + HiFiGAN text->wav measurement")
    p.add_argument("--no-xtts", action="store_true", help="skip the XTTS waveform-decoder measurement")
    p.add_argument("--no-vits", action="store_true", help="skip the VITS waveform-path measurement")
    p.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic_hifigan_r02.json"))
    return p.parse_args()


def dominant_kernel(rows):
    fam = {}
    for r in rows:
        f = fam.setdefault(r["name"], {"ms": 0.0, "flops": 0.0, "bytes": 0.0, "n": 0})
        f["ms"] += r["ms"]
        f["flops"] += r["flops"]
        f["bytes"] += r["bytes"]
        f["n"] += 1
    name, f = max(fam.items(), key=lambda kv: kv[1]["ms"])
    return name, f, fam


def winograd_fields(fam_name: str, achieved: float, peak: float) -> dict:
    """The Winograd F(4,4) convs ("mrf_wino_k<K>_c<C>", wino8_kernel.hpp) compute the same outputs
    with 7*ceil(K/4)/4 instead of K products per (output, co, ci): `achieved` stays the algorithmic
    (direct-conv) FLOP rate, and the MFMA work actually issued is reported next to it."""
    if not fam_name.startswith("mrf_wino_k"):
        return {"algorithm": "direct"}
    K = int(fam_name.split("_k")[1].split("_")[0])
    ratio = 7 * ((K + 3) // 4) / 4 / K
    return {"algorithm": "winograd F(4,4)", "mfma_products_per_direct": ratio,
            "mfma_executed_tflops": achieved * ratio, "mfma_executed_frac": achieved * ratio / peak}


def cpu_baseline(budget_s: float):
    """Time the CPU oracle on a bounded sample of the same workload (rank 0, N=1)."""
    sys.path.insert(0, REPO)
    from oracle import hifigan_ref  # test infrastructure: the baseline being timed, not the product
    from tts_amd import synthetic
    from tts_amd.config import HIFIGAN_V1

    cores = len(os.sched_getaffinity(0))
    threads = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(threads)
    cfg = dict(in_channels=80, out_channels=1, **HIFIGAN_V1)
    sd = synthetic.hifigan_state_dict(**cfg, seed=1234, weight_norm=False)
    sd = {k: v.float() for k, v in sd.items()}
    B, T = 1, 256
    mel = synthetic.mel(B, T, seed=0)
    with torch.no_grad():
        hifigan_ref.hifigan_forward(sd, mel[:, :, :8], pad=5, dtype=torch.float32, **cfg)  # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float32, **cfg)
            n += 1
            el = time.perf_counter() - t0
            if el >= budget_s or n >= 1000:
                break
    samples = n * B * 256 * (T + 10)
    return {
        "value": samples / el,
        "unit": "samples/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n} x HifiganGenerator.inference on [1,80,{T}] (oracle/hifigan_ref.py, torch-CPU fp32, "
                  f"{threads} threads, {el:.1f} s)",
        "rtf": el / (samples / SAMPLE_RATE),
    }


def build_generator(math_mode, dev):
    from tts_amd import synthetic
    from tts_amd.config import HIFIGAN_V1
    from tts_amd.vocoder import HifiganGenerator

    cfg = dict(in_channels=80, out_channels=1, **HIFIGAN_V1)
    g = HifiganGenerator(**cfg, math_mode=math_mode)
    with contextlib.redirect_stdout(sys.stderr):  # the reference prints "Removing weight norm..."
        g.remove_weight_norm()
    g.load_state_dict(synthetic.hifigan_state_dict(**cfg, seed=1234, weight_norm=False))
    g.eval()
    return g.to(dev)


def time_steps(g, mel, steps, warmup, dev, world):
    for _ in range(warmup):
        g.inference(mel)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        g.inference(mel)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()) / steps * 1e3


def accuracy_check(gens, dev):
    """Each math mode vs the fp64 CPU oracle on a small sample (B=1 x 48 frames)."""
    sys.path.insert(0, REPO)
    from oracle import hifigan_ref  # test infrastructure: the checker, not the measured path
    from tts_amd import synthetic
    from tts_amd.config import HIFIGAN_V1

    cfg = dict(in_channels=80, out_channels=1, **HIFIGAN_V1)
    sd = synthetic.hifigan_state_dict(**cfg, seed=1234, weight_norm=False)
    mel = synthetic.mel(1, 48, seed=7)
    ref = hifigan_ref.hifigan_forward(sd, mel, pad=5, dtype=torch.float64, **cfg)
    out = {}
    for mode, g in gens.items():
        y = g.inference(mel.to(dev)).cpu().double()
        d = y - ref
        out[mode] = {"max_abs": float(d.abs().max()), "rel_rms": float(d.pow(2).mean().sqrt() / ref.pow(2).mean().sqrt())}
    return out


def glow_bench(dev, math_mode, steps=10, warmup=3, B=16, T=768, cpu=True):
    """Glow-TTS decoder reverse flow (config 3's decoder: B=16, T=768 mel frames, LJSpeech cfg)."""
    from tts_amd import synthetic
    from tts_amd.config import GLOW_TTS_DECODER as G
    from tts_amd.tts import Decoder

    cfg = dict(in_channels=G["in_channels"], hidden_channels=G["hidden_channels"], kernel_size=G["kernel_size"],
               dilation_rate=G["dilation_rate"], num_flow_blocks=G["num_flow_blocks"],
               num_coupling_layers=G["num_coupling_layers"], num_splits=G["num_splits"],
               num_squeeze=G["num_squeeze"])
    sd = synthetic.glow_decoder_state_dict(**cfg, seed=4321)
    d = Decoder(**cfg, dropout_p=G["dropout_p"], math_mode=math_mode)
    d.load_state_dict(sd)
    d.eval()
    d.store_inverse()
    d = d.to(dev)
    x = torch.randn(B, cfg["in_channels"], T, generator=torch.Generator().manual_seed(3)).to(dev)
    m = torch.ones(B, 1, T, device=dev)
    for _ in range(warmup):
        d(x, m, reverse=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        d(x, m, reverse=True)
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / steps * 1e3
    _, rows = d.profile(x, m)
    name, fam, fams = dominant_kernel(rows)
    flops = sum(r["flops"] for r in rows)
    out = {
        "workload": f"Glow-TTS decoder reverse, [{B},80,{T}] (12 flows x 4 WN layers, hidden 192, k5)",
        "math_mode": math_mode,
        "ms_per_step": ms,
        "mel_frames_per_s": B * T / (ms / 1e3),
        "launches_per_step": len(rows),
        "tflops": flops / (ms / 1e3) / 1e12,
        "kernel_sum_ms": sum(r["ms"] for r in rows),
        "dominant_kernel": {"name": name, "avg_launch_ms": fam["ms"] / fam["n"],
                            "achieved_tflops": fam["flops"] / fam["ms"] / 1e9, "launches": fam["n"]},
        "breakdown_ms": {k: round(v["ms"], 3) for k, v in sorted(fams.items(), key=lambda kv: -kv[1]["ms"])},
    }
    if math_mode != "fp32":  # the same flow in exact fp32 MFMA arithmetic, on the full bench input
        d32 = Decoder(**cfg, dropout_p=G["dropout_p"], math_mode="fp32")
        d32.load_state_dict(sd)
        d32.eval()
        d32.store_inverse()
        d32 = d32.to(dev)
        y, y32 = d(x, m, reverse=True)[0].double(), d32(x, m, reverse=True)[0].double()
        out["vs_fp32_mode"] = {"max_abs": float((y - y32).abs().max()),
                               "rel_rms": float((y - y32).pow(2).mean().sqrt() / y32.pow(2).mean().sqrt())}
        del d32
    if cpu:
        sys.path.insert(0, REPO)
        from oracle import glow_ref  # test infrastructure: the baseline being timed, not the product

        xs = x[:2].cpu()
        ms_ = m[:2].cpu()
        glow_ref.glow_decoder_reverse(sd, xs[:, :, :64], ms_[:, :, :64], dtype=torch.float32, **cfg)
        n, c0 = 0, time.perf_counter()
        with torch.no_grad():
            while True:
                glow_ref.glow_decoder_reverse(sd, xs, ms_, dtype=torch.float32, **cfg)
                n += 1
                if time.perf_counter() - c0 > 5.0:
                    break
        el = time.perf_counter() - c0
        out["cpu_baseline"] = {"mel_frames_per_s": n * 2 * T / el, "cores": torch.get_num_threads(), "kind": "port",
                               "sample": f"{n} x Decoder.forward(reverse=True) on [2,80,{T}] (oracle/glow_ref.py fp32)"}
    return out


def glow_tts_e2e_bench(dev, modes, steps=10, warmup=3, B=16, T_x=128):
    """Config 3: Glow-TTS (LJSpeech cfg) + HiFiGAN-v1 end to end, token ids -> waveform, B = 16 x 128
    tokens (durations ~6 frames/token from the synthetic predictor -> ~768 mel frames).
    ``modes`` = (glow decoder mode, vocoder mode) per variant; the encoder always runs fp32x6, the
    fp32-faithful mode (its durations are ceil()-quantised, so they must match the reference's)."""
    from tts_amd import synthetic
    from tts_amd.config import GLOW_TTS_DECODER as G, GLOW_TTS_ENCODER as E
    from tts_amd.synthesizer import AudioNorm, Synthesizer
    from tts_amd.tts import GlowTTS

    ecfg = dict(E, num_chars=64)
    dcfg = dict(in_channels=G["in_channels"], hidden_channels=G["hidden_channels"], kernel_size=G["kernel_size"],
                dilation_rate=G["dilation_rate"], num_flow_blocks=G["num_flow_blocks"],
                num_coupling_layers=G["num_coupling_layers"], num_splits=G["num_splits"],
                num_squeeze=G["num_squeeze"])
    sd = {f"encoder.{k}": v for k, v in
          synthetic.glow_encoder_state_dict(**ecfg, seed=8642, log_duration=1.872).items()}
    sd.update({f"decoder.{k}": v for k, v in synthetic.glow_decoder_state_dict(**dcfg, seed=4321).items()})
    tok = synthetic.tokens(B, T_x, 64, seed=11).to(dev)
    lens = torch.full((B,), T_x, dtype=torch.int64, device=dev)
    out = {"workload": f"Glow-TTS LJSpeech cfg + on-device hand-off (denormalize/normalize) + HiFiGAN-v1, "
                       f"[{B} x {T_x}] token ids -> waveform (encoder fp32x6, noise_scale 0, length_scale 1)",
           "variants": {}}
    for label, (dmode, vmode) in modes.items():
        m = GlowTTS(dict(num_chars=64), decoder_math_mode=dmode)
        m.load_state_dict(sd)
        m.eval()
        m.store_inverse()
        m = m.to(dev)
        voc = build_generator(vmode, dev)
        syn = Synthesizer(m, voc, AudioNorm(), AudioNorm())  # BaseAudioConfig defaults both sides

        def step():
            return syn.tts_batch(tok, lens)[0]

        for _ in range(warmup):
            wav = step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            wav = step()
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / steps * 1e3
        samples = wav.numel()
        mel = m.inference(tok, {"x_lengths": lens})["model_outputs"].transpose(1, 2).contiguous()
        torch.cuda.synchronize(dev)
        e0 = time.perf_counter()
        for _ in range(steps):
            m.inference(tok, {"x_lengths": lens})
        torch.cuda.synchronize(dev)
        ms_glow = (time.perf_counter() - e0) / steps * 1e3
        _, erows = m.encoder.profile(tok, lens)
        out["mel_frames"] = int(mel.shape[2])
        out["variants"][label] = {
            "glow_decoder_math_mode": dmode, "vocoder_math_mode": vmode,
            "ms_per_step": ms, "samples_per_s": samples / (ms / 1e3),
            "rtf": (ms / 1e3) / (samples / SAMPLE_RATE),
            "glow_tts_inference_ms": ms_glow,
            "encoder_kernel_ms": sum(r["ms"] for r in erows), "encoder_launches": len(erows),
        }
        del m, voc, syn
    return out


def xtts_decoder_bench(dev, math_mode, steps=10, warmup=3, B=16, T=64):
    """XTTS waveform decoder (HifiDecoder, xtts/hifigan_decoder.py:603-700): GPT latents [B, T, 1024]
    -> linear resampling x4 and x24000/22050 -> HiFiGAN (1024 -> 512 ch, conds in every upsampling
    layer) -> 24 kHz waveform."""
    from tts_amd import synthetic
    from tts_amd.tts import HifiDecoder

    d = HifiDecoder(math_mode=math_mode)
    cfg = dict(in_channels=1024, out_channels=1, resblock_type="1",
               resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], resblock_kernel_sizes=[3, 7, 11],
               upsample_kernel_sizes=[16, 16, 4, 4], upsample_initial_channel=512, upsample_factors=[8, 8, 2, 2],
               cond_channels=512, conv_pre_weight_norm=False, conv_post_weight_norm=False, conv_post_bias=False,
               cond_in_each_up_layer=True)
    d.waveform_decoder.load_state_dict(synthetic.hifigan_state_dict(**cfg, seed=321, weight_norm=True))
    d.eval()
    d = d.to(dev)
    lat = torch.randn(B, T, 1024, generator=torch.Generator().manual_seed(1)).to(dev)
    g = (torch.randn(B, 512, 1, generator=torch.Generator().manual_seed(2)) * 0.5).to(dev)
    for _ in range(warmup):
        wav = d.inference(lat, g)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        wav = d.inference(lat, g)
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / steps * 1e3
    return {"workload": f"XTTS HifiDecoder, [{B} x {T}] GPT latents -> 24 kHz waveform ({wav.shape[2]} samples each)",
            "math_mode": math_mode, "ms_per_step": ms, "samples_per_s": wav.numel() / (ms / 1e3),
            "rtf": (ms / 1e3) / (wav.numel() / 24000)}


def vits_bench(dev, steps=10, warmup=3, B=8, T=1024, cond=256):
    """Config 5 per GPU (batch 64 over 8 GPUs = 8 utterances each): VITS waveform path,
    z_p [B, 192, T] -> ResidualCouplingBlocks reverse (4 flows, speaker-conditioned) -> z * mask ->
    HiFiGAN decoder (in 192, 512 ch, cond_layer, no conv_post bias, no padding; vits.py:1156-1162)."""
    from tts_amd import synthetic
    from tts_amd.config import VITS_DECODER, VITS_FLOW
    from tts_amd.tts import ResidualCouplingBlocks
    from tts_amd.vocoder import HifiganGenerator

    fcfg = dict(VITS_FLOW, cond_channels=cond)
    dcfg = dict(VITS_DECODER, cond_channels=cond)
    fsd = synthetic.vits_flow_state_dict(**fcfg, seed=2469)
    dsd = synthetic.hifigan_state_dict(**dcfg, seed=99, weight_norm=False)
    gen = torch.Generator().manual_seed(9)
    zp = torch.randn(B, 192, T, generator=gen).to(dev)
    mask = torch.ones(B, 1, T, device=dev)
    g = torch.randn(B, cond, 1, generator=gen).to(dev)
    out = {"workload": f"VITS waveform path, [{B}, 192, {T}] latents (4-flow reverse + 512-ch HiFiGAN decoder, "
                       f"speaker cond {cond}) per GPU", "variants": {}}
    for label, (fmode, dmode) in {"bf16": ("bf16", "bf16"), "fp32_faithful": ("f16x3", "f16x3")}.items():
        flow = ResidualCouplingBlocks(fcfg["channels"], fcfg["hidden_channels"], fcfg["kernel_size"],
                                      fcfg["dilation_rate"], fcfg["num_layers"], num_flows=fcfg["num_flows"],
                                      cond_channels=cond, math_mode=fmode)
        flow.load_state_dict(fsd)
        flow = flow.to(dev)
        dec = HifiganGenerator(**{k: v for k, v in dcfg.items()}, math_mode=dmode)
        with contextlib.redirect_stdout(sys.stderr):
            dec.remove_weight_norm()
        dec.load_state_dict(dsd)
        dec = dec.to(dev)

        def step():
            z = flow(zp, mask, g=g, reverse=True)
            return dec(z * mask, g=g)

        for _ in range(warmup):
            wav = step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            wav = step()
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / steps * 1e3
        out["variants"][label] = {"flow_math_mode": fmode, "decoder_math_mode": dmode, "ms_per_step": ms,
                                  "samples_per_s": wav.numel() / (ms / 1e3),
                                  "rtf": (ms / 1e3) / (wav.numel() / SAMPLE_RATE)}
        del flow, dec
    return out


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from tts_amd import synthetic

    g = build_generator(a.math_mode, dev)
    B, T, pad = a.batch, a.frames, g.inference_padding
    mel = synthetic.mel(B, T, seed=rank).to(dev)
    g.reserve(B, T)
    torch.cuda.synchronize(dev)
    ms_per_step = time_steps(g, mel, a.steps, a.warmup, dev, world)
    samples_per_step = B * g.hop_length * (T + 2 * pad)  # per GPU
    value = world * samples_per_step / (ms_per_step / 1e3)
    rtf = (ms_per_step / 1e3) / (world * samples_per_step / SAMPLE_RATE)

    comm = None
    if a.comm and world > 1:
        from tts_amd.sharding import gather_batch, scatter_batch

        n = B * world
        full = synthetic.mel(n, T, seed=99).to(dev) if rank == 0 else None
        dist.barrier()
        torch.cuda.synchronize(dev)
        c0 = time.perf_counter()
        shard = scatter_batch(full, n, (80, T), dev)
        gather_batch(g.inference(shard), n)
        torch.cuda.synchronize(dev)
        comm = {"scatter_infer_gather_ms": (time.perf_counter() - c0) * 1e3, "utterances": n}

    # dominant-kernel roofline from one profiled forward (hipEvents per launch)
    _, rows = g.profile(mel)
    if os.environ.get("TTS_FORWARD_NAMES") and rank == 0:  # launch sequence for scripts/traffic_from_pmc.py
        json.dump([r["name"] for r in rows], open(os.environ["TTS_FORWARD_NAMES"], "w"))
    fam_name, fam, fams = dominant_kernel(rows)
    per_launch_flops = fam["flops"] / fam["n"]
    avg_ms = fam["ms"] / fam["n"]
    achieved = per_launch_flops / (avg_ms / 1e3) / 1e12
    total_flops = sum(r["flops"] for r in rows)
    traffic = None
    fwd_bytes = None  # PMC HBM bytes of one forward (profiles/traffic_hifigan_r02.json)
    if os.path.exists(a.traffic_json):
        try:
            tj = json.load(open(a.traffic_json))
            traffic = tj.get("per_launch_bytes", {}).get(f"{a.math_mode}:{fam_name}")
            fwd_bytes = tj.get("per_launch_bytes", {}).get(f"{a.math_mode}:__forward__")
        except Exception:
            traffic = None
    algo_bytes = sum(r["bytes"] for r in rows)  # compulsory activation/weight bytes per launch, summed
    step_s = ms_per_step / 1e3
    hbm = {
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "algorithmic_bytes_per_step": algo_bytes,
        "algorithmic_frac": algo_bytes / step_s / 1e9 / HBM_PEAK_GBS,
        "pmc_bytes_per_step": fwd_bytes,
        "achieved": fwd_bytes / step_s / 1e9 if fwd_bytes else None,
        "frac": fwd_bytes / step_s / 1e9 / HBM_PEAK_GBS if fwd_bytes else None,
    }

    alt = None
    gens = {a.math_mode: g}
    if not a.no_alt:
        other = "fp32" if a.math_mode != "fp32" else "fp32x6"
        g2 = build_generator(other, dev)
        g2.reserve(B, T)
        ms2 = time_steps(g2, mel, max(3, a.steps // 2), 1, dev, world)
        alt = {"math_mode": other, "ms_per_step": ms2, "value": world * samples_per_step / (ms2 / 1e3)}
        gens[other] = g2

    cpu = None
    acc = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        acc = accuracy_check(gens, dev)
        cpu = cpu_baseline(a.cpu_seconds)

    glow = None
    if rank == 0 and not a.no_glow:
        glow = glow_bench(dev, a.math_mode, cpu=(world == 1 and not a.no_cpu_baseline))

    e2e = None
    if rank == 0 and world == 1 and not a.no_e2e:
        e2e = glow_tts_e2e_bench(dev, {"fp32_faithful": ("f16x3", "f16x3"), "bf16": ("bf16", "bf16")})

    xtts = None
    if rank == 0 and world == 1 and not a.no_xtts:
        xtts = xtts_decoder_bench(dev, a.math_mode)

    vits = None
    if rank == 0 and world == 1 and not a.no_vits:
        vits = vits_bench(dev)

    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": DTYPE[a.math_mode],
            "math_mode": a.math_mode,
            "data": "synthetic N(0,1) mel (seed=rank), synthetic variance-preserving HiFiGAN-v1 weights (seed 1234)",
            "config": {
                "workload": "HiFiGAN-v1 22.05kHz inference, [32,80,1024] mel per GPU (replicate pad 5), fp32",
                "model": "HiFiGAN-v1 (hifigan_config.py generator_model_params)",
                "global_batch": B * world,
                "seq_len": T,
                "parallelism": f"dp{world} (utterance sharding, no collectives)",
            },
            "rtf": rtf,
            # samples of the unpadded mel (B * 256 * T), beside the padded numel above
            "useful_samples_per_s": value * T / (T + 2 * pad),
            "model_tflops": total_flops / (ms_per_step / 1e3) / 1e12,
            "model_frac_fp32_peak": total_flops / (ms_per_step / 1e3) / 1e12 / FP32_PEAK_TFLOPS,
            "roofline": {
                "bound": "mfma",
                "kernel": fam_name,
                "launches_per_step": fam["n"],
                "achieved": achieved,
                "peak": MODE_PEAK[a.math_mode],
                "peak_basis": PEAK_BASIS[a.math_mode],
                "unit": "TFLOP/s",
                "frac": achieved / MODE_PEAK[a.math_mode],
                "traffic": traffic,
                "flops_per_launch": per_launch_flops,
                "avg_launch_ms": avg_ms,
                **winograd_fields(fam_name, achieved, MODE_PEAK[a.math_mode]),
            },
            "hbm_roofline_step": hbm,
            "kernel_breakdown_ms": {k: round(v["ms"], 3) for k, v in sorted(fams.items(), key=lambda kv: -kv[1]["ms"])},
            "cpu_baseline": cpu,
            "alt_math_mode": alt,
            "glow_decoder": glow,
            "glow_tts_e2e": e2e,
            "xtts_decoder": xtts,
            "vits_waveform": vits,
            "accuracy_vs_fp64_oracle": acc,
        }
        if comm:
            rec["comm"] = comm
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
