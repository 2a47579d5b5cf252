#!/usr/bin/env python3
"""Benchmark: HiFiGAN-v1 mel->waveform on MI355X (BASELINE.json metric / config 2).

One "step" = ``HifiganGenerator.inference`` on a resident [32, 80, 1024] fp32 mel batch
(replicate pad 5 -> 1034 frames -> 32 x 264,704 output samples), through the C-ABI library.
One process per GPU.  ``--gpus N`` with N > 1 and no torchrun environment starts N rank
processes itself (``torch.distributed.run``, before anything touches the GPU); under torchrun
WORLD_SIZE must equal N.  At N > 1 one step is config 4's serving shape: rank 0 holds the
whole 32*N-utterance mel batch in HBM, scatters one 32-utterance shard to every rank (RCCL over
xGMI), every rank vocodes its shard, and rank 0 gathers the waveforms (weak scaling: 256
utterances at N=8).  The compute-only step (each rank on its resident shard) and the scatter /
gather times are reported beside it.

Prints ONE JSON line (rank 0) with the driver contract fields plus:
  roofline     : the dominant kernel family's executed MFMA FLOP/s (the products its algorithm
                 issues: Winograd F(4,4) point products, x3 fp16 products per fp32 MAC in f16x3),
                 timed by a hipEvent pair per launch inside one profiled forward on the stream the
                 kernels run on, against the dense peak of the matrix pipe it uses (fp16 / bf16
                 2.5 PF, fp32 157.3 TF); the direct-conv-equivalent rate is reported beside it
  cpu_baseline : the CPU oracle (oracle/hifigan_ref.py, torch.nn.functional fp32, the same
                 ATen kernels as the reference) on the bench's whole [32,80,1024] mel batch
                 (median of 3 runs after one warm-up), rank 0 at N=1 only
  build        : provenance of the loaded library (source hash stamped at build time, .so sha256)
"""
from __future__ import annotations

import argparse
import contextlib
import faulthandler
import json
import os
import socket
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "tts-3_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_PEAK_TFLOPS = 157.3  # MI355X fp32 (vector = matrix), MI355X_MICROARCH.md
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 / fp16 MFMA
# MFMA products each mode issues per fp32 multiply-accumulate, and the dense peak of the pipe
PRODUCTS = {"fp32": 1, "fp32x6": 6, "f16x3": 3, "bf16": 1}
PIPE_PEAK = {"fp32": FP32_PEAK_TFLOPS, "fp32x6": BF16_PEAK_TFLOPS, "f16x3": BF16_PEAK_TFLOPS, "bf16": BF16_PEAK_TFLOPS}
PIPE_BASIS = {"fp32": "fp32 MFMA dense 157.3 TF", "fp32x6": "bf16 MFMA dense 2.5 PF",
              "f16x3": "fp16 MFMA dense 2.5 PF", "bf16": "bf16 MFMA dense 2.5 PF"}
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
    p.add_argument("--math-mode", default="f16x3", choices=sorted(MODE_PEAK),
                   help="conv contraction arithmetic (see include/tts_mi355x.h TTS_MATH_*)")
    p.add_argument("--no-alt", action="store_true", help="skip the secondary run in the other math mode")
    p.add_argument("--no-glow", action="store_true", help="skip the Glow-TTS decoder measurement")
    p.add_argument("--no-e2e", action="store_true", help="skip the Glow-TTS + HiFiGAN text->wav measurement")
    p.add_argument("--no-xtts", action="store_true", help="skip the XTTS waveform-decoder measurement")
    p.add_argument("--no-vits", action="store_true", help="skip the VITS waveform-path measurement")
    p.add_argument("--no-vits-tts", action="store_true", help="skip the VITS tokens -> waveform measurement")
    p.add_argument("--no-rb2", action="store_true", help="skip the ResBlock2 (YourTTS decoder) measurement")
    p.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic_hifigan_r06.json"))
    p.add_argument("--mfma-json", default=os.path.join(REPO, "profiles", "mfma_busy_r06.json"),
                   help="counter-derived MFMA-busy fractions per family (scripts/mfma_from_pmc.py)")
    p.add_argument("--cpu-utts", type=int, default=0,
                   help="utterances of the bench batch the CPU baseline vocodes (0: the whole batch)")
    p.add_argument("--vits-batch", type=int, default=64, help="config 5 global batch (N > 1 leg)")
    p.add_argument("--vits-frames", type=int, default=1024, help="config 5 latent frames per utterance")
    p.add_argument("--vits-math-mode", default="bf16", choices=sorted(MODE_PEAK),
                   help="arithmetic of the config-5 sharded leg (BASELINE.json configs[4] names bf16; "
                        "independent of --math-mode, which sets the headline leg)")
    p.add_argument("--rehearse-sharded", action="store_true",
                   help="N = 1 only: run the config-4 / config-5 sharded legs over a one-rank process group "
                        "(exercises the RCCL scatter/gather path on one GPU; reported under *_rehearsal)")
    p.add_argument("--comm-timeout", type=float, default=300.0, help="collective timeout (s), fail-fast")
    p.add_argument("--rank-timeout", type=float, default=1500.0,
                   help="a rank that runs longer than this dumps its stack and exits (hung peer)")
    p.add_argument("--stub", action="store_true",
                   help="TEST ONLY: CPU stand-in vocoder over gloo (exercises the launcher and sharding "
                        "path without a GPU; its numbers are not a measurement)")
    return p.parse_args()


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a) -> int:
    """--gpus N without a torchrun environment: run N ranks under torch.distributed.run as a
    child process group (nothing in this process has touched the GPU) and return its status.
    A launch that outlives --rank-timeout + 120 s is killed as a whole."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        return p.wait(timeout=a.rank_timeout + 120)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, 9)
        p.wait()
        print(f"bench.py: {a.gpus}-rank launch timed out", file=sys.stderr)
        return 124


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


def algorithm_ratio(fam_name: str):
    """Multiplies the family's algorithm issues per direct-conv multiply: the Winograd F(4,4)
    convs ("mrf_wino_k<K>_c<C>", wino8_kernel.hpp) take 7*ceil(K/4)/4 instead of K products per
    (output, co, ci); every other kernel is a direct conv (1)."""
    if not fam_name.startswith("mrf_wino_k"):
        return "direct", 1.0
    K = int(fam_name.split("_k")[1].split("_")[0])
    return "winograd F(4,4)", 7 * ((K + 3) // 4) / 4 / K


def activation_planes(mode: str) -> str:
    """Element type of the HiFiGAN executor's activation planes in HBM (bf16 in the bf16 scheme unless
    TTS_MI355X_BF16_PLANES=0, hifigan.hpp planes16_)."""
    return "bf16" if mode == "bf16" and os.environ.get("TTS_MI355X_BF16_PLANES", "1") != "0" else "fp32"


def family_roofline(rows, mode: str):
    """The dominant kernel family of one profiled forward against the dense peak of the matrix pipe
    its arithmetic issues on (the headline's roofline definition, for the side lines)."""
    name, f, _ = dominant_kernel(rows)
    algo, ratio = algorithm_ratio(name)
    avg_ms = f["ms"] / f["n"]
    exec_flops = f["flops"] / f["n"] * ratio * PRODUCTS[mode]
    achieved = exec_flops / (avg_ms / 1e3) / 1e12
    step_ms = sum(r["ms"] for r in rows)
    return {"bound": "mfma", "kernel": name, "launches": f["n"], "avg_launch_ms": avg_ms, "algorithm": algo,
            "achieved": achieved, "peak": PIPE_PEAK[mode], "unit": "TFLOP/s", "frac": achieved / PIPE_PEAK[mode],
            "peak_basis": PIPE_BASIS[mode],
            "forward_mfma_tflops": sum(r["flops"] * algorithm_ratio(r["name"])[1] * PRODUCTS[mode] for r in rows)
            / (step_ms / 1e3) / 1e12,
            "forward_hbm_algorithmic_gbs": sum(r["bytes"] for r in rows) / (step_ms / 1e3) / 1e9,
            "profiled_forward_ms": step_ms}


def progress(msg: str):
    """One line per long phase on stderr (the JSON line stays alone on stdout): a run that goes quiet
    for minutes, e.g. during the CPU baseline, reads as hung to a watchdog."""
    print(f"bench.py: {msg}", file=sys.stderr, flush=True)


def cpu_baseline(mel, n_utts: int, pad: int = 5):
    """Time the CPU oracle on the first ``n_utts`` utterances of the bench's own mel batch (rank 0,
    N=1): one warm-up on one utterance, then the median of 3 runs (same inputs as the
    GPU run, median of >= 3)."""
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
    x = (mel[:n_utts] if n_utts > 0 else mel).cpu().contiguous()
    B, _, T = x.shape
    runs = []
    with torch.no_grad():
        progress(f"cpu baseline: warm-up, then 3 runs on [{B},80,{T}] ({threads} threads)")
        hifigan_ref.hifigan_forward(sd, x[:1], pad=pad, dtype=torch.float32, **cfg)  # warm-up
        for i in range(3):
            t0 = time.perf_counter()
            hifigan_ref.hifigan_forward(sd, x, pad=pad, dtype=torch.float32, **cfg)
            runs.append(time.perf_counter() - t0)
            progress(f"cpu baseline run {i + 1}/3: {runs[-1]:.1f} s")
    el = statistics.median(runs)
    samples = B * 256 * (T + 2 * pad)
    return {
        "value": samples / el,
        "unit": "samples/s",
        "cores": threads,
        "kind": "port",
        "sample": f"HifiganGenerator.inference on mel[0:{B}] of the bench batch ([{B},80,{T}] of "
                  f"[{mel.shape[0]},80,{T}]), oracle/hifigan_ref.py torch-CPU fp32, {threads} threads, "
                  f"median of 3 runs after 1 warm-up",
        "runs_s": runs,
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


def sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def timed(fn, steps, warmup, dev, world):
    """W untimed calls, then K calls bracketed by barrier + device sync on both sides; the
    max over ranks of the wall time, per call, in ms."""
    for _ in range(warmup):
        fn()
    sync(dev)
    if world > 1:
        dist.barrier()
    sync(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync(dev)
    if world > 1:
        dist.barrier()
    sync(dev)
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()) / steps * 1e3


def time_steps(g, mel, steps, warmup, dev, world):
    return timed(lambda: g.inference(mel), steps, warmup, dev, world)


class StubVocoder:
    """TEST ONLY (--stub): a CPU stand-in with the generator's call surface and output shape
    (hop 256, replicate pad 5), so the launcher / scatter / gather path runs without a GPU."""
    hop_length = 256
    inference_padding = 5

    def inference(self, mel):
        B, _, T = mel.shape
        x = torch.nn.functional.pad(mel, (5, 5), mode="replicate").mean(1, keepdim=True)
        return torch.tanh(x).repeat_interleave(self.hop_length, dim=2)

    def reserve(self, B, T):
        pass


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

        xs = x.cpu()
        ms_ = m.cpu()
        runs = []
        with torch.no_grad():
            glow_ref.glow_decoder_reverse(sd, xs, ms_, dtype=torch.float32, **cfg)  # warm-up
            for _ in range(3):
                c0 = time.perf_counter()
                glow_ref.glow_decoder_reverse(sd, xs, ms_, dtype=torch.float32, **cfg)
                runs.append(time.perf_counter() - c0)
        el = statistics.median(runs)
        out["cpu_baseline"] = {"mel_frames_per_s": B * T / el, "cores": torch.get_num_threads(), "kind": "port",
                               "sample": f"Decoder.forward(reverse=True) on the same [{B},80,{T}] input "
                                         f"(oracle/glow_ref.py fp32), median of 3 runs after 1 warm-up",
                               "runs_s": runs}
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
        # the vocoder's kernels on a mel of the same shape (one profiled forward, serial schedule)
        _, vrows = voc.profile(mel)
        out["mel_frames"] = int(mel.shape[2])
        out["variants"][label] = {
            "glow_decoder_math_mode": dmode, "vocoder_math_mode": vmode,
            "vocoder_activation_planes": activation_planes(vmode),
            "ms_per_step": ms, "samples_per_s": samples / (ms / 1e3),
            "rtf": (ms / 1e3) / (samples / SAMPLE_RATE),
            "glow_tts_inference_ms": ms_glow,
            "encoder_kernel_ms": sum(r["ms"] for r in erows), "encoder_launches": len(erows),
            "vocoder_roofline": family_roofline(vrows, vmode),
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
        z = flow(zp, mask, g=g, reverse=True) * mask
        _, rows = dec.profile(z, g=g)
        out["variants"][label] = {"flow_math_mode": fmode, "decoder_math_mode": dmode,
                                  "decoder_activation_planes": activation_planes(dmode), "ms_per_step": ms,
                                  "samples_per_s": wav.numel() / (ms / 1e3),
                                  "rtf": (ms / 1e3) / (wav.numel() / SAMPLE_RATE),
                                  "decoder_roofline": family_roofline(rows, dmode)}
        del flow, dec
    return out


def rb2_bench(dev, steps=10, warmup=3, B=8, T=1024, cond=512):
    """ResBlock2 generator (hifigan_generator.py:108-159): the YourTTS waveform decoder, i.e. the VITS
    decoder with resblock_type_decoder "2" (recipes/vctk/yourtts/train_yourtts.py:134; vits.py:704-718:
    in 192, 512 channels, kernels 3 / 7 / 11 with ResBlock2 dilations (1, 3), speaker cond 512, no
    conv_post bias, no padding), on [B, 192, T] latents; the whole-block launches against the per-conv
    path (TTS_MI355X_RESBLOCK3=0) in each math mode."""
    from tts_amd import synthetic
    from tts_amd.config import VITS_DECODER
    from tts_amd.vocoder import HifiganGenerator

    dcfg = dict(VITS_DECODER, cond_channels=cond, resblock_type="2")
    dsd = synthetic.hifigan_state_dict(**dcfg, seed=77, weight_norm=False)
    gen = torch.Generator().manual_seed(10)
    z = torch.randn(B, 192, T, generator=gen).to(dev)
    g = torch.randn(B, cond, 1, generator=gen).to(dev)
    out = {"workload": f"YourTTS waveform decoder (HiFiGAN, ResBlock2), [{B}, 192, {T}] latents, speaker cond "
                       f"{cond}", "variants": {}}
    prev = os.environ.get("TTS_MI355X_RESBLOCK3")
    try:
        for mode in ("f16x3", "bf16"):
            for fused in (True, False):
                os.environ["TTS_MI355X_RESBLOCK3"] = "all" if fused else "0"  # read at create
                dec = HifiganGenerator(**dcfg, math_mode=mode)
                with contextlib.redirect_stdout(sys.stderr):
                    dec.remove_weight_norm()
                dec.load_state_dict(dsd)
                dec = dec.to(dev)
                for _ in range(warmup):
                    wav = dec(z, g=g)
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(steps):
                    wav = dec(z, g=g)
                torch.cuda.synchronize(dev)
                ms = (time.perf_counter() - t0) / steps * 1e3
                _, rows = dec.profile(z, g=g)
                fams = {}
                for r in rows:
                    fams[r["name"]] = fams.get(r["name"], 0.0) + r["ms"]
                out["variants"][f"{mode}_{'whole_block' if fused else 'per_conv'}"] = {
                    "math_mode": mode, "ms_per_step": ms, "samples_per_s": wav.numel() / (ms / 1e3),
                    "rtf": (ms / 1e3) / (wav.numel() / SAMPLE_RATE), "decoder_roofline": family_roofline(rows, mode),
                    "kernel_breakdown_ms": {k: round(v, 3) for k, v in sorted(fams.items(), key=lambda kv: -kv[1])}}
                del dec
    finally:
        if prev is None:
            os.environ.pop("TTS_MI355X_RESBLOCK3", None)
        else:
            os.environ["TTS_MI355X_RESBLOCK3"] = prev
    return out


def vits_tts_bench(dev, steps=5, warmup=2, B=16, T_x=128):
    """Vits.inference end to end (vits.py:1088-1174), token ids -> waveform on the device: TextEncoder,
    StochasticDurationPredictor(reverse), durations, alignment expansion, 4-flow reverse, 512-channel
    decoder; VitsArgs defaults (LJSpeech VITS: hidden 192, 6 text layers), synthetic weights, both
    noise draws on the device (inference_noise_scale 0.667, _dp 1.0)."""
    from tts_amd import synthetic
    from tts_amd.config import VITS_FLOW, VITS_SDP, VITS_TEXT_ENCODER
    from tts_amd.tts import Vits

    tok = synthetic.tokens(B, T_x, 64, seed=12).to(dev)
    lens = torch.full((B,), T_x, dtype=torch.int64, device=dev)
    out = {"workload": f"Vits.inference, [{B} x {T_x}] token ids -> 22.05 kHz waveform (VitsArgs defaults, "
                       "512-ch decoder; text encoder + SDP fp32x6)", "variants": {}}
    for label, (fm, dm) in {"fp32_faithful": ("f16x3", "f16x3"), "bf16": ("bf16", "bf16")}.items():
        v = Vits(dict(num_chars=64), text_math_mode="fp32x6", flow_math_mode=fm, decoder_math_mode=dm)
        v.text_encoder.load_state_dict(synthetic.vits_text_encoder_state_dict(num_chars=64, **VITS_TEXT_ENCODER))
        v.duration_predictor.load_state_dict(synthetic.vits_sdp_state_dict(**VITS_SDP, log_duration=1.2))
        v.flow.load_state_dict(synthetic.vits_flow_state_dict(**VITS_FLOW, seed=2469))
        v.waveform_decoder.load_state_dict(synthetic.hifigan_state_dict(
            in_channels=192, out_channels=1, upsample_initial_channel=512, conv_pre_weight_norm=False,
            conv_post_weight_norm=False, conv_post_bias=False, seed=99, weight_norm=True))
        v = v.eval().to(dev)
        gen = torch.Generator(device=dev)

        def step():
            gen.manual_seed(5)  # the same durations every step (both noise draws pinned)
            nz_dp = torch.randn(B, 2, T_x, device=dev, generator=gen)
            return v.inference(tok, {"x_lengths": lens, "noise_dp": nz_dp})

        for _ in range(warmup):
            o = step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            o = step()
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / steps * 1e3
        n = o["model_outputs"].numel()
        out["variants"][label] = {"flow_math_mode": fm, "decoder_math_mode": dm, "ms_per_step": ms,
                                  "samples_per_s": n / (ms / 1e3), "rtf": (ms / 1e3) / (n / SAMPLE_RATE),
                                  "mel_frames": int(o["z"].shape[2])}
        del v
    return out


class StubVits:
    """TEST ONLY (--stub): CPU stand-in of the VITS flow + decoder with the real output shape
    (z [B, 192, T] -> wav [B, 1, 256 T])."""

    def __call__(self, zp, mask, g):
        return torch.tanh(zp.mean(1, keepdim=True) * mask + g.mean(1, keepdim=True)).repeat_interleave(256, dim=2)


def vits_sharded_bench(dev, world, rank, steps, warmup, stub=False, global_batch=64, T=1024, cond=256,
                       mode="bf16"):
    """Config 5 (BASELINE.json configs[4]): VITS flow + 512-channel decoder, global batch 64 over the
    ranks (strong scaling: 64 / world utterances each).  Rank 0 holds the [64, 192, T] latents, the
    masks and the speaker vectors in HBM; one step scatters the three (RCCL), every rank runs
    ResidualCouplingBlocks(reverse=True) -> z * mask -> the decoder on its shard, and rank 0 gathers
    the waveforms.  Also reports the compute-only step and the collectives alone."""
    from tts_amd import synthetic
    from tts_amd.config import VITS_DECODER, VITS_FLOW
    from tts_amd.sharding import gather_batch, scatter_batch, shard_sizes

    n = global_batch
    per = shard_sizes(n, world)[rank]
    gen = torch.Generator().manual_seed(9)
    full_z = full_m = full_g = None
    if rank == 0:
        full_z = torch.randn(n, 192, T, generator=gen).to(dev)
        lens = torch.randint(T // 2, T + 1, (n,), generator=gen)
        lens[0] = T
        full_m = (torch.arange(T)[None] < lens[:, None]).float().unsqueeze(1).to(dev)
        full_g = torch.randn(n, cond, 1, generator=gen).to(dev)
    cap = max(shard_sizes(n, world))
    bz = torch.empty(cap, 192, T, device=dev)
    bm = torch.empty(cap, 1, T, device=dev)
    bg = torch.empty(cap, cond, 1, device=dev)
    if stub:
        step_fn = StubVits()
    else:
        from tts_amd.tts import ResidualCouplingBlocks
        from tts_amd.vocoder import HifiganGenerator

        fcfg = dict(VITS_FLOW, cond_channels=cond)
        dcfg = dict(VITS_DECODER, cond_channels=cond)
        flow = ResidualCouplingBlocks(fcfg["channels"], fcfg["hidden_channels"], fcfg["kernel_size"],
                                      fcfg["dilation_rate"], fcfg["num_layers"], num_flows=fcfg["num_flows"],
                                      cond_channels=cond, math_mode=mode)
        flow.load_state_dict(synthetic.vits_flow_state_dict(**fcfg, seed=2469))
        flow = flow.to(dev)
        dec = HifiganGenerator(**dcfg, math_mode=mode)
        with contextlib.redirect_stdout(sys.stderr):
            dec.remove_weight_norm()
        dec.load_state_dict(synthetic.hifigan_state_dict(**dcfg, seed=99, weight_norm=False))
        dec = dec.to(dev)

        def step_fn(zp, mask, g):
            return dec(flow(zp, mask, g=g, reverse=True) * mask, g=g)
    S = 256 * T
    wav_full = torch.empty(n, 1, S, device=dev) if rank == 0 else None

    def scatter():
        return (scatter_batch(full_z, n, (192, T), dev, out=bz), scatter_batch(full_m, n, (1, T), dev, out=bm),
                scatter_batch(full_g, n, (cond, 1), dev, out=bg))

    z, m, g = scatter()
    z, m, g = z.clone(), m.clone(), g.clone()  # resident shard for the compute-only timing
    wav = step_fn(z, m, g)

    def step():
        zs, ms, gs = scatter()
        gather_batch(step_fn(zs, ms, gs), n, out=wav_full)

    ms = timed(step, steps, warmup, dev, world)
    compute_ms = timed(lambda: step_fn(z, m, g), steps, warmup, dev, world)
    scatter_ms = timed(scatter, max(3, steps), 1, dev, world)
    gather_ms = timed(lambda: gather_batch(wav, n, out=wav_full), max(3, steps), 1, dev, world)
    step()
    check = None
    if rank == 0:  # rank 0's own rows, vocoded alone, equal the gathered ones bit for bit
        check = bool(torch.equal(wav_full[:per], step_fn(full_z[:per], full_m[:per], full_g[:per])))
    samples = n * S
    return {
        "workload": f"config 5: VITS flow reverse (4 flows, speaker cond {cond}) + 512-ch HiFiGAN decoder, global "
                    f"batch {n} x {T} latent frames over {world} rank(s) ({per} each), rank 0 scatters latents / "
                    f"masks / speaker vectors and gathers the waveforms (RCCL)",
        "math_mode": "stub" if stub else mode, "scaling": "strong", "world_size": world, "global_batch": n,
        "per_rank_batch": per, "ms_per_step": ms, "samples_per_s": samples / (ms / 1e3),
        "rtf": (ms / 1e3) / (samples / SAMPLE_RATE),
        "compute_only_ms_per_step": compute_ms, "scatter_ms": scatter_ms, "gather_ms": gather_ms,
        "rank0_rows_bitwise_equal": check,
    }


def rank_devices(world, rank, local, dev):
    """Every rank's (rank, local rank, device, PCI bus) as torch.distributed saw it."""
    me = {"rank": rank, "local_rank": local, "device": str(dev)}
    if dev.type == "cuda":
        p = torch.cuda.get_device_properties(dev)
        me.update(name=p.name, pci_bus_id=getattr(p, "pci_bus_id", None), gcn_arch=getattr(p, "gcnArchName", None))
    if world == 1:
        return [me]
    out = [None] * world
    dist.all_gather_object(out, me)
    return out


def sharded_step_bench(g, B, T, dev, world, rank, steps, warmup):
    """Config 4: rank 0 holds [B*world, 80, T] in HBM; one step = scatter the mel shards ->
    every rank vocodes B utterances -> gather the waveforms on rank 0.  Also times the scatter
    and the gather alone."""
    from tts_amd import synthetic
    from tts_amd.sharding import gather_batch, scatter_batch

    n = B * world
    S = g.hop_length * (T + 2 * g.inference_padding)
    full = synthetic.mel(n, T, seed=0).to(dev) if rank == 0 else None
    shard = torch.empty(B, 80, T, device=dev)
    wav = g.inference(shard.zero_())
    wav_full = torch.empty(n, 1, S, device=dev) if rank == 0 else None

    def step():
        x = scatter_batch(full, n, (80, T), dev, out=shard)
        gather_batch(g.inference(x), n, out=wav_full)

    ms = timed(step, steps, warmup, dev, world)
    scatter_ms = timed(lambda: scatter_batch(full, n, (80, T), dev, out=shard), max(3, steps), 1, dev, world)
    gather_ms = timed(lambda: gather_batch(wav, n, out=wav_full), max(3, steps), 1, dev, world)
    # parity of the sharded path: rank 0's gathered rows equal each shard vocoded alone (the
    # generator is batch-invariant bit for bit)
    step()
    check = None
    if rank == 0:
        check = bool(torch.equal(wav_full[-B:], g.inference(full[-B:])))
    return {"ms": ms, "scatter_ms": scatter_ms, "gather_ms": gather_ms, "utterances": n,
            "mel_bytes": 4 * n * 80 * T, "wav_bytes": 4 * n * S, "last_shard_bitwise_equal": check}


def main():
    a = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        sys.exit(launch_ranks(a))  # before anything touches the GPU
    world = int(env_world or 1)
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    faulthandler.dump_traceback_later(a.rank_timeout, exit=True)  # a hung peer ends this rank
    # stdout carries exactly the one JSON line: whatever native libraries print there (RCCL's
    # version banner at communicator setup) goes to stderr instead
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)

    def emit(rec):
        os.write(json_fd, (json.dumps(rec) + "\n").encode())

    rehearse = a.rehearse_sharded and world == 1
    dist_on = world > 1 or rehearse
    if rehearse:  # a one-rank process group (no torchrun needed)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if a.stub:
        dev = torch.device("cpu")
        if dist_on:
            from tts_amd.sharding import init_distributed
            init_distributed("gloo", local, a.comm_timeout)
        g = StubVocoder()
    else:
        dev = torch.device("cuda", local)
        if dist_on:
            from tts_amd.sharding import init_distributed
            init_distributed("nccl", local, a.comm_timeout)
        g = build_generator(a.math_mode, dev)
    devices = rank_devices(world, rank, local, dev)
    real_world = dist.get_world_size() if world > 1 else 1

    from tts_amd import synthetic

    B, T, pad = a.batch, a.frames, g.inference_padding
    samples_per_step = B * g.hop_length * (T + 2 * pad)  # per GPU
    mel = synthetic.mel(B, T, seed=rank).to(dev)  # this rank's resident shard
    g.reserve(B, T)
    sync(dev)
    compute_ms = time_steps(g, mel, a.steps, a.warmup, dev, world)
    shard = None
    if dist_on:
        shard = sharded_step_bench(g, B, T, dev, world, rank, a.steps, a.warmup)
    ms_per_step = shard["ms"] if world > 1 else compute_ms
    value = world * samples_per_step / (ms_per_step / 1e3)
    rtf = (ms_per_step / 1e3) / (world * samples_per_step / SAMPLE_RATE)

    rec = {
        "metric": METRIC,
        "value": value,
        "unit": "samples/s",
        "n_gpus": real_world,
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
            "workload": f"HiFiGAN-v1 22.05kHz inference, [{B},80,{T}] mel per GPU (replicate pad 5), fp32"
                        + (f"; config 4: rank 0 scatters [{B * world},80,{T}] and gathers the waveforms (RCCL)"
                           if world > 1 else ""),
            "model": "HiFiGAN-v1 (hifigan_config.py generator_model_params)",
            "global_batch": B * world,
            "seq_len": T,
            "parallelism": f"dp{world} (utterance sharding; " + ("RCCL scatter/gather from rank 0)" if world > 1
                                                                 else "no collectives)"),
        },
        "rtf": rtf,
        # samples of the unpadded mel (B * 256 * T), beside the padded numel above
        "useful_samples_per_s": value * T / (T + 2 * pad),
        "world_size": real_world,
        "devices": devices,
    }
    if shard is not None:
        rec["sharded_rehearsal" if rehearse else "sharded"] = {
            "compute_only_ms_per_step": compute_ms,
            "compute_only_value": world * samples_per_step / (compute_ms / 1e3),
            "scatter_ms": shard["scatter_ms"], "gather_ms": shard["gather_ms"],
            "comm_share_of_step": (shard["scatter_ms"] + shard["gather_ms"]) / ms_per_step,
            "utterances": shard["utterances"], "mel_bytes": shard["mel_bytes"], "wav_bytes": shard["wav_bytes"],
            "last_shard_bitwise_equal": shard["last_shard_bitwise_equal"],
        }
    if dist_on and not a.no_vits:  # config 5 at N > 1 (its N = 1 side line is vits_waveform)
        v5 = vits_sharded_bench(dev, world, rank, a.steps, a.warmup, stub=a.stub, global_batch=a.vits_batch,
                                T=a.vits_frames, mode=a.vits_math_mode)
        if rank == 0:
            rec["config5_sharded_rehearsal" if rehearse else "config5_sharded"] = v5
    if a.stub:
        rec["data"] = "STUB (test only): CPU stand-in vocoder, not a measurement"
        rec["dtype"] = "fp32"
        if rank == 0:
            emit(rec)
        if dist_on:
            dist.barrier()
            dist.destroy_process_group()
        return

    from tts_amd import _native

    rec["build"] = _native.build_info()

    # dominant-kernel roofline from one profiled forward (hipEvents per launch)
    _, rows = g.profile(mel)
    if os.environ.get("TTS_FORWARD_NAMES") and rank == 0:  # launch sequence for scripts/traffic_from_pmc.py
        json.dump([r["name"] for r in rows], open(os.environ["TTS_FORWARD_NAMES"], "w"))
    fam_name, fam, fams = dominant_kernel(rows)
    per_launch_flops = fam["flops"] / fam["n"]  # direct-conv FLOPs of one launch (2 per MAC)
    avg_ms = fam["ms"] / fam["n"]
    direct_tflops = per_launch_flops / (avg_ms / 1e3) / 1e12
    algo, ratio = algorithm_ratio(fam_name)
    exec_flops = per_launch_flops * ratio * PRODUCTS[a.math_mode]  # MFMA FLOPs the launch issues
    achieved = exec_flops / (avg_ms / 1e3) / 1e12
    total_flops = sum(r["flops"] for r in rows)
    traffic = None
    fwd_bytes = None  # PMC HBM bytes of one forward (profiles/traffic_hifigan_r06.json)
    if os.path.exists(a.traffic_json):
        try:
            tj = json.load(open(a.traffic_json))
            traffic = tj.get("per_launch_bytes", {}).get(f"{a.math_mode}:{fam_name}")
            fwd_bytes = tj.get("per_launch_bytes", {}).get(f"{a.math_mode}:__forward__")
        except Exception:
            traffic = None
    busy = {}
    if os.path.exists(a.mfma_json):
        try:
            mj = json.load(open(a.mfma_json))
            fb = mj.get("families", {}).get(f"{a.math_mode}:{fam_name}")
            if fb:
                busy = {"mfma_busy_frac": fb["mfma_busy_frac"], "clock_ghz": fb["clock_ghz"],
                        "mfma_busy_frac_at_clock": fb.get("mfma_busy_frac_at_clock"),
                        "mfma_busy_source": os.path.relpath(a.mfma_json, REPO)}
        except Exception:
            busy = {}
    algo_bytes = sum(r["bytes"] for r in rows)  # compulsory activation/weight bytes per launch, summed
    step_s = compute_ms / 1e3
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
    if not a.no_alt and world == 1:
        other = "fp32" if a.math_mode != "fp32" else "fp32x6"
        g2 = build_generator(other, dev)
        g2.reserve(B, T)
        ms2 = time_steps(g2, mel, max(3, a.steps // 2), 1, dev, world)
        alt = {"math_mode": other, "ms_per_step": ms2, "value": world * samples_per_step / (ms2 / 1e3)}
        gens[other] = g2

    cpu = None
    acc = None
    if rank == 0:
        progress(f"timed steps done: {ms_per_step:.2f} ms/step")
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        acc = accuracy_check(gens, dev)
        cpu = cpu_baseline(mel, a.cpu_utts, pad)

    side = rank == 0 and world == 1
    if side:
        progress("side lines")
    glow = glow_bench(dev, a.math_mode, cpu=not a.no_cpu_baseline) if side and not a.no_glow else None
    e2e = (glow_tts_e2e_bench(dev, {"fp32_faithful": ("f16x3", "f16x3"), "bf16": ("bf16", "bf16")})
           if side and not a.no_e2e else None)
    if side:
        progress("side lines: glow decoder and Glow-TTS e2e done")
    xtts = xtts_decoder_bench(dev, a.math_mode) if side and not a.no_xtts else None
    vits = vits_bench(dev) if side and not a.no_vits else None
    vits_tts = vits_tts_bench(dev) if side and not a.no_vits_tts else None
    rb2 = rb2_bench(dev) if side and not a.no_rb2 else None
    if side:
        progress("side lines done")

    if rank == 0:
        rec.update({
            "model_tflops": total_flops / step_s / 1e12,
            "model_frac_fp32_peak": total_flops / step_s / 1e12 / FP32_PEAK_TFLOPS,
            "roofline": {
                "bound": "mfma",
                "kernel": fam_name,
                "launches_per_step": fam["n"],
                "achieved": achieved,
                "peak": PIPE_PEAK[a.math_mode],
                "peak_basis": PIPE_BASIS[a.math_mode],
                "unit": "TFLOP/s",
                "frac": achieved / PIPE_PEAK[a.math_mode],
                "traffic": traffic,
                "achieved_basis": (f"MFMA FLOPs the launch issues ({algo}: {ratio:.4f} products per direct-conv "
                                   f"multiply, x{PRODUCTS[a.math_mode]} {a.math_mode} products per fp32 MAC) / "
                                   "avg launch time"),
                "mfma_flops_per_launch": exec_flops,
                "algorithm": algo,
                "products_per_direct_multiply": ratio,
                "avg_launch_ms": avg_ms,
                "avg_launch_ms_source": ("hipEvent pair around every launch of one profiled forward (serialised "
                                         "launches, not the timed steps)"),
                # the same launch as a direct conv's FLOP rate, against the mode's fp32 ceiling and
                # BASELINE.md's fp32 basis (a Winograd kernel's saving shows up here as > MFMA rate)
                "direct_conv_flops_per_launch": per_launch_flops,
                "direct_equivalent_tflops": direct_tflops,
                "direct_equivalent_frac_of_mode_ceiling": direct_tflops / MODE_PEAK[a.math_mode],
                "mode_ceiling_basis": PEAK_BASIS[a.math_mode],
                "direct_equivalent_vs_fp32_peak": direct_tflops / FP32_PEAK_TFLOPS,
                **busy,
            },
            "hbm_roofline_step": hbm,
            "kernel_breakdown_ms": {k: round(v["ms"], 3) for k, v in sorted(fams.items(), key=lambda kv: -kv[1]["ms"])},
            "kernel_breakdown_source": ("one profiled forward: a hipEvent pair around every launch serialises them, "
                                        "so the families sum above ms_per_step"),
            "cpu_baseline": cpu,
            "alt_math_mode": alt,
            "glow_decoder": glow,
            "glow_tts_e2e": e2e,
            "xtts_decoder": xtts,
            "vits_waveform": vits,
            "vits_tts_e2e": vits_tts,
            "resblock2_decoder": rb2,
            "accuracy_vs_fp64_oracle": acc,
        })
        emit(rec)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    main()
