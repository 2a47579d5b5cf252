"""Child process of tests/test_sharded_gpu.py: the sharded legs of configs 4 and 5 over a real
one-rank RCCL (torch.distributed "nccl") process group on cuda:0.

It runs in a fresh process so that the process group is built before any other GPU work (the
order bench.py's launcher uses), and writes what the parent test checks into ``<out>/result.npz``:

* config 4 (BASELINE.json configs[3], one GPU's shard): rank 0 holds a [32, 80, 1024] mel batch in
  HBM; ``scatter_batch`` -> ``HifiganGenerator.inference`` (f16x3) -> ``gather_batch``; the gathered
  waveforms must equal the unsharded forward bit for bit; rows 0 and 31 go to the parent for the
  fp64 oracle.
* config 5 (configs[4], one GPU's share of batch 64): latents [8, 192, 1024], ragged masks and
  speaker vectors scattered together, ``ResidualCouplingBlocks(reverse=True)`` -> z * mask -> the
  512-channel decoder in bf16, gathered; bitwise against the unsharded step; rows 0 and 6 (full and
  ragged) to the parent.

The reference has no inference collectives (vits.py:1156-1161 is the step each rank
runs).  usage: python tests/sharded_child.py OUT_DIR
"""
import os
import socket
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tts-3_amd"), os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main(out_dir: str) -> None:
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    import numpy as np
    import torch
    import torch.distributed as dist

    from tts_amd.sharding import gather_batch, init_distributed, scatter_batch, shard_sizes

    init_distributed("nccl", 0, timeout_s=180.0)  # before any other GPU work
    dev = torch.device("cuda", 0)
    res = {"backend": np.array(dist.get_backend()), "world": np.array(dist.get_world_size())}

    from tts_amd import synthetic
    from tts_amd.config import HIFIGAN_V1, VITS_DECODER, VITS_FLOW
    from tts_amd.tts import ResidualCouplingBlocks
    from tts_amd.vocoder import HifiganGenerator

    # ---- config 4: mel shard -> vocoder -> waveform shard
    V1 = dict(in_channels=80, out_channels=1, **HIFIGAN_V1)
    g = HifiganGenerator(**V1, math_mode="f16x3")
    g.remove_weight_norm()
    g.load_state_dict(synthetic.hifigan_state_dict(seed=1234, weight_norm=False))
    g = g.to(dev)
    n, T = 32, 1024
    full = synthetic.mel(n, T, seed=0).to(dev)
    shard_buf = torch.empty(max(shard_sizes(n, 1)), 80, T, device=dev)
    wav_full = torch.empty(n, 1, 256 * (T + 10), device=dev)
    x = scatter_batch(full, n, (80, T), dev, out=shard_buf)
    got = gather_batch(g.inference(x), n, out=wav_full)
    torch.cuda.synchronize()
    plain = g.inference(full)
    res["c4_scatter_bitwise"] = np.array(bool(torch.equal(x, full)))
    res["c4_bitwise"] = np.array(bool(torch.equal(got, plain)))
    res["c4_rows"] = got[[0, 31]].cpu().numpy()
    res["c4_shape"] = np.array(got.shape)
    del g, full, shard_buf, wav_full, got, plain, x

    # ---- config 5: latents + ragged masks + speaker vectors -> flow reverse -> decoder
    cond = 256
    B5, T5, lens5 = 8, 1024, [1024, 1024, 1024, 1024, 1024, 1024, 700, 1024]  # tests/test_configs_gpu.py
    gen = torch.Generator().manual_seed(9)
    zp = torch.randn(B5, 192, T5, generator=gen)
    gv = torch.randn(B5, cond, 1, generator=gen)
    mask = (torch.arange(T5)[None, :] < torch.tensor(lens5)[:, None]).float().unsqueeze(1)
    zp, gv, mask = zp.to(dev), gv.to(dev), mask.to(dev)
    fcfg = dict(VITS_FLOW, cond_channels=cond)
    dcfg = dict(VITS_DECODER, cond_channels=cond)
    flow = ResidualCouplingBlocks(fcfg["channels"], fcfg["hidden_channels"], fcfg["kernel_size"],
                                  fcfg["dilation_rate"], fcfg["num_layers"], num_flows=fcfg["num_flows"],
                                  cond_channels=cond, math_mode="bf16")
    flow.load_state_dict(synthetic.vits_flow_state_dict(**fcfg, seed=2469))
    flow = flow.to(dev)
    dec = HifiganGenerator(**dcfg, math_mode="bf16")
    dec.remove_weight_norm()
    dec.load_state_dict(synthetic.hifigan_state_dict(**dcfg, seed=99, weight_norm=False))
    dec = dec.to(dev)

    def step(z_, m_, g_):
        return dec(flow(z_, m_, g=g_, reverse=True) * m_, g=g_)

    zs = scatter_batch(zp, B5, (192, T5), dev)
    ms = scatter_batch(mask, B5, (1, T5), dev)
    gs = scatter_batch(gv, B5, (cond, 1), dev)
    got5 = gather_batch(step(zs, ms, gs), B5)
    torch.cuda.synchronize()
    plain5 = step(zp, mask, gv)
    res["c5_scatter_bitwise"] = np.array(bool(torch.equal(zs, zp) and torch.equal(ms, mask) and torch.equal(gs, gv)))
    res["c5_bitwise"] = np.array(bool(torch.equal(got5, plain5)))
    res["c5_rows"] = got5[[0, 6]].float().cpu().numpy()
    res["c5_shape"] = np.array(got5.shape)
    dist.barrier()
    dist.destroy_process_group()
    np.savez(os.path.join(out_dir, "result.npz"), **res)
    print("sharded child ok", flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
