"""Utterance sharding across ranks (tts_amd/sharding.py) on CPU with gloo, world_size 2 and 3."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tts_amd.sharding import gather_batch, scatter_batch, shard_bounds, shard_sizes


def test_shard_bounds_cover_exactly():
    for n in (0, 1, 7, 32, 256, 257):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (s0, e0), (s1, e1) in zip(spans, spans[1:]):
                assert e0 == s1
            sizes = shard_sizes(n, w)
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_bounds(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, T, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = torch.arange(n * 3 * T, dtype=torch.float32).view(n, 3, T) if rank == 0 else None
        shard = scatter_batch(full, n, (3, T), torch.device("cpu"))
        s, e = shard_bounds(n, world, rank)
        expect = torch.arange(n * 3 * T, dtype=torch.float32).view(n, 3, T)[s:e]
        ok_scatter = torch.equal(shard, expect)
        # per-utterance "vocoder": output length differs from the input (x256 like HiFiGAN)
        wav = shard.sum(1, keepdim=True).repeat_interleave(4, dim=2)
        out = gather_batch(wav, n)
        # a caller's non-contiguous `out` and an fp64 `full`: handled on the root,
        # without failing inside the collective
        full64 = full.double() if rank == 0 else None
        ok_scatter = ok_scatter and torch.equal(scatter_batch(full64, n, (3, T), torch.device("cpu")), expect)
        strided = torch.empty(n, 1, 8 * T).as_strided((n, 1, 4 * T), (8 * T, 8 * T, 2)) if rank == 0 else None
        out2 = gather_batch(wav, n, out=strided)
        if rank == 0:
            ref = torch.arange(n * 3 * T, dtype=torch.float32).view(n, 3, T).sum(1, keepdim=True).repeat_interleave(4, 2)
            q.put((rank, ok_scatter, torch.equal(out, ref) and out2 is strided and torch.equal(strided, ref)))
        else:
            q.put((rank, ok_scatter, out is None and out2 is None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 5), (2, 32), (3, 7)])
def test_scatter_gather_gloo(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, 6, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_s, ok_g in res:
        assert ok_s, f"rank {rank} scatter"
        assert ok_g, f"rank {rank} gather"
