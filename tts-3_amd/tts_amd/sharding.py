"""Utterance-batch sharding across the GPUs of one node (one process per GPU).

HiFiGAN is a pure per-utterance function, so a batch shards on its batch
axis with no exchange step: each rank vocodes its own contiguous slice with replicated
weights.  When the batch lives on one rank (a serving front end), ``scatter_batch`` /
``gather_batch`` move mel shards out and waveform shards back with torch.distributed
(RCCL over xGMI for the ``nccl`` backend, gloo on CPU), padding uneven shards to equal size.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous balanced split of n items: the first n % world ranks get one extra."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_sizes(n: int, world: int) -> List[int]:
    return [shard_bounds(n, world, r)[1] - shard_bounds(n, world, r)[0] for r in range(world)]


def scatter_batch(full: Optional[torch.Tensor], n: int, item_shape, device, src: int = 0,
                  dtype=torch.float32) -> torch.Tensor:
    """Rank ``src`` holds ``full`` [n, *item_shape]; every rank receives its shard."""
    world, rank = dist.get_world_size(), dist.get_rank()
    sizes = shard_sizes(n, world)
    cap = max(sizes)
    buf = torch.zeros(cap, *item_shape, device=device, dtype=dtype)
    chunks = None
    if rank == src:
        chunks = []
        for r in range(world):
            s, e = shard_bounds(n, world, r)
            c = torch.zeros(cap, *item_shape, device=device, dtype=dtype)
            c[: e - s] = full[s:e]
            chunks.append(c)
    dist.scatter(buf, chunks, src=src)
    return buf[: sizes[rank]]


def gather_batch(local: torch.Tensor, n: int, dst: int = 0) -> Optional[torch.Tensor]:
    """Inverse of scatter_batch: rank ``dst`` returns the full [n, ...] tensor, others None."""
    world, rank = dist.get_world_size(), dist.get_rank()
    sizes = shard_sizes(n, world)
    cap = max(sizes)
    buf = torch.zeros(cap, *local.shape[1:], device=local.device, dtype=local.dtype)
    buf[: local.shape[0]] = local
    outs = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, outs, dst=dst)
    if rank != dst:
        return None
    return torch.cat([o[:s] for o, s in zip(outs, sizes)], 0)
