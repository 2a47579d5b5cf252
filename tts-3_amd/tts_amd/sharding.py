"""Utterance-batch sharding across the GPUs of one node (one process per GPU).

HiFiGAN is a pure per-utterance function, so a batch shards on its batch
axis with no exchange step: each rank vocodes its own contiguous slice with replicated
weights.  When the batch lives on one rank (a serving front end), ``scatter_batch`` /
``gather_batch`` move mel shards out and waveform shards back with torch.distributed
(RCCL over xGMI for the ``nccl`` backend, gloo on CPU), padding uneven shards to equal size.

The reference has no inference collectives at all (its only distributed code is training:
``TTS/utils/distribute.py:13-20``; ``Synthesizer.tts`` vocodes one sentence at a time,
``TTS/utils/synthesizer.py:384-441``).  ``init_distributed`` adds the fail-fast behaviour SURVEY
§5 asks for: a bounded collective timeout and asynchronous RCCL error handling, so a dead or
hung peer tears the job down instead of hanging it.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def init_distributed(backend: str, local_rank: int, timeout_s: float = 300.0) -> None:
    """One process per GPU (or per CPU rank for gloo), rendezvous from the torchrun env
    (MASTER_ADDR / MASTER_PORT / RANK / WORLD_SIZE).

    Fail-fast: every collective times out after ``timeout_s``; with the nccl (RCCL) backend the
    process group's watchdog polls the communicator's asynchronous error state
    (ncclCommGetAsyncError) and aborts the communicator and the process on an error or a
    timeout (TORCH_NCCL_ASYNC_ERROR_HANDLING=1), so torchrun's agent then stops the other ranks.
    """
    timeout = datetime.timedelta(seconds=timeout_s)
    if backend == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this node type
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", timeout=timeout, device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend, timeout=timeout)


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous balanced split of n items: the first n % world ranks get one extra."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_sizes(n: int, world: int) -> List[int]:
    return [shard_bounds(n, world, r)[1] - shard_bounds(n, world, r)[0] for r in range(world)]


def _equal_views(t: torch.Tensor, world: int) -> Optional[List[torch.Tensor]]:
    """The world contiguous dim-0 slices of t when it splits evenly (no copy), else None."""
    if t is None or t.shape[0] == 0 or t.shape[0] % world or not t.is_contiguous():
        return None
    return list(t.split(t.shape[0] // world))


def scatter_batch(full: Optional[torch.Tensor], n: int, item_shape: Sequence[int], device, src: int = 0,
                  dtype=torch.float32, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Rank ``src`` holds ``full`` [n, *item_shape]; every rank receives its shard.

    ``out`` (optional, [max shard, *item_shape]) is the receive buffer, reused across calls.
    An evenly divisible contiguous ``full`` is sent as views (no staging copy)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    sizes = shard_sizes(n, world)
    cap = max(sizes)
    buf = out if out is not None else torch.empty(cap, *item_shape, device=device, dtype=dtype)
    if tuple(buf.shape) != (cap, *item_shape):
        raise ValueError(f"scatter_batch: out has shape {tuple(buf.shape)}, expected {(cap, *item_shape)}")
    chunks = None
    if rank == src:
        if tuple(full.shape) != (n, *item_shape):
            raise ValueError(f"scatter_batch: full has shape {tuple(full.shape)}, expected {(n, *item_shape)}")
        if full.dtype != buf.dtype or full.device != buf.device:
            # the collective needs send and receive buffers of one dtype on the communicator's device
            full = full.to(device=buf.device, dtype=buf.dtype)
        chunks = _equal_views(full, world)
        if chunks is None:
            chunks = []
            for r in range(world):
                s, e = shard_bounds(n, world, r)
                c = torch.zeros(cap, *item_shape, device=device, dtype=dtype)
                c[: e - s] = full[s:e]
                chunks.append(c)
    dist.scatter(buf, chunks, src=src)
    return buf[: sizes[rank]]


def gather_batch(local: torch.Tensor, n: int, dst: int = 0, out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """Inverse of scatter_batch: rank ``dst`` returns the full [n, ...] tensor, others None.

    ``out`` (optional, rank ``dst`` only, [n, ...] contiguous) receives the result in place when
    the shards are even (each peer's shard lands directly in its slice)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    sizes = shard_sizes(n, world)
    cap = max(sizes)
    if local.shape[0] != sizes[rank]:
        raise ValueError(f"gather_batch: rank {rank} holds {local.shape[0]} items, expected {sizes[rank]}")
    even = all(s == cap for s in sizes)
    buf = local if even and local.is_contiguous() else None
    if buf is None:
        buf = torch.zeros(cap, *local.shape[1:], device=local.device, dtype=local.dtype)
        buf[: local.shape[0]] = local
    if rank != dst:
        dist.gather(buf, None, dst=dst)
        return None
    if even:
        # receive straight into `out` only when it is exactly the full tensor's layout; otherwise
        # into a temporary (a bad `out` must not fail inside the collective after the peers have
        # entered it: they would wait for the timeout), copied into `out` afterwards
        direct = (out is not None and tuple(out.shape) == (n, *local.shape[1:]) and out.is_contiguous()
                  and out.dtype == local.dtype and out.device == local.device)
        full = out if direct else torch.empty(n, *local.shape[1:], device=local.device, dtype=local.dtype)
        dist.gather(buf, _equal_views(full, world), dst=dst)
        if out is not None and not direct:
            out.copy_(full)
            return out
        return full
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.gather(buf, outs, dst=dst)
    res = torch.cat([o[:s] for o, s in zip(outs, sizes)], 0)
    if out is not None:
        out.copy_(res)
        return out
    return res
