"""Multi-GPU sharding of a segment batch.

Segments are independent: the reference checksums each one on its own
(include/tcp-header.h:252-263, called per packet from socket-manager.cc:9-10 and
socket-manager.h:182), so a batch splits into contiguous index ranges, one per
GPU, with no exchange step -- no RCCL collective on the data path.  Each rank
owns its arena, descriptors and results; results concatenate by index.  The
only cross-rank traffic is the benchmark's barrier and the max-over-ranks of
the timed region.
"""
from __future__ import annotations

import numpy as np


def shard_range(count: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [start, stop) of `count` equal-size segments for `rank`
    (the first count % world ranks take one more)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    q, r = divmod(count, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def shard_by_bytes(lengths, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [start, stop) balanced by image bytes: rank r starts at the
    first segment whose byte prefix reaches r/world of the total (a 1492-B image
    is 15.5x a 96-B one, so counts would not balance a mixed batch)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    lengths = np.asarray(lengths, dtype=np.int64)
    pre = np.concatenate([[0], np.cumsum(lengths)])
    total = int(pre[-1])
    cut = lambda r: int(np.searchsorted(pre, (total * r) // world, side="left")) if r < world else lengths.size
    start = min(cut(rank), lengths.size)
    stop = min(cut(rank + 1), lengths.size)
    return start, max(start, stop)


def max_over_ranks(seconds: float, device=None) -> float:
    """Slowest rank's time (the job's time); identity without a process group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(seconds)
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_ranks(value: float, device=None) -> list[float]:
    """Every rank's `value`, in rank order (one all-reduce of a one-hot vector);
    [value] without a process group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(value)]
    t = torch.zeros(dist.get_world_size(), dtype=torch.float64, device=device)
    t[dist.get_rank()] = value
    dist.all_reduce(t)
    return [float(x) for x in t.cpu().tolist()]
