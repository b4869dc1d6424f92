"""Splitting rx work across GPUs.

Frames are independent, so a global batch splits into contiguous descriptor
ranges, one per rank, balanced by bytes (the kernel is HBM-bound, so bytes, not
frame counts, set each rank's time).  No data moves between ranks on the hot
path; the only collective is a small all-reduce of counters for reporting.
"""
from __future__ import annotations

import numpy as np


def shard_by_bytes(lens: np.ndarray, world: int) -> list:
    """Contiguous [lo, hi) frame ranges, one per rank, with ~equal sum(len)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    lens = np.asarray(lens, dtype=np.int64)
    n = lens.shape[0]
    if n == 0:
        return [(0, 0)] * world
    csum = np.cumsum(lens)
    total = int(csum[-1])
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        cuts.append(int(np.searchsorted(csum, target, side="left")) + 1)
    cuts.append(n)
    cuts = np.maximum.accumulate(np.minimum(np.asarray(cuts), n))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def counters(verdicts: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """[frames, bytes, drops, forwards] of one rank's batch (int64)."""
    v = np.asarray(verdicts)
    return np.array([v.shape[0], int(np.asarray(lens, dtype=np.int64).sum()),
                     int((v == -1).sum()), int((v >= 0).sum())], dtype=np.int64)


def allreduce_counters(dist, local: np.ndarray, device="cpu") -> np.ndarray:
    """Sum the counters of every rank (torch.distributed, any backend)."""
    import torch
    t = torch.as_tensor(local, dtype=torch.int64, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()
