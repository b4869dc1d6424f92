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


# ---- root distribution (collective 1) ------------------------
#
# When a global batch originates on one GPU (rank 0), the other ranks get
# their shards over xGMI before checksumming: each rank's frames occupy one
# contiguous byte span of the root's UMEM (contiguous descriptor ranges of a
# packed rx layout), so a shard moves as ONE point-to-point transfer of that
# span plus its descriptors, all ranks at once (batch_isend_irecv: the root's
# links run in parallel), not a ring collective.  This is not on the hot path
# (frames arrive per NIC queue, i.e. per worker, in the reference) and is
# measured separately (bench.py --root-scatter).

def effective_offsets(descs) -> np.ndarray:
    """UMEM byte offset of every frame (aligned or unaligned-mode addresses, as
    xsk_umem__add_offset_to_addr() translates them, src/xsknf.c:659)."""
    a = np.asarray(descs["addr"], dtype=np.uint64)
    return ((a & np.uint64((1 << 48) - 1)) + (a >> np.uint64(48))).astype(np.int64)


def _in_umem(descs, umem_size: int) -> np.ndarray:
    offs = effective_offsets(descs)
    return (offs <= umem_size) & (np.asarray(descs["len"], dtype=np.int64) <= umem_size - offs)


def shard_spans(descs, ranges, umem_size: int) -> list:
    """(b0, b1): the byte span of the UMEM holding each rank's frames
    (descriptors outside the UMEM hold no bytes)."""
    offs = effective_offsets(descs)
    ends = offs + np.asarray(descs["len"], dtype=np.int64)
    ok = _in_umem(descs, umem_size)
    out = []
    for lo, hi in ranges:
        m = ok[lo:hi]
        out.append((int(offs[lo:hi][m].min()), int(ends[lo:hi][m].max())) if m.any() else (0, 0))
    return out


OUT_OF_RANGE = np.uint64(1 << 47)   # an address past any UMEM: the frame is dropped untouched


def rebase_descs(descs, b0: int, umem_size: int) -> np.ndarray:
    """The same frames as plain (offset-free) addresses relative to byte b0;
    a descriptor outside the UMEM stays outside it (verdict -1, no bytes)."""
    from .frames import DESC_DTYPE
    out = np.zeros(len(descs), dtype=DESC_DTYPE)
    rel = (effective_offsets(descs) - b0).astype(np.uint64)
    out["addr"] = np.where(_in_umem(descs, umem_size), rel, OUT_OF_RANGE)
    out["len"] = descs["len"]
    out["options"] = descs["options"]
    return out


# Bytes per point-to-point message of the root distribution: one RCCL send of
# more than 1 GiB delivered only part of its bytes on this image (the C host's
# scatter, xsknf_amd/csrc/multi.hip kP2PPiece; profiles/r06/multi_p2p_pieces.jsonl),
# so spans go in 256 MiB pieces (matched send for send on both sides).
P2P_PIECE = 1 << 28


def scatter_from_root(dist, umem, descs, ranges, rank: int, world: int, device, root: int = 0):
    """Move every rank's shard from the root.  On the root: `umem` is the whole
    UMEM (uint8 tensor on `device`), `descs` the whole descriptor array
    (frames.DESC_DTYPE, host), `ranges` from shard_by_bytes(); elsewhere they
    are ignored.  Returns (local umem tensor, local descs as an (n, 2) int64
    tensor of xdp_desc bytes, (b0, b1)).  The root's own shard is a view."""
    import torch
    meta = torch.zeros((world, 3), dtype=torch.int64, device=device)
    spans = None
    if rank == root:
        spans = shard_spans(descs, ranges, umem.numel())
        meta.copy_(torch.tensor([[b0, b1, hi - lo] for (b0, b1), (lo, hi) in zip(spans, ranges)],
                                dtype=torch.int64))
    dist.broadcast(meta, src=root)
    b0, b1, n = (int(x) for x in meta[rank].tolist())
    ops = []
    if rank == root:
        for r in range(world):
            lo, hi = ranges[r]
            rb0, rb1 = spans[r]
            d = rebase_descs(descs[lo:hi], rb0, umem.numel())
            d = torch.from_numpy(d.view(np.int64).reshape(-1, 2).copy()).to(device)
            if r == root:
                local = (umem[rb0:rb1], d)
            else:
                for o in range(rb0, rb1, P2P_PIECE):
                    ops.append(dist.P2POp(dist.isend, umem[o:min(o + P2P_PIECE, rb1)].contiguous(), r))
                ops.append(dist.P2POp(dist.isend, d, r))
    else:
        # 16 spare bytes: the kernel's 16-byte chunk loads may end past the span
        buf = torch.empty(b1 - b0 + 16, dtype=torch.uint8, device=device)
        d = torch.empty((n, 2), dtype=torch.int64, device=device)
        for o in range(0, b1 - b0, P2P_PIECE):
            ops.append(dist.P2POp(dist.irecv, buf[o:min(o + P2P_PIECE, b1 - b0)], root))
        ops.append(dist.P2POp(dist.irecv, d, root))
        local = (buf, d)
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return local[0], local[1], (b0, b1)
