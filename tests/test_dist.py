"""Multi-rank path on CPU (gloo, world size 2): byte-balanced contiguous shards
that partition the batch, per-rank checksumming by the oracle on each shard, and
the counter all-reduce bench.py does on RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from xsknf_amd import frames
from xsknf_amd.shard import allreduce_counters, counters, shard_by_bytes


def test_shard_by_bytes_partitions_and_balances():
    rng = np.random.default_rng(3)
    lens = frames.imix_lengths(1 << 16, rng)
    for world in (1, 2, 3, 4, 8):
        r = shard_by_bytes(lens, world)
        assert r[0][0] == 0 and r[-1][1] == lens.shape[0]
        assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
        sums = [int(lens[lo:hi].sum()) for lo, hi in r]
        assert max(sums) - min(sums) <= 2 * 1500
    assert shard_by_bytes(np.zeros(0), 4) == [(0, 0)] * 4
    assert shard_by_bytes(np.array([1500]), 3)[-1][1] == 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import csum_oracle as O
    b = frames.aligned_batch(2000, "imix", seed=11)
    lo, hi = shard_by_bytes(b.descs["len"], world)[rank]
    sub = frames.HostBatch(b.umem.copy(), np.ascontiguousarray(b.descs[lo:hi]), b.layout)
    v = O.c_process_batch(sub.umem, sub.descs)
    c = allreduce_counters(dist, counters(v, sub.descs["len"]))
    out[rank] = (lo, hi, c.tolist())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_shards_and_counters():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    b = frames.aligned_batch(2000, "imix", seed=11)
    ranges = sorted((out[r][0], out[r][1]) for r in range(world))
    assert ranges[0][0] == 0 and ranges[-1][1] == b.n and ranges[0][1] == ranges[1][0]
    total = out[0][2]
    assert total == out[1][2]
    assert total[0] == b.n and total[1] == int(b.descs["len"].astype(np.int64).sum())
    assert total[2] + total[3] == b.n


def _root_worker(rank, world, port, out, piece=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import csum_oracle as O
    from xsknf_amd import shard
    from xsknf_amd.shard import scatter_from_root
    if piece:
        shard.P2P_PIECE = piece      # several messages per span, as past 256 MiB on the GPU
    umem = descs = ranges = None
    if rank == 0:
        b = frames.unaligned_batch(3000, "imix", seed=21)
        frames.inject_edge_cases(b, 0.05, seed=22)
        umem, descs = torch.from_numpy(b.umem.copy()), b.descs
        ranges = shard_by_bytes(b.descs["len"], world)
    lu, ld, (b0, b1) = scatter_from_root(dist, umem, descs, ranges, rank, world, "cpu")
    u = lu.numpy().copy()
    d = ld.numpy().view(frames.DESC_DTYPE).reshape(-1).copy()
    v = O.c_process_batch(u, d)
    out[rank] = (b0, b1, u[:b1 - b0].tobytes(), v.tolist())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,piece", [(2, None), (3, None), (3, 4099)])
def test_root_scatter_shards_are_bit_exact(world, piece):
    """bench.py --root-scatter's distribution (collective 1) on
    gloo: every rank checksums the shard it received, and the bytes and
    verdicts equal the oracle's pass over the whole batch on the root; also
    with every span sent as many pieces (shard.P2P_PIECE, 256 MiB on the GPU)."""
    from oracle import csum_oracle as O
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_root_worker, args=(world, _free_port(), out, piece), nprocs=world, join=True)
    b = frames.unaligned_batch(3000, "imix", seed=21)
    frames.inject_edge_cases(b, 0.05, seed=22)
    ranges = shard_by_bytes(b.descs["len"], world)
    full = b.umem.copy()
    fv = O.c_process_batch(full, b.descs)
    for r in range(world):
        b0, b1, ub, v = out[r]
        lo, hi = ranges[r]
        assert v == fv[lo:hi].tolist(), f"rank {r} verdicts"
        assert ub == full[b0:b1].tobytes(), f"rank {r} bytes"


class _FakeDist:
    """Records what scatter_from_root asks of torch.distributed (one process)."""

    class P2POp:
        def __init__(self, op, tensor, peer):
            self.op, self.tensor, self.peer = op, tensor, peer

    def __init__(self, meta=None):
        self.meta = meta
        self.ops = []

    def isend(self, *a):
        pass

    def irecv(self, *a):
        pass

    def broadcast(self, t, src):
        if self.meta is not None:      # a non-root rank: the root's table arrives
            t.copy_(self.meta)

    def batch_isend_irecv(self, ops):
        self.ops = list(ops)
        return []


@pytest.mark.parametrize("world", [2, 3, 8])
def test_root_scatter_bookkeeping(world):
    """The offsets and shapes scatter_from_root hands the backend, independent of
    where the tensors live (bench.py runs it on HBM tensors over RCCL at N > 1):
    the root sends each peer a view of exactly its span and an (n, 2) int64
    descriptor tensor; a peer posts receives of the same sizes into a buffer
    with 16 spare bytes; the rebased descriptors address the span."""
    from xsknf_amd.shard import rebase_descs, scatter_from_root, shard_spans
    b = frames.unaligned_batch(5000, "imix", seed=41)
    frames.inject_edge_cases(b, 0.05, seed=42)
    umem = torch.from_numpy(b.umem.copy())
    ranges = shard_by_bytes(b.descs["len"], world)
    spans = shard_spans(b.descs, ranges, umem.numel())
    fd = _FakeDist()
    lu, ld, (b0, b1) = scatter_from_root(fd, umem, b.descs, ranges, 0, world, "cpu")
    assert (b0, b1) == spans[0] and lu.data_ptr() == umem.data_ptr() + spans[0][0]
    assert ld.shape == (ranges[0][1] - ranges[0][0], 2) and ld.dtype == torch.int64
    sends = [(o.peer, o.tensor) for o in fd.ops]
    assert [p for p, _ in sends] == [r for r in range(1, world) for _ in (0, 1)]
    for r in range(1, world):
        span_t, desc_t = [t for p, t in sends if p == r]
        (rb0, rb1), (lo, hi) = spans[r], ranges[r]
        assert span_t.data_ptr() == umem.data_ptr() + rb0 and span_t.numel() == rb1 - rb0
        want = rebase_descs(b.descs[lo:hi], rb0, umem.numel())
        assert np.array_equal(desc_t.numpy().view(frames.DESC_DTYPE).reshape(-1), want)
        # the peer's side: receives sized from the broadcast table
        meta = torch.tensor([[s0, s1, h - l] for (s0, s1), (l, h) in zip(spans, ranges)], dtype=torch.int64)
        fp = _FakeDist(meta)
        pu, pd, (p0, p1) = scatter_from_root(fp, None, None, None, r, world, "cpu")
        assert (p0, p1) == (rb0, rb1) and pu.numel() == rb1 - rb0 + 16 and pd.shape == (hi - lo, 2)
        assert [(o.peer, o.tensor.numel()) for o in fp.ops] == [(0, rb1 - rb0), (0, 2 * (hi - lo))]


# ---- the C host's shard arithmetic (xsknf_gpu_shard_plan / _rebase, xsknf_amd/csrc/multi.hip) ----

def _desc_cases():
    rng = np.random.default_rng(77)
    yield "imix-aligned", frames.aligned_batch(20000, "imix", seed=5)
    yield "jumbo-unaligned", frames.unaligned_batch(3000, 9000, seed=6)
    b = frames.unaligned_batch(5000, "imix", seed=7)
    frames.inject_edge_cases(b, 0.1, seed=8)          # short, non-IP, ... and odd lengths
    yield "imix-edges", b
    b = frames.aligned_batch(4000, rng.integers(0, 1792, size=4000).astype(np.uint32), seed=9)
    b.descs["len"][::97] = 0                          # zero-length frames
    yield "random-lens", b
    b = frames.aligned_batch(3000, "imix", seed=10)
    b.descs["addr"][::50] += np.uint64(1 << 40)       # descriptors outside the UMEM
    yield "out-of-range", b


@pytest.mark.parametrize("world", [1, 2, 3, 4, 7, 8, 64])
def test_c_shard_plan_equals_shard_py(world):
    """The C host's byte-balanced cuts and spans are shard.py's, frame for frame
    (the C multi-device path and the rank path split config 4 the same way)."""
    from xsknf_amd import multi
    from xsknf_amd.shard import rebase_descs, shard_spans
    for name, b in _desc_cases():
        ranges, spans = multi.shard_plan(b.descs, world, b.umem.size)
        assert ranges == shard_by_bytes(b.descs["len"], world), name
        assert spans == shard_spans(b.descs, ranges, b.umem.size), name
        for (lo, hi), (b0, _) in zip(ranges, spans):
            got = multi.shard_rebase(b.descs[lo:hi], b0, b.umem.size)
            want = rebase_descs(b.descs[lo:hi], b0, b.umem.size)
            assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), name


def test_c_shard_plan_edges():
    from xsknf_amd import multi
    empty = np.zeros(0, dtype=frames.DESC_DTYPE)
    assert multi.shard_plan(empty, 4, 0) == ([(0, 0)] * 4, [(0, 0)] * 4)
    one = frames.aligned_batch(1, 1500, seed=1)
    r, s = multi.shard_plan(one.descs, 3, one.umem.size)
    assert r == shard_by_bytes(one.descs["len"], 3) and r[-1] == (1, 1) and s[-1] == (0, 0)
    # config 4's global batch at its full size (8,388,608 IMIX frames), 8 ways
    lens = frames.imix_lengths(8 * (1 << 20), np.random.default_rng(frames.SEED))
    d = np.zeros(lens.shape[0], dtype=frames.DESC_DTYPE)
    d["len"] = lens
    d["addr"] = np.arange(lens.shape[0], dtype=np.uint64) * np.uint64(2048) + np.uint64(256)
    r, _ = multi.shard_plan(d, 8, lens.shape[0] * 2048)
    assert r == shard_by_bytes(lens, 8)


def _pack_plan_py(descs, bounds, umem_addr, umem_size):
    """The packed layout restated in numpy (include/xsknf_gpu.h
    xsknf_gpu_shard_pack_plan): each in-UMEM frame of a shard, in order, in a
    16-byte aligned slot of round16(r + len) bytes at address mod 16 = r, its
    address within the shard's buffer = the slot's start + r."""
    from xsknf_amd.shard import OUT_OF_RANGE, _in_umem, effective_offsets
    out = np.zeros_like(descs)
    out["len"], out["options"] = descs["len"], descs["options"]
    inr = _in_umem(descs, umem_size)
    r = ((np.uint64(umem_addr) + effective_offsets(descs).astype(np.uint64)) & np.uint64(15)).astype(np.int64)
    ln = descs["len"].astype(np.int64)
    slot = np.where(inr & (ln > 0), (r + ln + 15) // 16 * 16, 0)
    sizes = []
    for k in range(len(bounds) - 1):
        lo, hi = bounds[k], bounds[k + 1]
        start = np.concatenate([[0], np.cumsum(slot[lo:hi])[:-1]]) if hi > lo else np.zeros(0, np.int64)
        out["addr"][lo:hi] = np.where(inr[lo:hi], (start + r[lo:hi]).astype(np.uint64), np.uint64(OUT_OF_RANGE))
        sizes.append(int(slot[lo:hi].sum()))
    return out, sizes


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("umem_addr", [0x7f0000000000, 0x7f0000000007])
def test_c_pack_plan_equals_numpy(world, umem_addr):
    """The packed scatter's layout (xsknf_gpu_shard_pack_plan, the C multi-device
    path's frames-only distribution) equals its numpy restatement for every
    descriptor case: odd starts, edge-case lengths, zero lengths, descriptors
    outside the UMEM; every slot holds its frame, slots never overlap, and the
    packed bytes are at most the frames' bytes + 31 per frame."""
    from xsknf_amd import multi
    for name, b in _desc_cases():
        ranges, _ = multi.shard_plan(b.descs, world, b.umem.size)
        bounds = [lo for lo, _ in ranges] + [ranges[-1][1]]
        got, sizes = multi.pack_plan(b.descs, bounds, umem_addr, b.umem.size)
        want, wsizes = _pack_plan_py(b.descs, bounds, umem_addr, b.umem.size)
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), name
        assert sizes == wsizes, name
        for k, (lo, hi) in enumerate(ranges):
            a, ln = got["addr"][lo:hi].astype(np.int64), got["len"][lo:hi].astype(np.int64)
            live = got["addr"][lo:hi] < np.uint64(1 << 47)
            assert (a[live] + ln[live] <= sizes[k]).all(), name
            held = live & (ln > 0)                                   # (a zero-length frame has no bytes to hold)
            ends = a[held] + ln[held]
            assert (a[held][1:] >= ends[:-1]).all(), name            # in order, no overlap
            assert sizes[k] <= int(ln[live].sum()) + 31 * int(live.sum()), name
