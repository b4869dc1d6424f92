"""Parity of the gfx950 batch path (through the C ABI) against the CPU oracle.

Bar: bit-exact -- every verdict and every UMEM byte (the kernel may change only
the two UDP check bytes of frames that reach checksummer_user.c:108).
Small seeded batches cover every branch of checksummer_user.c:30-112; the
BASELINE configs run at full size (1M frames) against the threaded C oracle.
"""
import os
import sys

import numpy as np
import pytest

from oracle import csum_oracle as O
from tests import oracles
from xsknf_amd import Checksummer, ChecksummerOptions, frames

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _pool_guard_never_trips():
    """Every launch of this module, and of the modules before it: no wave of the
    pooled split kernel found a unit of its block unclaimed (the device counter
    behind xsknf_gpu_pool_guard_trips; ADVICE r05: the grid bound is the only
    thing that keeps a pooled block's units inside its patch lists)."""
    yield
    from xsknf_amd import _lib
    assert _lib.pool_guard_trips() == 0


def _results(*tensors):
    """The launch's outputs on the host BEFORE any CPU oracle work: a fault in
    the launch is then reported here, inside the test that made it (HIP reports
    a GPU memory fault asynchronously, from its event thread; with the 16
    oracle threads on every CPU of the box it surfaced only at the next HIP call
    after the oracle -- DESIGN 3, the round-2 fault)."""
    import time
    torch.cuda.synchronize()
    # a second synchronize after a pause, with no new GPU work in between: a
    # fault reported here came from work already done (the launch), one
    # reported only at the copies below would implicate the copies
    time.sleep(0.05)
    torch.cuda.synchronize()
    return tuple(t.cpu().numpy() for t in tensors)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def run_gpu(b: frames.HostBatch, dev, *, ingress=0, iters=1, action=O.REDIRECT, nif=1, hint=0):
    cs = Checksummer(ChecksummerOptions(action=action, csum_iterations=iters), num_interfaces=nif,
                     frame_len_hint=hint)
    umem = torch.from_numpy(b.umem).to(dev)
    descs = torch.from_numpy(b.descs.view(np.uint8).reshape(-1, 16).copy()).to(dev)
    v = cs.process_batch(umem, descs, ingress_ifindex=ingress)
    torch.cuda.synchronize()
    return umem.cpu().numpy(), v.cpu().numpy()


def run_oracle(b: frames.HostBatch, *, ingress=0, iters=1, action=O.REDIRECT, nif=1):
    r = b.copy()
    v = O.c_process_batch(r.umem, r.descs, ingress=ingress, iters=iters, action=action, nif=nif)
    return r.umem, v


def assert_parity(b, dev, **kw):
    hint = kw.pop("hint", 0)
    gu, gv = run_gpu(b, dev, hint=hint, **kw)
    ou, ov = run_oracle(b, **kw)
    bad = np.nonzero(gv != ov)[0]
    assert bad.size == 0, f"verdict mismatch at {bad[:10]}: gpu {gv[bad[:10]]} oracle {ov[bad[:10]]}"
    if not np.array_equal(gu, ou):
        diff = np.nonzero(gu != ou)[0]
        raise AssertionError(f"{diff.size} UMEM bytes differ, first at {diff[:10]}")
    return gv


def test_known_answers_through_gpu(dev):
    from tests.test_oracle import KATS
    for name, frame, kw, ret, sl, chk in KATS:
        n = len(frame)
        for rs in (0, 1, 5, 15):     # every 16-byte phase class incl. odd starts
            umem = np.zeros(((rs + n + 255) // 256 + 1) * 256, dtype=np.uint8)
            umem[256 + rs:256 + rs + n] = np.frombuffer(bytes(frame), dtype=np.uint8)
            d = np.zeros(1, dtype=frames.DESC_DTYPE)
            d["addr"], d["len"] = 256 + rs, n
            b = frames.HostBatch(umem, d, "aligned")
            gu, gv = run_gpu(b, dev, **kw)
            assert gv[0] == ret, name
            if chk is not None:
                got = bytes(gu[256 + rs + sl[0]:256 + rs + sl[1]]).hex()
                assert got == chk, f"{name} rs={rs}"


@pytest.mark.parametrize("length", [60, 64, 65, 570, 1500, 1501, 4000, 9000, "imix"])
@pytest.mark.parametrize("layout", ["aligned", "unaligned"])
def test_seeded_batches_with_edge_cases(dev, length, layout):
    n = 3000
    if layout == "aligned":
        chunk = 2048 if length == "imix" or length <= 1792 else 16384
        b = frames.aligned_batch(n, length, chunk=chunk)
    else:
        b = frames.unaligned_batch(n, length)
    frames.inject_edge_cases(b, 0.05)
    assert_parity(b, dev, iters=1, action=O.REDIRECT, nif=1)


@pytest.mark.parametrize("iters,action,nif,ingress", [
    (1, O.DROP, 1, 0), (0, O.REDIRECT, 1, 0), (-3, O.REDIRECT, 2, 1), (2, O.REDIRECT, 3, 2),
    (10, O.DROP, 1, 0), (50, O.REDIRECT, 4, 3), (7919, O.DROP, 1, 0)])
def test_options(dev, iters, action, nif, ingress):
    b = frames.unaligned_batch(2000, "imix", seed=iters & 0xFFFF)
    frames.inject_edge_cases(b, 0.1)
    assert_parity(b, dev, iters=iters, action=action, nif=nif, ingress=ingress)


@pytest.mark.parametrize("hint", [1, 64, 100, 500, 1500, 4000, 9000, 60000])
def test_frame_len_hint_is_only_a_hint(dev, hint):
    """Every size class must handle every length (multi-pass loop, idle lanes)."""
    rng = np.random.default_rng(hint)
    lens = rng.integers(0, 12000, size=1500).astype(np.uint32)
    b = frames.unaligned_batch(1500, lens, seed=hint)
    frames.inject_edge_cases(b, 0.05)
    assert_parity(b, dev, hint=hint, iters=3)


def test_empty_and_tiny_batches(dev):
    cs = Checksummer()
    umem = torch.zeros(4096, dtype=torch.uint8, device=dev)
    descs = torch.zeros((0, 2), dtype=torch.int64, device=dev)
    v = cs.process_batch(umem, descs)
    assert v.numel() == 0
    for n in (1, 2, 3, 17, 63, 64, 65, 257):
        b = frames.aligned_batch(n, 64, chunk=2048, seed=n)
        assert_parity(b, dev)


def test_out_of_range_descriptors_are_dropped_untouched(dev):
    b = frames.aligned_batch(64, 1500, chunk=2048)
    size = b.umem.size
    b.descs["addr"][3] = size - 10          # runs off the end
    b.descs["addr"][7] = size + 4096        # starts past the end
    b.descs["addr"][9] = (np.uint64(size - 100)) | (np.uint64(200) << np.uint64(48))
    gu, gv = run_gpu(b, dev)
    for i in (3, 7, 9):
        assert gv[i] == -1
    keep = np.ones(64, bool)
    keep[[3, 7, 9]] = False
    good = frames.HostBatch(b.umem.copy(), b.descs[keep].copy(), "aligned")
    ou, ov = run_oracle(good)
    assert np.array_equal(gv[keep], ov)
    assert np.array_equal(gu, ou)


@pytest.mark.parametrize("hint", [0, 64, 1500, 9000])
def test_frames_ending_at_the_umem_end(dev, hint):
    """A UMEM whose size is not a multiple of 16 and whose last frames end on
    its last byte (odd starts): the 16-byte chunk loads may not change any
    result there; a frame one byte too long is dropped untouched."""
    rng = np.random.default_rng(hint + 5)
    lens = rng.integers(14, 2000, size=300).astype(np.uint32)
    lens[-4:] = (60, 7, 33, 1501)
    b = frames.unaligned_batch(300, lens, seed=hint + 5)
    frames.inject_edge_cases(b, 0.05, seed=hint + 6)
    addr = b.descs["addr"]
    offs = (addr & np.uint64((1 << 48) - 1)) + (addr >> np.uint64(48))
    end = int((offs + b.descs["len"]).max())
    last = int(np.argmax(offs + b.descs["len"]))
    t = frames.HostBatch(b.umem[:end].copy(), b.descs.copy(), "unaligned")
    assert_parity(t, dev, hint=hint, iters=2)
    over = frames.HostBatch(b.umem[:end].copy(), b.descs.copy(), "unaligned")
    over.descs["len"][last] += 1                     # one byte past the UMEM
    gu, gv = run_gpu(over, dev, hint=hint)
    assert gv[last] == -1
    keep = np.ones(over.n, bool)
    keep[last] = False
    ou, ov = run_oracle(frames.HostBatch(over.umem.copy(), over.descs[keep].copy(), "unaligned"))
    assert np.array_equal(gv[keep], ov)
    assert np.array_equal(gu, ou)


def test_reprocessing(dev):
    """A second pass over processed frames matches the oracle run on them, and on
    well-formed frames (ihl 5) it changes nothing: the check is cleared before
    summing.  (With ihl 2 or 3 the UDP check overlaps the IP addresses the
    pseudo-header reads, so there the second pass legitimately differs.)"""
    b = frames.unaligned_batch(5000, "imix")
    frames.inject_edge_cases(b, 0.05)
    gu, gv = run_gpu(b, dev)
    b2 = frames.HostBatch(gu.copy(), b.descs.copy(), b.layout)
    assert_parity(b2, dev)
    clean = frames.unaligned_batch(5000, "imix", seed=99)
    cu, cv = run_gpu(clean, dev)
    cu2, cv2 = run_gpu(frames.HostBatch(cu.copy(), clean.descs.copy(), clean.layout), dev)
    assert np.array_equal(cu, cu2) and np.array_equal(cv, cv2)


FULL = [
    ("64B-aligned", 1 << 20, 64, "aligned"),
    ("1500B-aligned", 1 << 20, 1500, "aligned"),
    ("imix-aligned", 1 << 20, "imix", "aligned"),
    ("9000B-unaligned", 1 << 20, 9000, "unaligned"),
]


@pytest.mark.slow
@pytest.mark.parametrize("name,n,length,layout", FULL, ids=[f[0] for f in FULL])
def test_full_size_configs_bit_exact(dev, name, n, length, layout):
    """BASELINE configs 2-5 at full size with 1 % edge cases mixed in (SURVEY.md
    8(d) row 2: non-IP, non-UDP, every ihl, truncated, odd lengths, ...), every
    verdict and byte compared with the oracle; then every well-formed frame's
    written check passes the RFC 768/1071 receive-side verification
    (tests/rfc1071.py), except the single-fold carry losses, which are off by
    exactly one."""
    from tests import rfc1071
    umem, descs, lens = frames.device_batch(n, length, layout=layout, device=dev)
    host_in = umem.cpu().numpy()
    host_descs = descs.cpu().numpy().view(frames.DESC_DTYPE).reshape(-1).copy()
    b = frames.HostBatch(host_in, host_descs, layout)
    edge = frames.inject_edge_cases(b, 0.01, seed=n + len(name))
    umem.copy_(torch.from_numpy(host_in))
    descs.copy_(torch.from_numpy(host_descs.view(np.int64).reshape(n, 2)))
    # the shape the bench runs: longest frame and mean length (xsknf_gpu_checksum_batch_lens)
    hint, mean = int(lens.max()), int(lens.mean())
    v = Checksummer(frame_len_hint=hint, frame_len_mean=mean).process_batch(umem, descs)
    gv, gu = _results(v, umem)
    _, ov = oracles.time_batch(host_in, host_descs)
    assert np.array_equal(gv, ov)
    assert np.array_equal(gu, host_in)
    # the clean frames are valid UDP frames: REDIRECT to iface 0
    clean = np.ones(n, bool)
    clean[edge] = False
    assert (gv[clean] == 0).all() and (gv[edge] != 0).any()
    # RFC receive-side check of what the GPU wrote, on every well-formed frame
    idx, V = rfc1071.verify(umem, b.frame_offsets().astype(np.int64), host_descs["len"])
    assert idx.size > 0.98 * n
    lost = V == 0x0001
    assert np.all((V == 0xFFFF) | lost)
    assert lost.mean() < {64: 0.001, 1500: 0.01, 9000: 0.05}.get(length, 0.01)


@pytest.mark.slow
@pytest.mark.parametrize("n,layout", [((2 << 20) + 4097, "aligned"), ((17 << 20) + 5, "unaligned")],
                         ids=["2M-aligned", "17M-packed"])
def test_lane_kernel_large_batches(dev, n, layout):
    """64 B frames: the lane kernel takes up to 16M frames in one launch (run()
    in checksummer.hip), so a 2M-frame batch is one launch whose waves take
    several times the tiles of a 1M-frame one, and a 17M-frame batch is a 16M
    launch plus a short one; every verdict and byte equal to the oracle's (the
    aligned batch through the write-through sector stores, the packed one
    through the non-temporal ones)."""
    umem, descs, lens = frames.device_batch(n, 64, layout=layout, device=dev, seed=79)
    host = umem.cpu().numpy()
    hd = descs.cpu().numpy().view(frames.DESC_DTYPE).reshape(-1).copy()
    frames.inject_edge_cases(frames.HostBatch(host, hd, layout), 0.01, seed=80)
    umem.copy_(torch.from_numpy(host))
    descs.copy_(torch.from_numpy(hd.view(np.int64).reshape(n, 2)))
    v = Checksummer(frame_len_hint=64).process_batch(umem, descs)
    gv, gu = _results(v, umem)
    _, ov = oracles.time_batch(host, hd)
    assert np.array_equal(gv, ov)
    assert np.array_equal(gu, host)


@pytest.mark.slow
@pytest.mark.parametrize("length", [1500, "imix"])
def test_batch_larger_than_one_launch(dev, length):
    """A batch of more than 1M frames runs as consecutive launches (run() in
    checksummer.hip): the deferred checks, record counters and verdicts of each
    launch land on their own frames."""
    n = (1 << 20) + 4097
    umem, descs, lens = frames.device_batch(n, length, layout="aligned", device=dev, seed=77)
    host = umem.cpu().numpy()
    hd = descs.cpu().numpy().view(frames.DESC_DTYPE).reshape(-1).copy()
    frames.inject_edge_cases(frames.HostBatch(host, hd, "aligned"), 0.01, seed=78)
    umem.copy_(torch.from_numpy(host))
    descs.copy_(torch.from_numpy(hd.view(np.int64).reshape(n, 2)))
    v = Checksummer(frame_len_hint=int(lens.max())).process_batch(umem, descs)
    gv, gu = _results(v, umem)
    _, ov = oracles.time_batch(host, hd)
    assert np.array_equal(gv, ov)
    assert np.array_equal(gu, host)


# lanes_per_frame, chunks_per_lane, frames_per_group, lds_ring, fused_stores[, kernel, window]
PRODUCT_SHAPES = [
    # the split kernel shapes of default_cfg() under every store mode
    # (0 per tile, 1 in-line, 2 deferred, +4 2-byte, +8 plain sectors, +16 tail scatter)
    (16, 2, 2, 0, 0, 1, 20), (16, 2, 2, 0, 1, 1, 20), (16, 2, 2, 0, 9, 1, 20), (16, 2, 2, 0, 5, 1, 20),
    (16, 2, 2, 0, 0, 1, 24), (16, 2, 2, 0, 1, 1, 24), (16, 2, 2, 0, 2, 1, 24), (16, 2, 2, 0, 18, 1, 24),
    (16, 3, 1, 0, 0, 1, 24), (16, 3, 1, 0, 1, 1, 24), (16, 3, 1, 0, 2, 1, 24), (16, 3, 1, 0, 16, 1, 24),
    (16, 3, 1, 0, 18, 1, 24), (16, 3, 1, 0, 4, 1, 24),
    (16, 3, 2, 0, 0, 1, 20), (16, 3, 2, 0, 2, 1, 20), (16, 3, 2, 0, 20, 1, 20), (16, 3, 2, 0, 1, 1, 20),
    # one 12-wave block per CU sharing the CU's tiles (window + 32)
    (16, 2, 2, 0, 18, 1, 56), (16, 2, 2, 0, 2, 1, 56), (16, 2, 2, 0, 0, 1, 56), (16, 2, 2, 0, 1, 1, 56),
    # jumbo: one 8-wave block per CU sharing the CU's tiles, 16-frame quarters at the end
    (16, 3, 2, 0, 0, 1, 52), (16, 3, 2, 0, 1, 1, 52), (16, 3, 2, 0, 2, 1, 52), (16, 3, 2, 0, 18, 1, 52),
    # the lane kernel (short frames) under every store mode
    (1, 5, 2, 0, 1), (1, 5, 2, 0, 9), (1, 5, 2, 0, 5), (1, 5, 2, 0, 2), (1, 5, 2, 0, 0),
    # ... and its default since round 5: windows transposed where a tile's frames lie apart (window field 1024)
    (1, 5, 2, 0, 1, 0, 1024), (1, 5, 2, 0, 9, 0, 1024), (1, 5, 2, 0, 5, 0, 1024), (1, 5, 2, 0, 2, 0, 1024),
    (1, 5, 2, 0, 0, 0, 1024),
    # the zero-copy host path's small-batch group shapes
    (32, 3, 2, 0, 0), (32, 3, 2, 0, 1), (32, 3, 2, 0, 5), (64, 2, 4, 0, 2), (64, 2, 4, 0, 1),
]
# every other family / shape: only in the A/B build (`make ab`, XSKNF_GPU_LIB=build/ab/libxsknf_gpu.so)
AB_SHAPES = [
    (8, 1, 2, 0, 0), (8, 1, 8, 0, 1), (16, 2, 4, 0, 2), (32, 3, 4, 0, 1),
    (64, 9, 2, 0, 2), (64, 2, 8, 0, 0),
    (4, 2, 4, 0, 1), (4, 2, 2, 0, 0), (4, 2, 4, 0, 5),
    (1, 5, 4, 0, 0), (1, 6, 2, 0, 9), (1, 7, 2, 0, 5),
    (8, 1, 4, 0, 5), (16, 2, 4, 0, 4), (32, 3, 4, 0, 5),
    (16, 2, 2, 0, 0, 1, 4), (16, 2, 1, 0, 1, 1, 4), (8, 4, 2, 0, 2, 1, 4), (32, 1, 2, 0, 5, 1, 4),
    (16, 4, 1, 0, 4, 1, 4), (16, 2, 2, 0, 0, 1, 5), (64, 2, 1, 0, 0, 1, 4), (32, 2, 1, 0, 1, 1, 4),
    (16, 2, 1, 0, 0, 1, 7), (16, 3, 1, 0, 2, 1, 4), (8, 2, 2, 0, 1, 1, 4),
    (16, 2, 1, 0, 5, 1, 20), (16, 3, 1, 0, 1, 1, 20), (16, 2, 1, 0, 1, 1, 24), (32, 3, 1, 0, 2, 1, 24),
    # 16 x 3 items with the 8-tile patch list (long-frame batches, not in the product)
    (16, 3, 2, 0, 18, 1, 24), (16, 3, 2, 0, 2, 1, 24), (16, 3, 2, 0, 0, 1, 24), (16, 3, 2, 0, 1, 1, 24),
    # the lane kernel with one 16-wave block per CU sharing the CU's tiles (window field 32), 128- and
    # 64-frame units
    (1, 5, 2, 0, 1, 0, 32), (1, 5, 2, 0, 9, 0, 32), (1, 5, 2, 0, 2, 0, 32), (1, 5, 2, 0, 0, 0, 32),
    (1, 5, 1, 0, 1, 0, 32), (1, 5, 1, 0, 2, 0, 32),
]
AB_BUILD = "ab" in os.path.basename(os.path.dirname(os.environ.get("XSKNF_GPU_LIB", "")))
SHAPES = PRODUCT_SHAPES + [pytest.param(s, marks=pytest.mark.skipif(not AB_BUILD, reason="A/B build only"))
                           for s in AB_SHAPES]


def _shape_id(s):
    s = s.values[0] if hasattr(s, "values") else s
    return "-".join(map(str, s))


def launch_cfg(shape, bpc=4, fused=None):
    from xsknf_amd import _lib
    kernel, window = (shape[5], shape[6]) if len(shape) > 5 else (0, 0)
    return _lib.LaunchCfg(shape[0], shape[1], shape[2], bpc, shape[3], shape[4] if fused is None else fused,
                          kernel, window)


@pytest.mark.parametrize("shape", SHAPES, ids=[_shape_id(s) for s in SHAPES])
@pytest.mark.parametrize("layout", ["aligned", "unaligned"])
def test_every_launch_shape_is_bit_exact(dev, shape, layout):
    """Each kernel family / shape / store mode, through xsknf_gpu_checksum_batch_cfg."""
    import ctypes
    from xsknf_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(sum(shape))
    lens = rng.integers(0, 3000, size=2500).astype(np.uint32)
    if layout == "aligned":
        b = frames.aligned_batch(2500, np.minimum(lens, 1792), chunk=2048, seed=sum(shape))
    else:
        b = frames.unaligned_batch(2500, lens, seed=sum(shape))
    frames.inject_edge_cases(b, 0.1)
    ou, ov = run_oracle(b, iters=2, action=O.REDIRECT, nif=3, ingress=1)
    umem = torch.from_numpy(b.umem).to(dev)
    descs = torch.from_numpy(b.descs.view(np.uint8).reshape(-1, 16).copy()).to(dev)
    v = torch.empty(b.n, dtype=torch.int32, device=dev)
    cfg = launch_cfg(shape)
    rc = lib.xsknf_gpu_checksum_batch_cfg(
        ctypes.c_void_p(umem.data_ptr()), umem.numel(), ctypes.c_void_p(descs.data_ptr()), b.n, 1,
        ctypes.byref(_lib.CsumOpts(2, O.REDIRECT, 3, 0)), ctypes.c_void_p(v.data_ptr()),
        ctypes.byref(cfg), None)
    assert rc == 0
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy(), ov)
    assert np.array_equal(umem.cpu().numpy(), ou)


def _nic_batch(seed, layout, n=2500):
    """Mixed lengths with the UDP checksums a NIC offload writes
    (tests/gen-traffic.lua:120), then 5 % edge cases."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 3000, size=n).astype(np.uint32)
    if layout == "aligned":
        b = frames.aligned_batch(n, np.minimum(lens, 1792), chunk=2048, seed=seed)
    else:
        b = frames.unaligned_batch(n, lens, seed=seed)
    frames.offload_checks_host(b)
    frames.inject_edge_cases(b, 0.05, seed=seed + 1)
    return b


@pytest.mark.parametrize("shape", SHAPES, ids=[_shape_id(s) for s in SHAPES])
@pytest.mark.parametrize("store_unchanged", [False, True], ids=["elide", "store32"])
def test_nic_offloaded_checks_every_shape(dev, shape, store_unchanged):
    """Frames whose UDP checksums a NIC already filled in: the checksummer
    computes the value each frame holds for all but its carry-loss frames, and
    every shape leaves those frames untouched (or rewrites the same bytes with
    fused_stores + 32): every verdict and byte equal to the oracle's."""
    import ctypes
    from xsknf_amd import _lib
    lib = _lib.load()
    b = _nic_batch(sum(shape) + 7, "unaligned" if sum(shape) & 1 else "aligned")
    ou, ov = run_oracle(b, iters=1, action=O.REDIRECT, nif=3, ingress=1)
    umem = torch.from_numpy(b.umem).to(dev)
    descs = torch.from_numpy(b.descs.view(np.uint8).reshape(-1, 16).copy()).to(dev)
    v = torch.empty(b.n, dtype=torch.int32, device=dev)
    cfg = launch_cfg(shape)
    if store_unchanged:
        cfg.fused_stores += 32
    rc = lib.xsknf_gpu_checksum_batch_cfg(
        ctypes.c_void_p(umem.data_ptr()), umem.numel(), ctypes.c_void_p(descs.data_ptr()), b.n, 1,
        ctypes.byref(_lib.CsumOpts(1, O.REDIRECT, 3, 0)), ctypes.c_void_p(v.data_ptr()),
        ctypes.byref(cfg), None)
    assert rc == 0
    gv, gu = _results(v, umem)
    assert np.array_equal(gv, ov)
    assert np.array_equal(gu, ou)


@pytest.mark.parametrize("shape", [(1, 5, 2, 0), (32, 3, 2, 0), (16, 2, 2, 0, 0, 1, 24), (16, 2, 2, 0, 0, 1, 56),
                                   (16, 3, 2, 0, 0, 1, 52)],
                         ids=["lane", "reg32", "split-w8", "split-pool", "split-w4-pool"])
def test_records_mark_exactly_the_changed_checks(dev, shape):
    """Records-only mode over NIC-checksummed frames: a frame gets a record
    exactly when the oracle changes its check bytes (the carry-loss frames,
    the edge cases with odd headers); every other frame carries its verdict.
    So the kernels elide exactly the writes that would not change a byte."""
    import ctypes
    from xsknf_amd import _lib
    lib = _lib.load()
    b = _nic_batch(91, "unaligned", n=20000)
    ou, ov = run_oracle(b, iters=1, action=O.REDIRECT, nif=1)
    offs = b.frame_offsets().astype(np.int64)
    lens = b.descs["len"].astype(np.int64)
    umem = torch.from_numpy(b.umem).to(dev)
    descs = torch.from_numpy(b.descs.view(np.uint8).reshape(-1, 16).copy()).to(dev)
    v = torch.empty(b.n, dtype=torch.int32, device=dev)
    cfg = launch_cfg(shape, fused=3)
    assert lib.xsknf_gpu_checksum_batch_cfg(
        ctypes.c_void_p(umem.data_ptr()), umem.numel(), ctypes.c_void_p(descs.data_ptr()), b.n, 0,
        ctypes.byref(_lib.CsumOpts(1, O.REDIRECT, 1, 0)), ctypes.c_void_p(v.data_ptr()),
        ctypes.byref(cfg), None) == 0
    gv, gu = _results(v, umem)
    assert np.array_equal(gu, b.umem)
    rec = gv.view(np.uint32)
    tagged = (rec & 0xC0000000) == 0x40000000
    changed = np.zeros(b.n, bool)
    for i in np.flatnonzero(ov >= 0):          # summed frames: their check is at u + 6
        u = 14 + 4 * (int(b.umem[offs[i] + 14]) & 0x0F)
        at = int(offs[i]) + u + 6
        if at + 2 <= offs[i] + lens[i]:
            changed[i] = not np.array_equal(ou[at:at + 2], b.umem[at:at + 2])
    assert np.array_equal(tagged, changed)
    assert 0 < tagged.sum() < 0.1 * b.n
    assert np.array_equal(np.where(tagged, 0, gv), np.where(tagged, 0, ov))


@pytest.mark.slow
@pytest.mark.parametrize("length,layout", [(1500, "aligned"), ("imix", "aligned"), (64, "aligned"),
                                           (9000, "unaligned")])
def test_full_size_nic_offloaded_bit_exact(dev, length, layout):
    """The bench's NIC-checksum workloads at full size (1M frames, 1 % edge
    cases): bit-exact with the oracle; the oracle changes the checks of < 5 %
    of the frames (carry losses and edge cases), the rest stay as they were."""
    n = 1 << 20
    umem, descs, lens = frames.device_batch(n, length, layout=layout, device=dev, seed=123)
    frames.offload_checks_device(umem, descs)
    host_in = umem.cpu().numpy()
    hd = descs.cpu().numpy().view(frames.DESC_DTYPE).reshape(-1).copy()
    frames.inject_edge_cases(frames.HostBatch(host_in, hd, layout), 0.01, seed=124)
    umem.copy_(torch.from_numpy(host_in))
    descs.copy_(torch.from_numpy(hd.view(np.int64).reshape(n, 2)))
    before = host_in.copy()
    v = Checksummer(frame_len_hint=int(lens.max()), frame_len_mean=int(lens.mean())).process_batch(umem, descs)
    gv, gu = _results(v, umem)
    _, ov = oracles.time_batch(host_in, hd)
    assert np.array_equal(gv, ov)
    assert np.array_equal(gu, host_in)
    offs = frames.HostBatch(before, hd, layout).frame_offsets().astype(np.int64)
    at = offs[(hd["len"] >= 42)] + 40
    assert (gu[at] != before[at]).mean() < 0.05


@pytest.mark.parametrize("shape", [(32, 3, 2, 0), (64, 2, 4, 0), (16, 3, 1, 0, 0, 1, 24), (16, 2, 2, 0, 0, 1, 20),
                                   (16, 2, 2, 0, 0, 1, 56), (16, 3, 2, 0, 0, 1, 52)],
                         ids=["reg32", "reg64", "split-w8", "split-w4", "split-pool", "split-w4-pool"])
def test_records_only_mode(dev, shape):
    """fused_stores = 3: the UMEM is only read; applying the records as
    include/xsknf_gpu.h documents them gives the oracle's bytes and verdicts."""
    import ctypes
    from xsknf_amd import _lib
    lib = _lib.load()
    b = frames.unaligned_batch(3000, "imix", seed=77)
    frames.inject_edge_cases(b, 0.1)
    ou, ov = run_oracle(b, iters=2, action=O.REDIRECT, nif=3, ingress=1)
    umem = torch.from_numpy(b.umem).to(dev)
    descs = torch.from_numpy(b.descs.view(np.uint8).reshape(-1, 16).copy()).to(dev)
    v = torch.empty(b.n, dtype=torch.int32, device=dev)
    cfg = launch_cfg(shape, fused=3)
    assert lib.xsknf_gpu_checksum_batch_cfg(
        ctypes.c_void_p(umem.data_ptr()), umem.numel(), ctypes.c_void_p(descs.data_ptr()), b.n, 1,
        ctypes.byref(_lib.CsumOpts(2, O.REDIRECT, 3, 0)), ctypes.c_void_p(v.data_ptr()),
        ctypes.byref(cfg), None) == 0
    torch.cuda.synchronize()
    assert np.array_equal(umem.cpu().numpy(), b.umem)          # not written
    rec = v.cpu().numpy().view(np.uint32)
    host = b.umem.copy()
    verd = rec.view(np.int32).copy()
    tagged = (rec & 0xC0000000) == 0x40000000
    offs = b.frame_offsets()
    for i in np.flatnonzero(tagged):
        at = int(offs[i]) + int((rec[i] >> 16) & 0x7F) + 6
        host[at] = rec[i] & 0xFF
        host[at + 1] = (rec[i] >> 8) & 0xFF
        verd[i] = (1 + 1) % 3                                    # forward verdict
    assert tagged.sum() > b.n // 2
    assert np.array_equal(verd, ov)
    assert np.array_equal(host, ou)


@pytest.mark.parametrize("checks", ["zero", "nic"])
@pytest.mark.parametrize("order", ["rx", "scattered"])
@pytest.mark.parametrize("path", ["zerocopy", "staged", "resident"])
@pytest.mark.parametrize("layout", ["aligned", "unaligned"])
def test_host_path_bit_exact(dev, path, layout, order, checks):
    """UMEM in (pinned) host memory, descriptors / verdicts in host arrays.
    `scattered`: descriptors in a random order, as the fill ring recycles
    frames -- every batch spans the whole UMEM (STAGED gathers on the CPU).
    `nic`: checks as a NIC's offload writes them, so the kernels write (and
    STAGED's records carry) only the frames whose check changes."""
    from xsknf_amd import HostPath
    b = (frames.aligned_batch(3000, "imix", chunk=2048) if layout == "aligned"
         else frames.unaligned_batch(3000, "imix"))
    if checks == "nic":
        frames.offload_checks_host(b)
    frames.inject_edge_cases(b, 0.1)
    if order == "scattered":
        b.descs = b.descs[np.random.default_rng(5).permutation(b.n)].copy()
    iters = 1 if checks == "nic" else 3          # (with -i 3 every NIC check would change)
    ou, ov = run_oracle(b, iters=iters, action=O.REDIRECT, nif=2, ingress=1)
    cs = Checksummer(ChecksummerOptions(action=O.REDIRECT, csum_iterations=iters), num_interfaces=2,
                     frame_len_hint=1500)
    umem = b.umem.copy()
    # batch sizes across the zero-copy shapes: split kernel (> 2048 frames),
    # group kernels 32 x 3 (<= 256) and 64 x 2 (<= 2048)
    cuts = np.cumsum([0, 2100, 64, 200, 636])
    assert cuts[-1] == b.n
    with HostPath(cs, umem, path=path, max_batch=4096) as hp:
        v = np.concatenate([hp.process_batch(b.descs[lo:hi], ingress_ifindex=1)
                            for lo, hi in zip(cuts[:-1], cuts[1:])])
        st = hp.stats()
    assert st["frames"] == b.n
    assert np.array_equal(v, ov)
    assert np.array_equal(umem, ou)


@pytest.mark.parametrize("path", ["zerocopy", "staged", "resident"])
def test_host_path_two_batches_in_flight(dev, path):
    """xsknf_gpu_ctx_submit / _wait: batches enqueued back to back (two slots in
    flight, each submit completing the batch two back), contiguous, 2-D-strided
    and scattered batches mixed, one larger than a slot piece; every verdict and
    byte equals the oracle's."""
    from xsknf_amd import HostPath
    rng = np.random.default_rng(9)
    b = frames.aligned_batch(80000, "imix", chunk=2048, seed=9)
    frames.inject_edge_cases(b, 0.05, seed=10)
    ou, ov = run_oracle(b, iters=1, action=O.DROP, nif=1)
    perm = np.arange(b.n)
    perm[5000:9000] = rng.permutation(perm[5000:9000])          # a scattered stretch
    descs = b.descs[perm].copy()
    cuts = [0, 64, 1000, 5000, 9000, 9100, 80000]                # 70900 > one 65536-frame piece
    cs = Checksummer(ChecksummerOptions(action=O.DROP), frame_len_hint=1500)
    umem = b.umem.copy()
    outs = [np.full(hi - lo, 7, dtype=np.int32) for lo, hi in zip(cuts[:-1], cuts[1:])]
    with HostPath(cs, umem, path=path, max_batch=80000) as hp:
        tickets = [hp.submit(descs[lo:hi], out) for (lo, hi), out in zip(zip(cuts[:-1], cuts[1:]), outs)]
        hp.wait(tickets[-1])
        st = hp.stats()
    assert st["frames"] == b.n
    assert np.array_equal(np.concatenate(outs), ov[perm])
    assert np.array_equal(umem, ou)


@pytest.mark.parametrize("checks", ["zero", "nic"])
def test_resident_ring(dev, checks):
    """XSKNF_GPU_PATH_RESIDENT: many small batches through the resident
    kernel's ring (more in flight than it has entries, so submits wait for old
    entries), pauses longer than its idle exit (the next submit relaunches it),
    batches of 1 frame up to several entries' worth (cut into 256-frame
    pieces), runs of <= 64-frame batches (one block of an entry's group works,
    the others fall behind the entry's numbers) followed by 256-frame batches
    (all four work, the idle ones catching up); every verdict and byte equals
    the oracle's."""
    import time
    from xsknf_amd import HostPath
    b = frames.unaligned_batch(12000, "imix", seed=21)
    if checks == "nic":
        frames.offload_checks_host(b)
    frames.inject_edge_cases(b, 0.05, seed=22)
    ou, ov = run_oracle(b, iters=1, action=O.REDIRECT, nif=2, ingress=1)
    cs = Checksummer(ChecksummerOptions(action=O.REDIRECT), num_interfaces=2, frame_len_hint=1500)
    umem = b.umem.copy()
    rng = np.random.default_rng(23)
    sizes = [1, 64, 1024, 3000] + [10] * 16 + [256] * 8 + [65] * 8 + list(rng.integers(1, 700, size=40))
    cuts = [0]
    for k in sizes:
        if cuts[-1] + k >= b.n:
            break
        cuts.append(cuts[-1] + int(k))
    cuts.append(b.n)
    outs = [np.full(hi - lo, 7, dtype=np.int32) for lo, hi in zip(cuts[:-1], cuts[1:])]
    with HostPath(cs, umem, path="resident", max_batch=8192) as hp:
        tickets = []
        for j, ((lo, hi), out) in enumerate(zip(zip(cuts[:-1], cuts[1:]), outs)):
            tickets.append(hp.submit(b.descs[lo:hi], out, ingress_ifindex=1))
            if j in (5, 20):            # past the kernel's 1 ms idle exit
                hp.wait(tickets[-1])
                time.sleep(0.03)
        hp.wait(tickets[-1])
        st = hp.stats()
    assert st["frames"] == b.n
    assert np.array_equal(np.concatenate(outs), ov)
    assert np.array_equal(umem, ou)


def test_resident_ring_one_block_per_entry(dev):
    """A resident context for batches of up to 64 frames runs one block per
    ring entry (ResArgs::group = 1): 300 batches of 1..64 frames, more in
    flight than the ring has entries; verdicts and bytes equal the oracle's."""
    from xsknf_amd import HostPath
    b = frames.unaligned_batch(10000, "imix", seed=24)
    frames.inject_edge_cases(b, 0.05, seed=25)
    ou, ov = run_oracle(b, iters=1, action=O.REDIRECT, nif=1)
    cs = Checksummer(ChecksummerOptions(action=O.REDIRECT), num_interfaces=1, frame_len_hint=1500)
    umem = b.umem.copy()
    rng = np.random.default_rng(26)
    cuts = [0]
    while cuts[-1] < b.n:
        cuts.append(min(b.n, cuts[-1] + int(rng.integers(1, 65))))
    outs = [np.full(hi - lo, 7, dtype=np.int32) for lo, hi in zip(cuts[:-1], cuts[1:])]
    with HostPath(cs, umem, path="resident", max_batch=64) as hp:
        tickets = [hp.submit(b.descs[lo:hi], out) for (lo, hi), out in zip(zip(cuts[:-1], cuts[1:]), outs)]
        hp.wait(tickets[-1])
    assert np.array_equal(np.concatenate(outs), ov)
    assert np.array_equal(umem, ou)


def _entries(n):
    return -(-n // 256) if n else 0


@pytest.mark.parametrize("n_ctx,max_batch,batch", [(8, 2000, 100), (8, 64, 50), (40, 300, 257)],
                         ids=["8-groups-of-4", "8-groups-of-1", "40-blocks-serve-several-entries"])
def test_resident_contexts_share_one_kernel(dev, n_ctx, max_batch, batch):
    """Many RESIDENT contexts on one device at once -- one per worker and UMEM,
    as the hook makes them (the reference runs up to XSKNF_MAX_WORKERS = 32
    workers, src/xsknf.h:12, one per queue, src/xsknf.c:992) -- with batches
    interleaved over them.  Every context stays resident: each of its batches
    is a ring entry completed by the device's ONE resident kernel
    (resident_batches), whose launches every context shares.  40 contexts of
    four-block groups need more blocks than the kernel's grid may hold, so a
    block serves several entries of its ring.  Every context's verdicts and
    bytes equal the oracle's."""
    from xsknf_amd import HostPath
    total = 1200 if n_ctx > 8 else 2000
    bs = [frames.aligned_batch(total, "imix", chunk=2048, seed=40 + k) for k in range(n_ctx)]
    for k, b in enumerate(bs):
        frames.inject_edge_cases(b, 0.05, seed=50 + k)
    refs = [run_oracle(b, iters=1, action=O.DROP, nif=1) for b in bs]
    cs = Checksummer(ChecksummerOptions(action=O.DROP), frame_len_hint=1500)
    umems = [b.umem.copy() for b in bs]
    hps = []
    try:
        for u in umems:
            hps.append(HostPath(cs, u, path="resident", max_batch=max_batch))
        outs = [np.full(b.n, 7, dtype=np.int32) for b in bs]
        tickets = [[] for _ in bs]
        for lo in range(0, total, batch):
            for k, (hp, b) in enumerate(zip(hps, bs)):
                tickets[k].append(hp.submit(b.descs[lo:lo + batch], outs[k][lo:lo + batch]))
        for hp, t in zip(hps, tickets):
            hp.wait(t[-1])
        stats = [hp.stats() for hp in hps]
    finally:
        for hp in hps:
            hp.close()
    want = sum(_entries(min(batch, total - lo)) for lo in range(0, total, batch))
    for st in stats:
        assert st["frames"] == total
        assert st["resident_batches"] == want, st
        assert st["resident_launches"] >= n_ctx      # (each context's arrival relaunches the kernel)
    for (ou, ov), u, v in zip(refs, umems, outs):
        assert np.array_equal(v, ov)
        assert np.array_equal(u, ou)


def test_resident_rings_join_and_leave_under_traffic(dev):
    """A ring joining (a new worker's first batch) and one leaving (a context
    destroyed) stop and relaunch the shared kernel while other contexts have
    batches in flight: those batches are picked up by the relaunch, none is
    processed twice (ihl 2/3 frames would show it: reprocessing them is not
    idempotent), and every context's output equals the oracle's."""
    from xsknf_amd import HostPath
    bs = [frames.unaligned_batch(1500, "imix", seed=60 + k) for k in range(4)]
    for k, b in enumerate(bs):
        frames.inject_edge_cases(b, 0.1, seed=70 + k)
    refs = [run_oracle(b, iters=2, action=O.REDIRECT, nif=3, ingress=1) for b in bs]
    cs = Checksummer(ChecksummerOptions(action=O.REDIRECT, csum_iterations=2), num_interfaces=3,
                     frame_len_hint=1500)
    umems = [b.umem.copy() for b in bs]
    outs = [np.full(b.n, 7, dtype=np.int32) for b in bs]
    hp = {}
    try:
        hp[0] = HostPath(cs, umems[0], path="resident", max_batch=256)
        hp[1] = HostPath(cs, umems[1], path="resident", max_batch=64)
        t = {0: [], 1: [], 2: [], 3: []}
        pos = {k: 0 for k in range(4)}

        def feed(k, size):
            lo = pos[k]
            hi = min(bs[k].n, lo + size)
            if hi > lo:
                t[k].append(hp[k].submit(bs[k].descs[lo:hi], outs[k][lo:hi], ingress_ifindex=1))
            pos[k] = hi

        for _ in range(4):
            feed(0, 200)
            feed(1, 64)
        hp[2] = HostPath(cs, umems[2], path="resident", max_batch=256)   # joins: 0 and 1 in flight
        for _ in range(3):
            feed(0, 200)
            feed(1, 64)
            feed(2, 256)
        hp[1].wait(t[1][-1])
        hp[1].close()                                                     # leaves: 0 and 2 in flight
        hp[3] = HostPath(cs, umems[3], path="resident", max_batch=1500)  # joins
        while any(pos[k] < bs[k].n for k in (0, 2, 3)):
            for k in (0, 2, 3):
                feed(k, 150)
        for k in (0, 2, 3):
            hp[k].wait(t[k][-1])
    finally:
        for h in hp.values():
            h.close()
    # context 1 left after pos[1] frames: exactly those are done
    n1 = pos[1]
    assert np.array_equal(outs[1][:n1], refs[1][1][:n1])
    offs = bs[1].frame_offsets()
    end1 = int(offs[n1 - 1] + bs[1].descs["len"][n1 - 1])
    assert np.array_equal(umems[1][:end1], refs[1][0][:end1])
    for k in (0, 2, 3):
        assert np.array_equal(outs[k], refs[k][1]), k
        assert np.array_equal(umems[k], refs[k][0]), k


def test_mixed_paths_from_worker_threads(dev):
    """Worker threads on one device, each with its own context and UMEM as the
    reference's workers (src/xsknf.c:1075-1095), on different host paths at
    once: two RESIDENT (the shared kernel's hardware queue), two ZEROCOPY and
    two STAGED (launches on their own streams), each keeping four batches out.
    Every worker's verdicts and bytes equal the oracle's."""
    import threading
    from xsknf_amd import HostPath
    paths = ["resident", "zerocopy", "staged"] * 2
    bs = [frames.unaligned_batch(3000, "imix", seed=90 + k) for k in range(len(paths))]
    for k, b in enumerate(bs):
        frames.inject_edge_cases(b, 0.05, seed=100 + k)
    refs = [run_oracle(b, iters=3, action=O.REDIRECT, nif=2, ingress=1) for b in bs]
    cs = Checksummer(ChecksummerOptions(action=O.REDIRECT, csum_iterations=3), num_interfaces=2,
                     frame_len_hint=1500)
    umems = [b.umem.copy() for b in bs]
    outs = [np.full(b.n, 7, dtype=np.int32) for b in bs]
    errors, stats = [], [None] * len(paths)
    start = threading.Barrier(len(paths))

    def worker(k):
        try:
            with HostPath(cs, umems[k], path=paths[k], max_batch=64) as hp:
                start.wait()
                tickets = []
                for lo in range(0, bs[k].n, 64):
                    tickets.append(hp.submit(bs[k].descs[lo:lo + 64], outs[k][lo:lo + 64], ingress_ifindex=1))
                    if len(tickets) >= 4:
                        hp.wait(tickets[-4])
                hp.wait(tickets[-1])
                stats[k] = hp.stats()
        except Exception as e:   # noqa: BLE001 -- reported below
            errors.append((k, repr(e)))
            start.abort()

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(len(paths))]
    for t in threads:
        t.start()
    for t in threads:
        t.join(120)
    assert not any(t.is_alive() for t in threads), "a worker did not finish"
    assert not errors, errors
    for k, p in enumerate(paths):
        assert stats[k]["frames"] == bs[k].n
        if p == "resident":
            assert stats[k]["resident_batches"] == sum(_entries(min(64, bs[k].n - lo)) for lo in range(0, bs[k].n, 64))
        assert np.array_equal(outs[k], refs[k][1]), (k, p)
        assert np.array_equal(umems[k], refs[k][0]), (k, p)


def test_resident_rings_past_the_device_limit_are_refused(dev):
    """64 rings per device (XSKNF_MAX_WORKERS x a zero-copy and a copy-mode
    UMEM); a 65th RESIDENT context is refused with -ENOSPC instead of running
    some other way; the 64 keep working, bit-exact."""
    from xsknf_amd import HostPath
    from xsknf_amd._lib import XsknfGpuError
    cs = Checksummer(ChecksummerOptions(action=O.REDIRECT), num_interfaces=1, frame_len_hint=1500)
    bs = [frames.unaligned_batch(100, "imix", seed=300 + k) for k in range(64)]
    refs = [run_oracle(b, iters=1, action=O.REDIRECT, nif=1) for b in bs]
    umems = [b.umem.copy() for b in bs]
    hps = []
    try:
        for k, u in enumerate(umems):   # (one- and four-block groups: both fit at 8 entries per block)
            hps.append(HostPath(cs, u, path="resident", max_batch=64 if k % 4 else 512))
        extra = np.zeros(4096, dtype=np.uint8)
        with pytest.raises(XsknfGpuError, match="rc=-28"):
            HostPath(cs, extra, path="resident", max_batch=64)
        outs = [np.concatenate([hp.process_batch(b.descs[lo:lo + 50]) for lo in range(0, b.n, 50)])
                for hp, b in zip(hps, bs)]
    finally:
        for hp in hps:
            hp.close()
    for (ou, ov), u, v in zip(refs, umems, outs):
        assert np.array_equal(v, ov)
        assert np.array_equal(u, ou)


@pytest.mark.parametrize("checks", ["zero", "nic"])
@pytest.mark.parametrize("length", [4000, 9000])
def test_resident_ring_long_frames(dev, length, checks):
    """The resident kernel's register tiles cover 1536 B per pass; longer
    frames take further passes (finish_long_frames).  Unaligned UMEM (the -u
    layout of config 5, odd starts) with 4000 / 9000 B frames and edge cases,
    in batches under and over 64 frames (one block and four per entry), with
    zero checks and with the checks a NIC wrote; bit-exact."""
    from xsknf_amd import HostPath
    b = frames.unaligned_batch(700, length, seed=80 + length)
    if checks == "nic":
        frames.offload_checks_host(b)
    frames.inject_edge_cases(b, 0.1, seed=81)
    ou, ov = run_oracle(b, iters=1, action=O.REDIRECT, nif=1)
    cs = Checksummer(ChecksummerOptions(action=O.REDIRECT), num_interfaces=1, frame_len_hint=length)
    umem = b.umem.copy()
    cuts = [0, 1, 40, 104, 360, 361, 600, 700]
    outs = [np.full(hi - lo, 7, dtype=np.int32) for lo, hi in zip(cuts[:-1], cuts[1:])]
    with HostPath(cs, umem, path="resident", max_batch=512) as hp:
        tk = [hp.submit(b.descs[lo:hi], out) for (lo, hi), out in zip(zip(cuts[:-1], cuts[1:]), outs)]
        hp.wait(tk[-1])
        assert hp.stats()["resident_batches"] == sum(_entries(hi - lo) for lo, hi in zip(cuts[:-1], cuts[1:]))
    assert np.array_equal(np.concatenate(outs), ov)
    assert np.array_equal(umem, ou)


@pytest.mark.parametrize("shape", [(16, 2, 2, 0, 1, 1, 20), (16, 3, 1, 0, 0, 1, 24), (16, 3, 2, 0, 2, 1, 20),
                                   (16, 2, 2, 0, 5, 1, 24)], ids=["w4-16x2", "w8-16x3", "w4-16x3u2", "w8-16x2-2B"])
def test_huge_frames_take_the_whole_wave_path(dev, shape):
    """Frames with more payload items than the split kernel's per-frame item
    budget (over ~27-43 KB) are summed by the whole wave; mixed in the same
    tiles with short and ordinary frames, and with frames past 64 KB."""
    import ctypes
    from xsknf_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(5)
    n = 300
    lens = np.where(rng.random(n) < 0.3, rng.integers(30000, 200000, size=n),
                    rng.integers(0, 2000, size=n)).astype(np.uint32)
    b = frames.unaligned_batch(n, lens, seed=5)
    frames.inject_edge_cases(b, 0.05)
    ou, ov = run_oracle(b, iters=3, action=O.REDIRECT, nif=2, ingress=0)
    umem = torch.from_numpy(b.umem).to(dev)
    descs = torch.from_numpy(b.descs.view(np.uint8).reshape(-1, 16).copy()).to(dev)
    v = torch.empty(n, dtype=torch.int32, device=dev)
    assert lib.xsknf_gpu_checksum_batch_cfg(
        ctypes.c_void_p(umem.data_ptr()), umem.numel(), ctypes.c_void_p(descs.data_ptr()), n, 0,
        ctypes.byref(_lib.CsumOpts(3, O.REDIRECT, 2, 0)), ctypes.c_void_p(v.data_ptr()),
        ctypes.byref(launch_cfg(shape)), None) == 0
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy(), ov)
    assert np.array_equal(umem.cpu().numpy(), ou)


def test_concurrent_streams(dev):
    """Many batches in flight at once on separate streams (as the AF_XDP hook
    runs one stream per worker): every one bit-exact.  The scatter pass's
    per-launch record counters (64 sets) are reused by launches 64 apart:
    with more than 64 launches queued at once, a reused set must make the
    pass scan, never skip (g_rec_count in checksummer.hip)."""
    nstreams = 24
    jobs = []
    for i in range(nstreams):
        length = (1500, "imix", 64)[i % 3]
        b = frames.aligned_batch(4096, length, chunk=2048, seed=100 + i)
        frames.inject_edge_cases(b, 0.05, seed=200 + i)
        ref = b.copy()
        for _ in range(4):   # reprocessing is not idempotent for ihl 2/3 frames
            ov = O.c_process_batch(ref.umem, ref.descs)
        jobs.append((b, ref.umem, ov, torch.cuda.Stream(device=dev)))
    outs = []
    for b, ou, ov, st in jobs:
        with torch.cuda.stream(st):
            umem = torch.from_numpy(b.umem).to(dev, non_blocking=False)
            descs = torch.from_numpy(b.descs.view(np.uint8).reshape(-1, 16).copy()).to(dev)
        outs.append((umem, descs))
    torch.cuda.synchronize()
    cs = Checksummer(frame_len_hint=1500)
    res = []
    for rep in range(4):   # several launches per stream, none waited for in between
        for (umem, descs), (b, ou, ov, st) in zip(outs, jobs):
            with torch.cuda.stream(st):
                res.append(cs.process_batch(umem, descs))
    torch.cuda.synchronize()
    for k, ((umem, descs), (b, ou, ov, st)) in enumerate(zip(outs, jobs)):
        assert np.array_equal(res[3 * nstreams + k].cpu().numpy(), ov), f"stream {k}"
        assert np.array_equal(umem.cpu().numpy(), ou), f"stream {k}"


@pytest.mark.slow
@pytest.mark.parametrize("shape", [(16, 2, 2, 0, 18, 1, 24), (16, 2, 2, 0, 18, 1, 56),
                                   pytest.param((16, 3, 2, 0, 18, 1, 24),
                                                marks=pytest.mark.skipif(not AB_BUILD, reason="A/B build only"))],
                         ids=_shape_id)
def test_one_block_per_cu_asked_is_bit_exact(dev, shape):
    """One block per CU asked for over 600K frames -- the launch of the three
    unexplained faults, whose waves then had more tiles than their
    LDS patch lists.  The launch now raises the grid until no wave does
    (test_no_wave_passes_its_patch_list); every verdict and byte matches the
    oracle."""
    import ctypes
    from xsknf_amd import _lib
    lib = _lib.load()
    n = 600_000
    umem, descs, lens = frames.device_batch(n, "imix", layout="aligned", device=dev, seed=31)
    host = umem.cpu().numpy()
    hd = descs.cpu().numpy().view(frames.DESC_DTYPE).reshape(-1).copy()
    frames.inject_edge_cases(frames.HostBatch(host, hd, "aligned"), 0.01, seed=32)
    umem.copy_(torch.from_numpy(host))
    descs.copy_(torch.from_numpy(hd.view(np.int64).reshape(n, 2)))
    v = torch.empty(n, dtype=torch.int32, device=dev)
    opts = _lib.CsumOpts(1, O.REDIRECT, 1, 0)
    cfg = launch_cfg(shape, bpc=1)
    # where the arrays lie (to place a faulting address)
    print(f"small-grid test arrays: umem [{umem.data_ptr():#x}, {umem.data_ptr() + umem.numel():#x}) "
          f"descs [{descs.data_ptr():#x}, {descs.data_ptr() + 16 * n:#x}) v [{v.data_ptr():#x}, "
          f"{v.data_ptr() + 4 * n:#x})", file=sys.stderr, flush=True)
    assert lib.xsknf_gpu_checksum_batch_cfg(
        ctypes.c_void_p(umem.data_ptr()), umem.numel(), ctypes.c_void_p(descs.data_ptr()), n, 0,
        ctypes.byref(opts), ctypes.c_void_p(v.data_ptr()), ctypes.byref(cfg), None) == 0
    gv, gu = _results(v, umem)
    _, ov = oracles.time_batch(host, hd)
    assert np.array_equal(gv, ov)
    assert np.array_equal(gu, host)


@pytest.mark.slow
@pytest.mark.parametrize("length,n,mean,window", [(64, 20000, False, 1024), (1500, 20000, False, 56),
                                                  ("imix", 20000, True, 24), ("imix", 20000, False, 56),
                                                  (9000, 6000, False, 52)],
                         ids=["64-lane", "1500-pool", "imix-static", "imix-pool", "jumbo-pool"])
def test_umem_past_the_patch_list_index(dev, length, n, mean, window):
    """A UMEM of 128 GiB or more (kPatchMaxUmem: the patch lists index 64-byte
    sectors in 32 bits) parks its checks for scatter_checks instead of the lists
    (DESIGN 3).  A 128 GiB + 64 MiB device UMEM (MI355X holds 288 GB) with the
    batch's frames placed past 128 GiB, every product shape: every verdict and
    byte matches the oracle."""
    big_size = (1 << 37) + (64 << 20)
    free, _ = torch.cuda.mem_get_info(dev)
    if free < big_size + (8 << 30):
        pytest.skip(f"{free >> 30} GiB free on the device")
    if length == 9000:
        b = frames.unaligned_batch(n, length, seed=n)
    else:
        b = frames.aligned_batch(n, length, seed=n)
    frames.inject_edge_cases(b, 0.02, seed=n + 1)
    lens = b.descs["len"]
    ou, ov = run_oracle(b)
    size = b.umem.size
    base_off = (big_size - size) & ~4095
    assert base_off >= 1 << 37
    big = torch.empty(big_size, dtype=torch.uint8, device=dev)
    try:
        big[base_off:base_off + size].copy_(torch.from_numpy(b.umem))
        d = b.descs.copy()
        mask = np.uint64((1 << frames.OFFSET_SHIFT) - 1)
        d["addr"] = ((d["addr"] & mask) + np.uint64(base_off)) | (d["addr"] & ~mask)
        descs = torch.from_numpy(d.view(np.uint8).reshape(-1, 16).copy()).to(dev)
        cs = Checksummer(ChecksummerOptions(), num_interfaces=1, frame_len_hint=int(lens.max()),
                         frame_len_mean=int(lens.mean()) if mean else 0)
        assert cs.launch_cfg().window_chunks == window
        v = cs.process_batch(big, descs)
        gv, gu = _results(v, big[base_off:base_off + size])
    finally:
        del big
        torch.cuda.empty_cache()
    assert np.array_equal(gv, ov)
    if not np.array_equal(gu, ou):
        diff = np.nonzero(gu != ou)[0]
        raise AssertionError(f"{diff.size} UMEM bytes differ, first at {diff[:10]}")


TL_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "tl", "libxsknf_gpu.so")


@pytest.mark.skipif(not os.path.exists(TL_LIB), reason="timeline build absent (make tl)")
@pytest.mark.parametrize("frames_n,bpc", [(600_000, 1), (1 << 20, 1), (1 << 20, 8)])
@pytest.mark.parametrize("window,limit", [(24, 6), (56, 7), (52, 20)], ids=["static", "pool", "pool-jumbo"])
def test_no_wave_passes_its_patch_list(dev, window, limit, frames_n, bpc):
    """launch_split sizes the grid so that no wave of a patch-list shape gets
    more tiles than its list holds (static: each wave's share of the tiles;
    pool: a wave with a full list claims no more), whatever blocks_per_cu asks
    (DESIGN 3).  Per-wave tile counts from the timeline build (tools/timeline.py),
    in a child process (the instrumented library is a second copy)."""
    import json
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, XSKNF_GPU_LIB=TL_LIB)
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "timeline.py"), "--workload", "imix",
                          "--frames", str(frames_n), "--reps", "2", "--bpc", str(bpc),
                          "--variant", f"16,{3 if window == 52 else 2},2,0,18,1,{window}"],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    med = json.loads(out.stdout.strip().splitlines()[-1])["median"]
    tiles = {int(k): v for k, v in med["tiles"].items()}
    assert sum(k * v for k, v in tiles.items()) >= (frames_n + 63) // 64   # every tile (pool halves: more units)
    assert max(tiles) <= limit, tiles


@pytest.mark.parametrize("length,n,window", [(9000, 4 * 120 * 64, 52), (9000, 4 * 104 * 64 + 1, 52),
                                             ("imix", 4 * 72 * 64 + 4095, 56), ("imix-mean", 4 * 8 * 24 * 64 + 4095, 24),
                                             (64, 300_000, 1024)],
                         ids=["jumbo-120", "jumbo-104", "imix-pool", "imix-static", "64-lane"])
def test_grid_sizing_on_a_smaller_device(length, n, window):
    """launch_split's grid on a device of 4 CUs (XSKNF_GPU_CU_LIMIT, a test hook
    read once per process, hence the child): a pool block of bt tiles has
    bt + (parts - 1) * k * SW units, so a jumbo block (its last 3 SW tiles in
    quarters, 8 waves of 20-unit lists) holds 88 tiles, not SW * (PT - 1) -- at
    4 x 120 and 4 x 104 tiles (round 4's bound with 16-unit lists, and 104 with
    the last SW tiles split) the grid must grow past 4 blocks, and every frame still
    bit-exact.  The pooled W = 8, static and lane shapes at (or past)
    their bounds at 4 CUs too."""
    import json
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, XSKNF_GPU_CU_LIMIT="4")
    args = ["--frames", str(n), "--length", str(length).replace("-mean", ""),
            "--layout", "unaligned" if length == 9000 else "aligned"] + (["--mean"] if length == "imix-mean" else [])
    out = subprocess.run([sys.executable, os.path.join(root, "tests", "cu_limit_child.py")] + args,
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["cus_limit"] == "4"
    assert r["window_chunks"] == window   # the shape the product picks: jumbo / W = 8 pooled, static, lane
    assert r["bad_verdicts"] == 0 and r["bad_bytes"] == 0, r
    assert r["pool_guard_trips"] == 0, r


@pytest.mark.skipif(not AB_BUILD, reason="A/B build only (XSKNF_AB_NO_GRID_BOUND)")
def test_pool_guard_trips_without_the_grid_bound():
    """The pool guard works: in the A/B build with launch_split's grid bound left
    out (XSKNF_AB_NO_GRID_BOUND) and the grids sized for 4 CUs, a 30720-frame
    jumbo batch gives each pool block 120 tiles, more units than its waves'
    20-unit lists hold; the waves stop claiming, units go unclaimed, their
    frames stay unsummed, and xsknf_gpu_pool_guard_trips counts it (with the
    bound, the same batch is bit-exact and the count 0:
    test_grid_sizing_on_a_smaller_device)."""
    import json
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, XSKNF_GPU_CU_LIMIT="4", XSKNF_AB_NO_GRID_BOUND="1")
    out = subprocess.run([sys.executable, os.path.join(root, "tests", "cu_limit_child.py"), "--frames", "30720",
                          "--length", "9000", "--layout", "unaligned"],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["window_chunks"] == 52 and r["pool_guard_trips"] > 0, r
    assert r["bad_bytes"] > 0 or r["bad_verdicts"] > 0, r


@pytest.mark.parametrize("shape", [(16, 2, 2, 0, 18, 1, 56), (16, 3, 2, 0, 18, 1, 52), (16, 3, 2, 0, 0, 1, 52),
                                   pytest.param((1, 5, 2, 0, 1, 0, 32),
                                                marks=pytest.mark.skipif(not AB_BUILD, reason="A/B build only")),
                                   pytest.param((1, 5, 1, 0, 1, 0, 32),
                                                marks=pytest.mark.skipif(not AB_BUILD, reason="A/B build only"))],
                         ids=["pool-w8", "pool-jumbo", "pool-jumbo-scatter", "pool-lane", "pool-lane-64"])
@pytest.mark.parametrize("n", [1, 17, 33, 95, 12 * 64 + 5, 3 * 12 * 64 - 7, 256 * 12 * 64 + 4095])
def test_pool_units_cover_every_frame(dev, shape, n):
    """The CU-wide tile pool (window + 32): the block's last tiles run as
    halves (W = 8) or quarters (jumbo), and a batch whose length is not a
    multiple of 64, 32 or 16 leaves partial and empty units; batches from one
    frame to more than a full grid of tiles, every frame bit-exact."""
    import ctypes
    from xsknf_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(n)
    lens = rng.integers(40, {56: 1600, 52: 9000, 32: 129}[shape[6]], size=n).astype(np.uint32)
    if shape[6] != 52:
        b = frames.aligned_batch(n, np.minimum(lens, 1792), chunk=2048, seed=n)
    else:
        b = frames.unaligned_batch(n, lens, seed=n)
    frames.inject_edge_cases(b, 0.05)
    ou, ov = run_oracle(b)
    umem = torch.from_numpy(b.umem).to(dev)
    descs = torch.from_numpy(b.descs.view(np.uint8).reshape(-1, 16).copy()).to(dev)
    v = torch.empty(b.n, dtype=torch.int32, device=dev)
    assert lib.xsknf_gpu_checksum_batch_cfg(
        ctypes.c_void_p(umem.data_ptr()), umem.numel(), ctypes.c_void_p(descs.data_ptr()), b.n, 0,
        ctypes.byref(_lib.CsumOpts(1, O.REDIRECT, 1, 0)), ctypes.c_void_p(v.data_ptr()),
        ctypes.byref(launch_cfg(shape, bpc=8)), None) == 0
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy(), ov)
    assert np.array_equal(umem.cpu().numpy(), ou)
