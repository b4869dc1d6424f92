"""The RFC 768/1071 receive-side checker (tests/rfc1071.py) on CPU, and the
oracle against it: independent of every restatement of checksummer_user.c.

The reference's traffic carries NIC-computed RFC checksums (tests/gen-traffic.lua:120),
so a correct checksummer output verifies as 0xFFFF on every frame whose single fold
(checksummer_user.c:105-106) loses no carry, and as 0x0001 (the RFC value + 1) on
the frames where it does (KAT C2).
"""
import numpy as np
import pytest

from oracle import csum_oracle as O
from tests import rfc1071
from tests.test_oracle import KATS
from xsknf_amd import frames

torch = pytest.importorskip("torch")


def _verify(b):
    return rfc1071.verify(torch.from_numpy(b.umem), b.frame_offsets().astype(np.int64), b.descs["len"])


@pytest.mark.parametrize("kat,want", [("C1", 0xFFFF), ("C2", 0x0001), ("C4", 0xFFFF)])
def test_known_answers_verify(kat, want):
    name, frame, kw, ret, sl, chk = next(k for k in KATS if k[0] == kat)
    f = bytearray(frame)
    O.c_packet_processor(f, **kw)
    umem = np.frombuffer(bytes(f), dtype=np.uint8).copy()
    d = np.zeros(1, dtype=frames.DESC_DTYPE)
    d["len"] = len(f)
    idx, V = _verify(frames.HostBatch(umem, d, "aligned"))
    assert idx.tolist() == [0] and V[0] == want


@pytest.mark.parametrize("length,layout", [(64, "aligned"), (1500, "aligned"), ("imix", "aligned"),
                                           (9000, "unaligned"), ("imix", "unaligned")])
def test_oracle_output_passes_the_receive_check(length, layout):
    b = (frames.aligned_batch(4000, length, chunk=2048) if layout == "aligned"
         else frames.unaligned_batch(2000, length, seed=7))
    frames.inject_edge_cases(b, 0.02)
    O.c_process_batch(b.umem, b.descs)
    idx, V = _verify(b)
    assert idx.size > 0.95 * b.n
    assert np.all((V == 0xFFFF) | (V == 0x0001))
    assert (V == 0xFFFF).mean() > 0.9


def test_receive_check_catches_a_wrong_check():
    b = frames.aligned_batch(200, 570, chunk=2048)
    O.c_process_batch(b.umem, b.descs)
    offs = b.frame_offsets().astype(np.int64)
    b.umem[offs[17] + 40] ^= 0x10
    idx, V = _verify(b)
    assert V[list(idx).index(17)] not in (0xFFFF, 0x0001)


@pytest.mark.parametrize("length,layout", [(1500, "aligned"), ("imix", "aligned"), (64, "aligned"),
                                           (9000, "unaligned"), ("imix", "unaligned")])
def test_nic_offloaded_checks_verify_and_mostly_stay(length, layout):
    """frames.offload_checks_host gives each frame the check a NIC's UDP
    offload writes (tests/gen-traffic.lua:120): every frame verifies as 0xFFFF,
    and the oracle, run over them, changes only the checks of its carry-loss
    frames (the RFC value + 1) -- no other byte."""
    b = (frames.aligned_batch(6000, length, seed=5) if layout == "aligned"
         else frames.unaligned_batch(6000, length, seed=5))
    assert frames.offload_checks_host(b) == b.n
    idx, V = _verify(b)
    assert idx.size == b.n and np.all(V == 0xFFFF)
    before = b.umem.copy()
    O.c_process_batch(b.umem, b.descs)
    offs = b.frame_offsets().astype(np.int64)
    diff = np.flatnonzero(before != b.umem)
    assert np.isin(diff, np.concatenate([offs + 40, offs + 41])).all()
    changed = np.unique(np.searchsorted(np.sort(offs), diff, side="right"))
    assert changed.size < {64: 0.001, 1500: 0.01, 9000: 0.05}.get(length, 0.01) * b.n + 1
    idx2, V2 = _verify(b)
    assert np.all((V2 == 0xFFFF) | (V2 == 0x0001))


def test_offload_skips_malformed_frames():
    """Edge-case frames (non-IPv4, non-UDP, ihl != 5, short) keep their bytes."""
    b = frames.unaligned_batch(3000, "imix", seed=8)
    frames.inject_edge_cases(b, 0.3, seed=9)
    before = b.umem.copy()
    frames.offload_checks_host(b)
    offs = b.frame_offsets().astype(np.int64)
    lens = b.descs["len"].astype(np.int64)
    ok = np.array([lens[i] >= 42 and before[offs[i] + 12] == 8 and before[offs[i] + 13] == 0
                   and before[offs[i] + 14] == 0x45 and before[offs[i] + 23] == 17 for i in range(b.n)])
    diff = np.flatnonzero(before != b.umem)
    allowed = np.concatenate([offs[ok] + 40, offs[ok] + 41])
    assert np.isin(diff, allowed).all()
