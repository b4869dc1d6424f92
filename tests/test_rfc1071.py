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
