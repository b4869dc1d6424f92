"""The CPU oracle, pinned before it is trusted.

Pins: the reference's own checksummer_user.c:30-112, compiled here from its
verbatim text (oracle/_ref, tests/test_ref_pin.py), and the known answers C1-C6
of SURVEY.md Appendix C, which that library reproduces.
Cross-checks: three independent restatements (C literal loop, Python literal
loop, numpy closed form) must agree byte-for-byte on randomized frames covering
every branch of checksummer_user.c:30-112.  Golden fixtures are checked in
test_golden.py.
"""
import numpy as np
import pytest

from oracle import csum_oracle as O
from xsknf_amd import frames


def base_frame(n):
    """SURVEY.md Appendix C base header for length n (42 bytes, then zeros)."""
    f = bytearray(n)
    h = bytes.fromhex("0a0000000000" "0a0000000001" "0800" "4500" + "%04x" % max(n - 14, 0) +
                      "0000" "0000" "4011" "0000" "0a000000" "ac000001" "1388" "0050" +
                      "%04x" % max(n - 34, 0) + "0000")
    f[:min(n, 42)] = h[:min(n, 42)]
    return f


def kat_frames():
    """(name, frame, kwargs, expected_ret, check_slice, expected_check_hex or None)."""
    out = []
    f = base_frame(60)
    for i in range(42, 60):
        f[i] = (i * 7) & 0xFF
    out.append(("C1", f, dict(iters=1, action=O.REDIRECT, nif=1), 0, (40, 42), "e450"))
    f = base_frame(1500)
    for i in range(42, 1498):
        f[i] = (i * 131 + 7) & 0xFF
    f[1498], f[1499] = 0x52, 0x3B
    out.append(("C2", f, dict(iters=1, action=O.REDIRECT, nif=1), 0, (40, 42), "ffff"))
    f = base_frame(9000)
    for i in range(42, 9000):
        f[i] = 0xFF
    out.append(("C3", f, dict(iters=50, action=O.DROP, nif=1), -1, (40, 42), "7280"))
    f = base_frame(61)
    for i in range(42, 61):
        f[i] = (i * 7) & 0xFF
    out.append(("C4", f, dict(ingress=1, iters=1, action=O.REDIRECT, nif=2), 0, (40, 42), "404e"))
    f = base_frame(60)
    f[12], f[13] = 0x08, 0x06
    out.append(("C5", f, dict(iters=1, action=O.DROP, nif=1), 0, None, None))
    f = base_frame(60)
    f[23] = 6
    out.append(("C6-tcp", f, dict(iters=1, action=O.DROP, nif=1), 0, None, None))
    out.append(("C6-33", base_frame(33), dict(iters=1, action=O.REDIRECT, nif=1), -1, None, None))
    out.append(("C6-13", base_frame(13), dict(iters=1, action=O.REDIRECT, nif=1), -1, None, None))
    f = base_frame(60)
    f[14] = 0x4F
    out.append(("C6-ihl15", f, dict(iters=1, action=O.REDIRECT, nif=1), -1, None, None))
    f = base_frame(64)
    for i in range(42, 64):
        f[i] = (i * 13) & 0xFF
    f[14] = 0x46
    out.append(("C6-ihl6", f, dict(iters=1, action=O.REDIRECT, nif=1), 0, (44, 46), "5249"))
    return out


KATS = kat_frames()


@pytest.mark.parametrize("impl", ["c", "py", "np"])
@pytest.mark.parametrize("kat", KATS, ids=[k[0] for k in KATS])
def test_known_answers(impl, kat):
    name, frame, kw, ret, sl, chk = kat
    f = bytearray(frame)
    orig = bytes(f)
    if impl == "c":
        r = O.c_packet_processor(f, **kw)
    elif impl == "py":
        r = O.py_packet_processor(f, len(f), **kw)
    else:
        a = np.frombuffer(f, dtype=np.uint8).copy()
        r = O.np_packet_processor(a, **kw)
        f = bytearray(a.tobytes())
    assert r == ret
    if chk is None:
        assert bytes(f) == orig, "frame must be untouched on this branch"
    else:
        assert bytes(f[sl[0]:sl[1]]).hex() == chk
        diff = [i for i in range(len(f)) if f[i] != orig[i]]
        assert all(sl[0] <= i < sl[1] for i in diff), "only the 2 check bytes may change"


def test_single_fold_trap_differs_from_rfc1071():
    """C2 is the case where the reference's single fold (carry dropped) differs
    from a correct RFC 1071 fold; an oracle that 'fixes' the fold fails here."""
    f = bytearray(KATS[1][1])
    O.c_packet_processor(f, iters=1, action=O.REDIRECT, nif=1)
    u = 34
    g = bytearray(KATS[1][1])
    g[u + 6] = g[u + 7] = 0
    s = sum(g[i] | (g[i + 1] << 8) for i in (26, 28, 30, 32)) + 0x1100 + (g[u + 4] | g[u + 5] << 8)
    s += sum(g[i] | (g[i + 1] << 8) for i in range(u, 1500, 2))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    rfc = (~s) & 0xFFFF
    assert bytes(f[40:42]) == b"\xff\xff"
    assert rfc.to_bytes(2, "little") == b"\xfe\xff"


def _random_frames(rng, count, max_len=600):
    out = []
    for i in range(count):
        n = int(rng.integers(0, max_len))
        f = bytearray(rng.integers(0, 256, size=n, dtype=np.uint8).tobytes())
        if n >= 14 and rng.random() < 0.85:
            f[12], f[13] = 0x08, 0x00
        if n >= 24 and rng.random() < 0.85:
            f[23] = 17
        if n >= 15 and rng.random() < 0.5:
            f[14] = (f[14] & 0xF0) | 5
        out.append(f)
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_three_restatements_agree(seed):
    rng = np.random.default_rng(seed)
    for f0 in _random_frames(rng, 400):
        kw = dict(ingress=int(rng.integers(0, 4)), iters=int(rng.integers(-1, 6)),
                  action=int(rng.integers(0, 2)), nif=int(rng.integers(1, 5)))
        a, b = bytearray(f0), bytearray(f0)
        c = np.frombuffer(bytes(f0), dtype=np.uint8).copy()
        ra = O.c_packet_processor(a, **kw)
        rb = O.py_packet_processor(b, len(b), **kw)
        rc = O.np_packet_processor(c, **kw)
        assert ra == rb == rc
        assert bytes(a) == bytes(b) == c.tobytes()


def test_batch_loop_matches_per_frame_aligned_and_unaligned():
    for b in (frames.aligned_batch(300, "imix", chunk=2048),
              frames.unaligned_batch(300, "imix")):
        frames.inject_edge_cases(b, 0.3)
        ref = b.copy()
        v = O.c_process_batch(b.umem, b.descs, iters=2, action=O.REDIRECT, nif=3, ingress=1)
        offs = ref.frame_offsets()
        for i in range(ref.n):
            o, n = int(offs[i]), int(ref.descs["len"][i])
            fr = np.ascontiguousarray(ref.umem[o:o + n])
            r = O.np_packet_processor(fr, ingress=1, iters=2, action=O.REDIRECT, nif=3)
            ref.umem[o:o + n] = fr
            assert r == v[i]
        assert np.array_equal(ref.umem, b.umem)


def test_iterations_closed_form_wraps():
    """C3-style frames with many iterations exercise the u32 wrap of the sum."""
    rng = np.random.default_rng(7)
    for _ in range(20):
        n = int(rng.integers(42, 9001))
        f = base_frame(n)
        f[42:] = bytes([0xFF]) * (n - 42)
        it = int(rng.integers(1, 200))
        a, c = bytearray(f), np.frombuffer(bytes(f), dtype=np.uint8).copy()
        assert O.c_packet_processor(a, iters=it, action=O.DROP) == O.np_packet_processor(
            c, iters=it, action=O.DROP) == -1
        assert bytes(a) == c.tobytes()
