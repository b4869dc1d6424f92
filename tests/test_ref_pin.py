"""The oracle pinned to the reference itself.

`oracle/_ref/libcsum_ref.so` is the reference's own xsknf_packet_processor()
(examples/checksummer/checksummer_user.c:30-112, verbatim, extracted and compiled
by `make -C oracle ref`; oracle/ref.py).  Here the restatement
(oracle/csum_oracle.c) must equal it byte for byte: on the known answers, on
20,000 randomized frames over every branch of :34-55 with odd starts, iterations
-3..7919, both actions, 1-4 interfaces and every ingress, and on the committed
golden fixtures (which tests/golden/make_golden.py generates from it).
Skipped only where neither the built library nor a reference checkout exists.
"""
import os

import numpy as np
import pytest

from oracle import csum_oracle as O
from oracle import ref as R
from xsknf_amd import frames

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def ref():
    if not R.available() and not R.build():
        pytest.skip("reference not compiled here (no oracle/_ref and no reference checkout)")
    return R.load()


def test_ref_exports(ref):
    for sym in ("xsknf_packet_processor", "ref_set_options", "ref_packet_processor", "ref_process_batch",
                "ref_time_batch"):
        assert hasattr(ref, sym)


def test_known_answers_from_the_reference(ref):
    from tests.test_oracle import KATS
    for name, frame, kw, ret, sl, chk in KATS:
        f = bytearray(frame)
        orig = bytes(f)
        assert R.packet_processor(f, **kw) == ret, name
        if chk is None:
            assert bytes(f) == orig, name
        else:
            assert bytes(f[sl[0]:sl[1]]).hex() == chk, name
            assert all(sl[0] <= i < sl[1] for i in range(len(f)) if f[i] != orig[i]), name


def _group(rng, n, max_len, seed):
    """n frames packed at random (about half odd) offsets, every branch mixed in."""
    lens = rng.integers(0, max_len + 1, size=n).astype(np.uint32)
    lens[: n // 10] = rng.integers(0, 64, size=n // 10)          # the short-frame boundaries
    b = frames.unaligned_batch(n, lens, seed=seed)
    frames.inject_edge_cases(b, 0.35, seed=seed + 1)
    offs = b.frame_offsets()
    # extra: ihl 0..15 on well-formed frames (udp may overlap the IP header or run past the end)
    for i in rng.choice(n, size=n // 8, replace=False):
        if b.descs["len"][i] >= 15:
            o = int(offs[i])
            b.umem[o + 14] = (b.umem[o + 14] & 0xF0) | int(rng.integers(0, 16))
    return b


# (iterations, max frame length): the repeated sum wraps u32 at large counts,
# so the 7919-iteration group keeps its frames short (CPU time)
ITERS = [(-3, 1600), (-1, 9100), (0, 1600), (1, 9100), (1, 1600), (2, 1600), (3, 600), (5, 1600),
         (7, 9100), (50, 1600), (127, 600), (7919, 256)]


def test_oracle_equals_reference_on_20000_frames(ref):
    rng = np.random.default_rng(0x58534B4E)
    total = 0
    for g in range(40):
        it, max_len = ITERS[g % len(ITERS)]
        kw = dict(iters=it, action=int(g % 2), nif=int(1 + g % 4), ingress=int(rng.integers(0, 4)))
        kw["ingress"] %= 8
        b = _group(rng, 500, max_len, seed=1000 + g)
        a, c = b.copy(), b.copy()
        va = R.process_batch(a.umem, a.descs, **kw)
        vc = O.c_process_batch(c.umem, c.descs, **kw)
        assert np.array_equal(va, vc), (g, kw, np.nonzero(va != vc)[0][:8])
        assert np.array_equal(a.umem, c.umem), (g, kw, np.nonzero(a.umem != c.umem)[0][:8])
        total += b.n
        # every branch was exercised: forwards, drops, untouched non-IP/non-UDP
        if kw["action"] == O.DROP:
            assert (va == -1).any() and (va == 0).any()
    assert total == 20000


def test_numpy_closed_form_equals_reference(ref):
    rng = np.random.default_rng(7)
    for it in (-2, 0, 1, 3, 7919):
        b = _group(rng, 300, 1600 if it < 100 else 200, seed=77 + it)
        a = b.copy()
        va = R.process_batch(a.umem, a.descs, iters=it, action=O.REDIRECT, nif=3, ingress=1)
        offs = b.frame_offsets()
        for i in range(b.n):
            o, L = int(offs[i]), int(b.descs["len"][i])
            f = b.umem[o:o + L].copy()
            r = O.np_packet_processor(f, iters=it, action=O.REDIRECT, nif=3, ingress=1)
            assert r == va[i]
            assert np.array_equal(f, a.umem[o:o + L])


def test_golden_fixtures_are_the_references_output(ref):
    from tests.test_golden import NAMES, case
    assert NAMES
    for name in NAMES:
        umem, descs, kw, v_exp, u_exp = case(name)
        v = R.process_batch(umem, descs, **kw)
        assert np.array_equal(v, v_exp), name
        assert np.array_equal(umem, u_exp), name


def test_golden_fixtures_record_their_generator():
    g = np.load(os.path.join(HERE, "golden", "checksummer_golden.npz"))
    assert "meta__generator" in g.files
    assert bytes(g["meta__generator"]).decode().startswith("reference")
