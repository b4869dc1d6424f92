#!/usr/bin/env python3
"""Regenerate tests/golden/checksummer_golden.npz (regression fixtures).

Inputs are seeded synthetic rx batches (xsknf_amd.frames, with edge cases);
expected outputs come from the REFERENCE's own xsknf_packet_processor()
(examples/checksummer/checksummer_user.c:30-112), compiled here from its verbatim
text by `make -C oracle ref` (oracle/ref_extract.sh, oracle/ref_harness.c) and
called in process_batch_1if()'s batch loop (src/xsknf.c:654-672).  The C
restatement must give the same bytes (checked here before writing, and by
tests/test_golden.py / tests/test_ref_pin.py).  Stored compactly:
the input UMEM, the descriptors, the options, the expected verdicts and the
(offset, byte) pairs the path must change.  Run from the repo root:

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import csum_oracle as O  # noqa: E402
from oracle import ref as R  # noqa: E402
from xsknf_amd import frames  # noqa: E402

CASES = [
    # name, layout, n, length, (iters, action, nif, ingress), edge fraction, seed
    ("imix_unaligned_redirect", "unaligned", 240, "imix", (1, O.REDIRECT, 1, 0), 0.15, 101),
    ("mixed_unaligned_drop_iter5", "unaligned", 160, "mixed", (5, O.DROP, 1, 0), 0.2, 202),
    ("imix_aligned_nif3_iter-1", "aligned", 48, "imix", (-1, O.REDIRECT, 3, 2), 0.25, 303),
    ("jumbo_unaligned_iter50", "unaligned", 12, 9000, (50, O.REDIRECT, 2, 1), 0.0, 404),
    ("ihl_overlap_unaligned_nif4", "unaligned", 96, "ihl", (2, O.REDIRECT, 4, 3), 0.1, 505),
    ("short_unaligned_iter7919", "unaligned", 64, "short", (7919, O.DROP, 1, 0), 0.2, 606),
]


def build(layout, n, length, seed):
    if isinstance(length, str) and length == "mixed":
        length = np.random.default_rng(seed).integers(0, 1600, size=n).astype(np.uint32)
    elif isinstance(length, str) and length in ("ihl", "short"):
        length = np.random.default_rng(seed).integers(34, 300, size=n).astype(np.uint32)
    if layout == "aligned":
        return frames.aligned_batch(n, length, chunk=2048, seed=seed)
    return frames.unaligned_batch(n, length, seed=seed)


def main():
    if not R.build():
        sys.exit("make_golden: the reference is not compiled here (oracle/_ref); nothing written")
    out = {"meta__generator": np.frombuffer(
        b"reference: checksummer_user.c:30-112 compiled by oracle/ref_extract.sh + ref_harness.c", dtype=np.uint8)}
    for name, layout, n, length, (it, act, nif, ing), edge, seed in CASES:
        b = build(layout, n, length, seed)
        if edge:
            frames.inject_edge_cases(b, edge, seed=seed + 1)
        if name.startswith("ihl_overlap"):
            # every ihl nibble: the udp header overlaps the IP header (ihl 2/3
            # put the check on the addresses the pseudo-header reads) or leaves the frame
            offs = b.frame_offsets()
            for i in range(b.n):
                if b.descs["len"][i] >= 15:
                    o = int(offs[i])
                    b.umem[o + 14] = (b.umem[o + 14] & 0xF0) | (i % 16)
        ref = b.copy()
        v = R.process_batch(ref.umem, ref.descs, ingress=ing, iters=it, action=act, nif=nif)
        chk = b.copy()
        vo = O.c_process_batch(chk.umem, chk.descs, ingress=ing, iters=it, action=act, nif=nif)
        if not (np.array_equal(v, vo) and np.array_equal(chk.umem, ref.umem)):
            sys.exit(f"make_golden: the restatement differs from the reference on {name}; nothing written")
        pos = np.nonzero(ref.umem != b.umem)[0].astype(np.uint32)
        out[f"{name}__umem"] = b.umem
        out[f"{name}__descs"] = b.descs.view(np.uint8).reshape(-1, 16)
        out[f"{name}__opts"] = np.array([it, act, nif, ing], dtype=np.int64)
        out[f"{name}__verdicts"] = v
        out[f"{name}__pos"] = pos
        out[f"{name}__val"] = ref.umem[pos]
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "checksummer_golden.npz")
    np.savez_compressed(path, **out)
    print(path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
