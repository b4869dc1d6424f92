#!/usr/bin/env python3
"""Regenerate tests/golden/checksummer_golden.npz (regression fixtures).

Inputs are seeded synthetic rx batches (xsknf_amd.frames, with edge cases);
expected outputs come from the C oracle (oracle/csum_oracle.c), itself pinned by
the SURVEY.md Appendix C known answers (tests/test_oracle.py).  Stored compactly:
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
from xsknf_amd import frames  # noqa: E402

CASES = [
    # name, layout, n, length, (iters, action, nif, ingress), edge fraction, seed
    ("imix_unaligned_redirect", "unaligned", 240, "imix", (1, O.REDIRECT, 1, 0), 0.15, 101),
    ("mixed_unaligned_drop_iter5", "unaligned", 160, "mixed", (5, O.DROP, 1, 0), 0.2, 202),
    ("imix_aligned_nif3_iter-1", "aligned", 48, "imix", (-1, O.REDIRECT, 3, 2), 0.25, 303),
    ("jumbo_unaligned_iter50", "unaligned", 12, 9000, (50, O.REDIRECT, 2, 1), 0.0, 404),
]


def build(layout, n, length, seed):
    if length == "mixed":
        length = np.random.default_rng(seed).integers(0, 1600, size=n).astype(np.uint32)
    if layout == "aligned":
        return frames.aligned_batch(n, length, chunk=2048, seed=seed)
    return frames.unaligned_batch(n, length, seed=seed)


def main():
    out = {}
    for name, layout, n, length, (it, act, nif, ing), edge, seed in CASES:
        b = build(layout, n, length, seed)
        if edge:
            frames.inject_edge_cases(b, edge, seed=seed + 1)
        ref = b.copy()
        v = O.c_process_batch(ref.umem, ref.descs, ingress=ing, iters=it, action=act, nif=nif)
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
