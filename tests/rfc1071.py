"""An independent receive-side check of the written UDP checksums (RFC 768 / 1071).

The reference's traffic arrives with NIC-computed, RFC-correct UDP checksums
(tests/gen-traffic.lua:120 offloads them to the generator's NIC), so whatever
the checksummer writes must pass the standard receive-side verification
wherever its single fold (checksummer_user.c:105-106) loses no carry:

    V = one's-complement sum (fully folded) of the pseudo-header
        {src, dst, 0x0011, udp.len} and the UDP bytes [u, len) with the check
        the kernel wrote                                     ==  0xFFFF

Where the fold does lose its carry the reference writes the RFC value + 1
(mod 2^16), so V = 0xFFFF +' 1 = 0x0001.  This is written from the RFC, not
from the oracle: it pins the checksummer's output to the convention of the
reference's own traffic for every frame, at full batch sizes.  The sum is
byte-order independent (RFC 1071 section 2(B)); it is taken here over
little-endian words, with an odd tail byte as the low byte of a zero-padded
word.  Test infrastructure (torch on the batch's device), never product code.
"""
from __future__ import annotations

import numpy as np


def _fold(s):
    while bool((s >> 16).any()):
        s = (s & 0xFFFF) + (s >> 16)
    return s


def verify(umem, offs: np.ndarray, lens: np.ndarray, *, chunk_frames: int = 16384):
    """V per frame for the well-formed IPv4/UDP frames with ihl 5 (udp at 34).

    `umem`: uint8 torch tensor (any device); `offs`/`lens`: numpy frame offsets
    and lengths.  Returns (index array of the frames checked, V as numpy int64).
    Frames that are not IPv4/UDP with ihl 5 and len >= 42 are skipped."""
    import torch

    dev = umem.device
    offs = np.asarray(offs, dtype=np.int64)
    lens = np.asarray(lens, dtype=np.int64)
    cand = np.flatnonzero(lens >= 42)
    if cand.size == 0:
        return cand, np.zeros(0, dtype=np.int64)
    o_t = torch.from_numpy(offs[cand]).to(dev)
    hdr = umem[o_t[:, None] + torch.arange(42, device=dev)[None, :]].to(torch.int64)
    ok = ((hdr[:, 12] == 0x08) & (hdr[:, 13] == 0x00) & (hdr[:, 14] == 0x45) & (hdr[:, 23] == 17)).cpu().numpy()
    idx = cand[ok]
    out = np.zeros(idx.size, dtype=np.int64)
    if idx.size == 0:
        return idx, out
    L = lens[idx]
    pos = np.arange(idx.size)
    for length in np.unique(L):
        sel = pos[L == length]
        for c0 in range(0, sel.size, chunk_frames):
            s_idx = sel[c0:c0 + chunk_frames]
            o = torch.from_numpy(offs[idx[s_idx]]).to(dev)
            f = umem[o[:, None] + torch.arange(int(length), device=dev)[None, :]].to(torch.int64)
            le = lambda i: f[:, i] | (f[:, i + 1] << 8)   # noqa: E731
            s = le(26) + le(28) + le(30) + le(32) + 0x1100 + le(38)
            seg = f[:, 34:]
            s = s + seg[:, 0::2].sum(dim=1) + (seg[:, 1::2].sum(dim=1) << 8)
            out[s_idx] = _fold(s).cpu().numpy()
    return idx, out
