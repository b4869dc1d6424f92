"""Synthetic rx batches: a UMEM byte buffer plus an array of xdp_desc.

Frames follow the reference's traffic generator (tests/gen-traffic.lua:16,92-100):
Ethernet 0a:00:00:00:00:01 -> 0a:00:00:00:00:00, IPv4 (ihl 5, proto 17)
10.0.0.x -> 172.0.0.1 with x spread over 256 flows, UDP 5000 -> 80, random payload.

UMEM layouts (reference src/xsknf.c:928-939, 165-172 and linux/if_xdp.h):
* aligned:   frame i lives in chunk i of `chunk` bytes, data at +`headroom`
             (the kernel's XDP_PACKET_HEADROOM of 256); desc.addr = i*chunk + headroom.
* unaligned: frames packed back to back at arbitrary (also odd) byte offsets;
             desc.addr = base | (offset << 48) with base + offset = frame start,
             the encoding xsk_umem__add_offset_to_addr() undoes (src/xsknf.c:659).

Host (numpy) builders feed the parity tests; device (torch) builders make the
1M-frame bench batches directly in HBM.
"""
from __future__ import annotations

import numpy as np

DESC_DTYPE = np.dtype([("addr", "<u8"), ("len", "<u4"), ("options", "<u4")])
SEED = 0x58534B4E           # "XSKN"
HEADROOM = 256              # XDP_PACKET_HEADROOM
CHUNK = 2048
HDR_LEN = 42
OFFSET_SHIFT = 48
IMIX_SIZES = (64, 570, 1500)
IMIX_WEIGHTS = (7, 4, 1)

_ETH = bytes.fromhex("0a0000000000" "0a0000000001" "0800")


def headers(lens: np.ndarray, flows: np.ndarray) -> np.ndarray:
    """(n, 42) uint8 Eth/IPv4/UDP headers for frames of the given lengths."""
    lens = np.asarray(lens, dtype=np.int64)
    n = lens.shape[0]
    h = np.zeros((n, HDR_LEN), dtype=np.uint8)
    h[:, 0:14] = np.frombuffer(_ETH, dtype=np.uint8)
    h[:, 14] = 0x45
    iplen = np.clip(lens - 14, 0, 0xFFFF)
    h[:, 16] = iplen >> 8
    h[:, 17] = iplen & 0xFF
    h[:, 22] = 64           # ttl
    h[:, 23] = 17           # UDP
    h[:, 26:30] = [10, 0, 0, 0]
    h[:, 29] = np.asarray(flows, dtype=np.uint8)
    h[:, 30:34] = [172, 0, 0, 1]
    h[:, 34:36] = [0x13, 0x88]   # 5000
    h[:, 36:38] = [0x00, 0x50]   # 80
    udplen = np.clip(lens - 34, 0, 0xFFFF)
    h[:, 38] = udplen >> 8
    h[:, 39] = udplen & 0xFF
    return h


def imix_lengths(n: int, rng: np.random.Generator) -> np.ndarray:
    """IMIX 64/570/1500 in ratio 7:4:1, shuffled."""
    w = np.asarray(IMIX_WEIGHTS, dtype=np.float64)
    return rng.choice(np.asarray(IMIX_SIZES, dtype=np.uint32), size=n, p=w / w.sum())


class HostBatch:
    """A host-resident rx batch: `umem` (uint8) and `descs` (DESC_DTYPE)."""

    def __init__(self, umem: np.ndarray, descs: np.ndarray, layout: str):
        self.umem = umem
        self.descs = descs
        self.layout = layout

    @property
    def n(self) -> int:
        return int(self.descs.shape[0])

    def frame_offsets(self) -> np.ndarray:
        a = self.descs["addr"]
        return (a & np.uint64((1 << OFFSET_SHIFT) - 1)) + (a >> np.uint64(OFFSET_SHIFT))

    def frame(self, i: int) -> np.ndarray:
        o = int(self.frame_offsets()[i])
        return self.umem[o:o + int(self.descs["len"][i])]

    def copy(self) -> "HostBatch":
        return HostBatch(self.umem.copy(), self.descs.copy(), self.layout)


def _lens(n, length, rng):
    if isinstance(length, str):
        if length != "imix":
            raise ValueError(length)
        return imix_lengths(n, rng)
    arr = np.asarray(length, dtype=np.uint32)
    if arr.ndim == 0:
        return np.full(n, int(arr), dtype=np.uint32)
    if arr.shape[0] != n:
        raise ValueError("lens must have n entries")
    return arr


def aligned_batch(n: int, length, *, chunk: int = CHUNK, headroom: int = HEADROOM,
                  seed: int = SEED) -> HostBatch:
    rng = np.random.default_rng(seed)
    lens = _lens(n, length, rng)
    if n and int(lens.max()) + headroom > chunk:
        raise ValueError("frame does not fit its chunk")
    umem = rng.integers(0, 256, size=n * chunk, dtype=np.uint8)
    flows = rng.integers(0, 256, size=n)
    hv = umem.reshape(n, chunk)
    h = headers(lens, flows)
    hv[:, headroom:headroom + HDR_LEN] = np.where(
        np.arange(HDR_LEN)[None, :] < lens[:, None], h, hv[:, headroom:headroom + HDR_LEN])
    descs = np.zeros(n, dtype=DESC_DTYPE)
    descs["addr"] = np.arange(n, dtype=np.uint64) * np.uint64(chunk) + np.uint64(headroom)
    descs["len"] = lens
    return HostBatch(umem, descs, "aligned")


def unaligned_batch(n: int, length, *, seed: int = SEED, max_gap: int = 7,
                    max_offset: int = 255) -> HostBatch:
    """Frames packed back to back with 0..max_gap random gap bytes, so about half
    of them start at odd addresses; addr = base | (offset << 48)."""
    rng = np.random.default_rng(seed)
    lens = _lens(n, length, rng).astype(np.uint64)
    gaps = rng.integers(0, max_gap + 1, size=n).astype(np.uint64)
    starts = np.cumsum(gaps + lens) - lens
    total = int(starts[-1] + lens[-1]) + 16 if n else 16
    umem = rng.integers(0, 256, size=total, dtype=np.uint8)
    flows = rng.integers(0, 256, size=n)
    h = headers(lens.astype(np.int64), flows)
    cols = np.arange(HDR_LEN, dtype=np.uint64)
    idx = starts[:, None] + cols[None, :]
    mask = cols[None, :] < lens[:, None]
    umem[idx[mask]] = h[mask]
    offs = np.minimum(rng.integers(0, max_offset + 1, size=n).astype(np.uint64), starts)
    descs = np.zeros(n, dtype=DESC_DTYPE)
    descs["addr"] = (starts - offs) | (offs << np.uint64(OFFSET_SHIFT))
    descs["len"] = lens.astype(np.uint32)
    return HostBatch(umem, descs, "unaligned")


def inject_edge_cases(b: HostBatch, frac: float, *, seed: int = SEED + 1) -> np.ndarray:
    """Mutate ~frac of the frames into the branches the reference distinguishes
    (checksummer_user.c:34-55): short frames, non-IPv4 / VLAN ethertypes,
    non-UDP protocols, every ihl nibble, odd lengths, random garbage.
    Lengths only shrink and writes stay inside [start, start+len), so packed
    (unaligned) neighbours are never touched.  Returns the indices."""
    rng = np.random.default_rng(seed)
    n = b.n
    k = int(round(n * frac))
    if k == 0:
        return np.zeros(0, dtype=np.int64)
    sel = rng.choice(n, size=k, replace=False)
    offs = b.frame_offsets()
    for j, i in enumerate(sel):
        o = int(offs[i])
        L = int(b.descs["len"][i])
        kind = j % 9
        if kind == 0:      # truncated below each header boundary
            b.descs["len"][i] = min(L, int(rng.choice([0, 1, 13, 14, 20, 33, 34, 35, 41, 42])))
        elif kind == 1 and L >= 14:    # non-IPv4 ethertypes (IPv6, VLAN, ARP)
            b.umem[o + 12:o + 14] = [[0x86, 0xDD], [0x81, 0x00], [0x08, 0x06]][j % 3]
        elif kind == 2 and L >= 24:    # non-UDP (TCP, ICMP, garbage)
            b.umem[o + 23] = [6, 1, 255][j % 3]
        elif kind == 3 and L >= 15:    # every ihl value (udp header may overlap the IP header)
            b.umem[o + 14] = (b.umem[o + 14] & 0xF0) | int(rng.integers(0, 16))
        elif kind == 4:    # odd lengths (trailing byte)
            b.descs["len"][i] = max(1, L - 1 - 2 * int(rng.integers(0, 8)))
        elif kind == 5 and L >= 34:    # ihl that pushes udp past the end
            b.umem[o + 14] = 0x4F
            b.descs["len"][i] = min(L, int(rng.integers(34, 82)))
        elif kind == 6:    # all-0xff payload (sum wraps, fold edge)
            if L > 42:
                b.umem[o + 42:o + L] = 0xFF
        elif kind == 7 and L >= 24:    # random garbage frame
            b.umem[o:o + L] = rng.integers(0, 256, size=L, dtype=np.uint8)
            b.umem[o + 12:o + 14] = [0x08, 0x00]
            b.umem[o + 23] = 17
        elif kind == 8:    # minimal legal frames around the udp boundary
            b.descs["len"][i] = min(L, int(rng.choice([42, 43, 44, 50, 51])))
    return np.sort(sel)


# ---- NIC checksum offload ------------------------------------------------

def _offload(umem, starts, lens, budget: int = 1 << 24) -> int:
    """UDP checksums as a NIC's transmit offload fills them in (RFC 768: the
    one's-complement sum, fully folded, of the pseudo-header {src, dst, 17,
    udp.len} and the UDP bytes with the check as 0; a result of 0 is sent as
    0xFFFF), written big-endian at frame offset 40.  Only well-formed frames
    are touched: Ethernet/IPv4, ihl 5, protocol 17, len >= 42.  `umem` is a
    uint8 torch tensor (any device), `starts` / `lens` int64 tensors on the same
    device.  Returns the number of frames given a check."""
    import torch

    dev = umem.device
    n = int(starts.shape[0])
    done = 0
    if n == 0:
        return 0
    maxlen = int(lens.max())
    step = max(256, budget // max(64, maxlen))
    for a in range(0, n, step):
        st, ln = starts[a:a + step], lens[a:a + step]
        width = max(42, int(ln.max()))
        col = torch.arange(width, device=dev)
        idx = (st[:, None] + col[None, :]).clamp_(max=umem.numel() - 1)
        f = umem[idx].to(torch.int64)
        f = torch.where(col[None, :] < ln[:, None], f, torch.zeros_like(f))
        ok = ((ln >= 42) & (f[:, 12] == 0x08) & (f[:, 13] == 0x00) & (f[:, 14] == 0x45) & (f[:, 23] == 17))
        be = lambda i: (f[:, i] << 8) | f[:, i + 1]   # noqa: E731
        s = be(26) + be(28) + be(30) + be(32) + 17 + be(38)
        udp = f[:, 34:].clone()
        udp[:, 6:8] = 0                               # the check itself counts as 0
        s = s + (udp[:, 0::2].sum(dim=1) << 8) + udp[:, 1::2].sum(dim=1)
        for _ in range(4):
            s = (s & 0xFFFF) + (s >> 16)
        c = (~s) & 0xFFFF
        c = torch.where(c == 0, torch.full_like(c, 0xFFFF), c)
        sel = ok.nonzero().squeeze(1)
        if sel.numel():
            at = st[sel] + 40
            umem[at] = (c[sel] >> 8).to(torch.uint8)
            umem[at + 1] = (c[sel] & 0xFF).to(torch.uint8)
        done += int(sel.numel())
    return done


def offload_checks_host(b: HostBatch) -> int:
    """Give a host batch's well-formed frames the UDP checksums a NIC's offload
    computes (the reference's traffic: tests/gen-traffic.lua:120,
    `bufs:offloadUdpChecksums()`), in place.  Apply before inject_edge_cases."""
    import torch

    return _offload(torch.from_numpy(b.umem), torch.from_numpy(b.frame_offsets().astype(np.int64)),
                    torch.from_numpy(b.descs["len"].astype(np.int64)))


def offload_checks_device(umem, descs) -> int:
    """offload_checks_host for a device batch (umem uint8, descs int64 (n, 2)
    holding struct xdp_desc, as device_batch returns them)."""
    import torch

    addr = descs[:, 0]
    mask = (1 << OFFSET_SHIFT) - 1
    starts = (addr & mask) + ((addr >> OFFSET_SHIFT) & 0xFFFF)
    lens = descs[:, 1] & 0xFFFFFFFF
    return _offload(umem, starts.to(torch.int64), lens.to(torch.int64))


# ---- device builders (torch) ---------------------------------------------

def device_batch(n: int, length, *, layout: str = "aligned", chunk: int = CHUNK,
                 headroom: int = HEADROOM, seed: int = SEED, device="cuda"):
    """Build an rx batch directly in device memory.

    Returns (umem uint8 tensor, descs int64 tensor of shape (n, 2) whose bytes
    are exactly struct xdp_desc, lens numpy array)."""
    import torch

    rng = np.random.default_rng(seed)
    lens = _lens(n, length, rng).astype(np.int64)
    flows = rng.integers(0, 256, size=n)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    if layout == "aligned":
        if int(lens.max()) + headroom > chunk:
            raise ValueError("frame does not fit its chunk")
        starts = np.arange(n, dtype=np.int64) * chunk + headroom
        addr = starts.astype(np.uint64)
        total = n * chunk
    elif layout == "unaligned":
        gaps = rng.integers(0, 8, size=n).astype(np.int64)
        starts = np.cumsum(gaps + lens) - lens
        total = int(starts[-1] + lens[-1]) + 16
        offs = np.minimum(rng.integers(0, 256, size=n), starts).astype(np.uint64)
        addr = (starts.astype(np.uint64) - offs) | (offs << np.uint64(OFFSET_SHIFT))
    else:
        raise ValueError(layout)
    umem = torch.randint(0, 256, (total,), dtype=torch.uint8, device=device, generator=g)
    h = torch.from_numpy(headers(lens, flows)).to(device)
    hl = min(HDR_LEN, int(lens.min()))
    if layout == "aligned":
        umem.view(n, chunk)[:, headroom:headroom + hl] = h[:, :hl]
    else:
        st = torch.from_numpy(starts).to(device)
        idx = st[:, None] + torch.arange(hl, device=device)[None, :]
        umem[idx.reshape(-1)] = h[:, :hl].reshape(-1)
    d = np.zeros(n, dtype=DESC_DTYPE)
    d["addr"] = addr
    d["len"] = lens.astype(np.uint32)
    descs = torch.from_numpy(d.view(np.int64).reshape(n, 2).copy()).to(device)
    return umem, descs, lens
