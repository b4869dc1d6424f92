"""One process over several devices: the C host's multi-device calls (include/xsknf_gpu.h).

A global batch that starts on one device -- BASELINE config 4 -- is split into
contiguous descriptor ranges balanced by frame bytes (xsknf_gpu_shard_plan, the
same cuts as shard.shard_by_bytes), every range's UMEM span and rebased
descriptors move from the root device to their own by grouped RCCL ncclSend /
ncclRecv, each device checksums its shard on its own stream, and the counters
are summed by an RCCL all-reduce (xsknf_gpu_multi_*, xsknf_amd/csrc/multi.hip).
This is the path a C host takes (no torch.distributed: one process, one RCCL
communicator per device); bench.py's ranks are the one-process-per-GPU path.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .checksummer import ChecksummerOptions

COUNTER_NAMES = ("frames", "bytes", "drop", "forward", "checks_sum", "checks_weighted")


def _descs_array(descs) -> np.ndarray:
    d = np.ascontiguousarray(descs)
    if d.dtype.itemsize != 16:
        raise ValueError("descriptors must be struct xdp_desc records (16 bytes)")
    return d


def shard_plan(descs, nshards: int, umem_size: int):
    """([(lo, hi)] frame ranges, [(b0, b1)] UMEM spans), from the C library (no GPU)."""
    lib = _lib.load()
    d = _descs_array(descs)
    n = int(d.shape[0])
    bounds = np.zeros(nshards + 1, dtype=np.uint64)
    spans = np.zeros(2 * nshards, dtype=np.uint64)
    _lib.check(lib.xsknf_gpu_shard_plan(d.ctypes.data if n else None, n, umem_size, nshards,
                                        bounds.ctypes.data, spans.ctypes.data), "xsknf_gpu_shard_plan")
    return ([(int(bounds[k]), int(bounds[k + 1])) for k in range(nshards)],
            [(int(spans[2 * k]), int(spans[2 * k + 1])) for k in range(nshards)])


def shard_rebase(descs, b0: int, umem_size: int) -> np.ndarray:
    """The descriptors relative to b0, from the C library (no GPU)."""
    lib = _lib.load()
    d = _descs_array(descs)
    out = np.zeros_like(d)
    n = int(d.shape[0])
    _lib.check(lib.xsknf_gpu_shard_rebase(d.ctypes.data if n else None, n, b0, umem_size,
                                          out.ctypes.data if n else None), "xsknf_gpu_shard_rebase")
    return out


def pack_plan(descs, bounds, umem_addr: int, umem_size: int):
    """(packed descriptors, [packed bytes per shard]) of xsknf_gpu_shard_pack_plan
    for shard bounds [b0 = 0, b1, ..., n], from the C library (no GPU)."""
    lib = _lib.load()
    d = _descs_array(descs)
    n = int(d.shape[0])
    b = np.ascontiguousarray(np.asarray(bounds, dtype=np.uint64))
    out = np.zeros_like(d)
    sizes = np.zeros(b.size - 1, dtype=np.uint64)
    _lib.check(lib.xsknf_gpu_shard_pack_plan(d.ctypes.data if n else None, n, umem_addr, umem_size, b.size - 1,
                                             b.ctypes.data, out.ctypes.data if n else None, sizes.ctypes.data),
               "xsknf_gpu_shard_pack_plan")
    return out, [int(x) for x in sizes]


class MultiDevice:
    """xsknf_gpu_multi over `devices` (HIP device ids, each once)."""

    def __init__(self, devices):
        self._lib = _lib.load()
        self.devices = [int(x) for x in devices]
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        _lib.check(self._lib.xsknf_gpu_multi_create(ctypes.byref(h), arr, len(self.devices)),
                   "xsknf_gpu_multi_create")
        self._h = h

    def close(self):
        if self._h:
            self._lib.xsknf_gpu_multi_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def scatter(self, root: int, umem_ptr: int, umem_size: int, descs) -> float:
        """Move every shard of the batch (UMEM at device pointer umem_ptr on
        devices[root], descriptors in host memory) to its device; seconds."""
        d = _descs_array(descs)
        secs = ctypes.c_double()
        _lib.check(self._lib.xsknf_gpu_multi_scatter(self._h, root, ctypes.c_void_p(umem_ptr), umem_size,
                                                     d.ctypes.data if d.shape[0] else None, int(d.shape[0]),
                                                     ctypes.byref(secs)), "xsknf_gpu_multi_scatter")
        return secs.value

    def scatter_packed(self, root: int, umem_ptr: int, umem_size: int, descs) -> float:
        """As scatter(), moving only the frames' bytes (xsknf_gpu_multi_scatter_packed:
        packed into 16-byte slots on the root first); seconds."""
        d = _descs_array(descs)
        secs = ctypes.c_double()
        _lib.check(self._lib.xsknf_gpu_multi_scatter_packed(self._h, root, ctypes.c_void_p(umem_ptr), umem_size,
                                                            d.ctypes.data if d.shape[0] else None,
                                                            int(d.shape[0]), ctypes.byref(secs)),
                   "xsknf_gpu_multi_scatter_packed")
        return secs.value

    def return_results(self, umem_ptr: int, verdicts_ptr: int, opts: ChecksummerOptions | None = None,
                       num_interfaces: int = 1, ingress_ifindex: int = 0, frame_len_max: int = 0,
                       frame_len_mean: int = 0):
        """xsknf_gpu_multi_return: every shard's results (records-only pass) back to
        the root's UMEM at umem_ptr and int32 verdicts at verdicts_ptr (device
        pointers on the root); (each device's milliseconds, seconds in all)."""
        o = opts or ChecksummerOptions()
        c = _lib.CsumOpts(o.csum_iterations, o.action, num_interfaces, 0)
        ms = (ctypes.c_float * len(self.devices))()
        secs = ctypes.c_double()
        _lib.check(self._lib.xsknf_gpu_multi_return(self._h, ingress_ifindex, ctypes.byref(c), frame_len_max,
                                                    frame_len_mean, ctypes.c_void_p(umem_ptr),
                                                    ctypes.c_void_p(verdicts_ptr), ms, ctypes.byref(secs)),
                   "xsknf_gpu_multi_return")
        return list(ms), secs.value

    def process(self, opts: ChecksummerOptions | None = None, num_interfaces: int = 1, ingress_ifindex: int = 0,
                frame_len_max: int = 0, frame_len_mean: int = 0):
        """Checksum every shard; returns each device's milliseconds."""
        o = opts or ChecksummerOptions()
        c = _lib.CsumOpts(o.csum_iterations, o.action, num_interfaces, 0)
        ms = (ctypes.c_float * len(self.devices))()
        _lib.check(self._lib.xsknf_gpu_multi_process(self._h, ingress_ifindex, ctypes.byref(c), frame_len_max,
                                                     frame_len_mean, ms), "xsknf_gpu_multi_process")
        return list(ms)

    def counters(self) -> dict:
        out = np.zeros(_lib.MULTI_COUNTERS, dtype=np.uint64)
        _lib.check(self._lib.xsknf_gpu_multi_counters(self._h, out.ctypes.data), "xsknf_gpu_multi_counters")
        return dict(zip(COUNTER_NAMES, (int(x) for x in out)))

    def shard_info(self, k: int) -> dict:
        info = _lib.ShardInfo()
        _lib.check(self._lib.xsknf_gpu_multi_shard_info(self._h, k, ctypes.byref(info)), "xsknf_gpu_multi_shard_info")
        return {name: getattr(info, name) for name, _ in info._fields_}

    def fetch(self, k: int, descs: bool = False):
        """(UMEM span bytes, verdicts) of shard k in host memory, and its rebased
        descriptors third if `descs`."""
        info = self.shard_info(k)
        umem = np.empty(info["span_hi"] - info["span_lo"], dtype=np.uint8)
        nf = info["frame_hi"] - info["frame_lo"]
        v = np.empty(nf, dtype=np.int32)
        d = np.empty(nf if descs else 0, dtype=[("addr", "<u8"), ("len", "<u4"), ("options", "<u4")])
        _lib.check(self._lib.xsknf_gpu_multi_fetch(self._h, k, umem.ctypes.data if umem.size else None,
                                                   d.ctypes.data if d.size else None,
                                                   v.ctypes.data if v.size else None), "xsknf_gpu_multi_fetch")
        return (umem, v, d) if descs else (umem, v)


def expected_counters(umem: np.ndarray, descs, verdicts: np.ndarray) -> dict:
    """The same counters computed on the host over a whole batch (its UMEM after
    the pass, its descriptors and verdicts): what xsknf_gpu_multi_counters must
    return for that batch however it is sharded."""
    d = _descs_array(descs)
    a = d["addr"].astype(np.uint64)
    off = ((a & np.uint64((1 << 48) - 1)) + (a >> np.uint64(48))).astype(np.int64)
    ln = d["len"].astype(np.int64)
    ok = (ln >= 42) & (off <= umem.size) & (ln <= umem.size - off)
    o = off[ok]
    c = umem[o + 40].astype(np.uint64) | (umem[o + 41].astype(np.uint64) << np.uint64(8))
    w = (o.astype(np.uint64) % np.uint64(65521)) + np.uint64(1)
    return {"frames": int(d.shape[0]), "bytes": int(ln.sum()), "drop": int((verdicts == -1).sum()),
            "forward": int((verdicts >= 0).sum()), "checks_sum": int(c.sum(dtype=np.uint64)),
            "checks_weighted": int((c * w).sum(dtype=np.uint64))}
