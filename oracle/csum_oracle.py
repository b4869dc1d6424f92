"""Python side of the oracle -- TEST INFRASTRUCTURE ONLY (see csum_oracle.c).

Three independent restatements of reference examples/checksummer/checksummer_user.c:30-112:
  * `c_process_batch`   the C restatement (literal per-word loop), via ctypes;
  * `py_packet_processor` a pure-Python literal transliteration (small inputs);
  * `np_packet_processor` the closed byte-parity form in numpy,
    which is how the GPU kernel computes, but written independently of it.
All three are cross-checked against each other (tests/test_oracle.py) and pinned
to the reference's own function compiled here (oracle/ref.py, tests/test_ref_pin.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libcsum_oracle.so")

REDIRECT = 0
DROP = 1


class _Opts(ctypes.Structure):
    _fields_ = [("csum_iterations", ctypes.c_int32), ("action", ctypes.c_int32),
                ("num_interfaces", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = ctypes.CDLL(LIB_PATH)
        lib.oracle_packet_processor.restype = ctypes.c_int
        lib.oracle_packet_processor.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint,
                                                ctypes.POINTER(_Opts)]
        lib.oracle_process_batch.restype = None
        lib.oracle_process_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.POINTER(_Opts),
                                             ctypes.c_void_p, ctypes.c_uint32]
        lib.oracle_time_batch.restype = ctypes.c_double
        lib.oracle_time_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                          ctypes.POINTER(_Opts), ctypes.c_void_p,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int]
        _lib = lib
    return _lib


def _opts(iters, action, nif):
    return _Opts(int(iters), int(action), int(nif), 0)


def c_packet_processor(frame: bytearray, ingress=0, iters=1, action=REDIRECT, nif=1) -> int:
    buf = (ctypes.c_uint8 * max(1, len(frame))).from_buffer(frame) if len(frame) else (ctypes.c_uint8 * 1)()
    return load().oracle_packet_processor(ctypes.addressof(buf), len(frame), ingress,
                                          ctypes.byref(_opts(iters, action, nif)))


def c_process_batch(umem: np.ndarray, descs: np.ndarray, ingress=0, iters=1, action=REDIRECT,
                    nif=1, batch=64) -> np.ndarray:
    """Run the C restatement over a host batch IN PLACE; returns int32 verdicts."""
    assert umem.dtype == np.uint8 and umem.flags.c_contiguous
    assert descs.flags.c_contiguous and descs.dtype.itemsize == 16
    n = int(descs.shape[0])
    v = np.empty(n, dtype=np.int32)
    load().oracle_process_batch(umem.ctypes.data, descs.ctypes.data, n, ingress,
                                ctypes.byref(_opts(iters, action, nif)), v.ctypes.data, batch)
    return v


def _pin_mode(pin) -> int:
    """pin: False (unpinned), True / "first" (the first CPUs of the affinity
    mask), "last" (the last ones, away from the HIP runtime's threads)."""
    if pin == "last":
        return 2
    return 1 if pin else 0


def c_time_batch(umem, descs, iters=1, action=REDIRECT, nif=1, threads=1, reps=1, pin=True):
    n = int(descs.shape[0])
    v = np.empty(n, dtype=np.int32)
    t = load().oracle_time_batch(umem.ctypes.data, descs.ctypes.data, n,
                                 ctypes.byref(_opts(iters, action, nif)), v.ctypes.data,
                                 threads, reps, _pin_mode(pin))
    if t < 0:
        raise RuntimeError("oracle_time_batch failed")
    return t, v


def py_packet_processor(f: bytearray, n: int, ingress=0, iters=1, action=REDIRECT, nif=1) -> int:
    """Literal transliteration, one wrapping add per 16-bit word."""
    if n < 14:
        return -1
    if f[12] != 0x08 or f[13] != 0x00:
        return 0
    if n < 34:
        return -1
    if f[23] != 17:
        return 0
    u = 14 + 4 * (f[14] & 0x0F)
    if u + 8 > n:
        return -1

    def le(i):
        return f[i] | (f[i + 1] << 8)

    s = (le(26) + le(28) + le(30) + le(32) + 0x1100 + le(u + 4)) & 0xFFFFFFFF
    f[u + 6] = 0
    f[u + 7] = 0
    for _ in range(iters):
        p = u
        while p + 2 <= n:
            s = (s + le(p)) & 0xFFFFFFFF
            p += 2
        if p < n:
            s = (s + f[p]) & 0xFFFFFFFF
    c = (~(((s & 0xFFFF) + (s >> 16)) & 0xFFFF)) & 0xFFFF
    f[u + 6] = c & 0xFF
    f[u + 7] = c >> 8
    return (ingress + 1) % nif if action == REDIRECT else -1


def np_packet_processor(f: np.ndarray, ingress=0, iters=1, action=REDIRECT, nif=1) -> int:
    """Closed byte-parity form: s = pseudo + max(iters,0) * P (mod 2^32)."""
    n = int(f.shape[0])
    if n < 14:
        return -1
    if f[12] != 0x08 or f[13] != 0x00:
        return 0
    if n < 34:
        return -1
    if f[23] != 17:
        return 0
    u = 14 + 4 * (int(f[14]) & 0x0F)
    if u + 8 > n:
        return -1
    w = f.astype(np.uint64)
    le = lambda i: int(w[i]) | (int(w[i + 1]) << 8)  # noqa: E731
    pseudo = le(26) + le(28) + le(30) + le(32) + 0x1100 + le(u + 4)
    body = w[u:].copy()
    body[6] = 0
    body[7] = 0
    P = int(body[0::2].sum()) + 256 * int(body[1::2].sum())
    s = (pseudo + max(iters, 0) * P) & 0xFFFFFFFF
    c = (~(((s & 0xFFFF) + (s >> 16)) & 0xFFFF)) & 0xFFFF
    f[u + 6] = c & 0xFF
    f[u + 7] = c >> 8
    return (ingress + 1) % nif if action == REDIRECT else -1
