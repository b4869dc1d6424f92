"""The reference's own per-packet function, compiled here -- TEST INFRASTRUCTURE ONLY.

`oracle/_ref/libcsum_ref.so` is built by `make -C oracle ref` from the verbatim
text of reference examples/checksummer/checksummer_user.c:15-18,24-25,28,30-112
(+ src/xsknf.h:4,11-12,23,25-40), extracted by oracle/ref_extract.sh and driven
by oracle/ref_harness.c (options set as the app's main() sets them, frames fed
in process_batch_1if()'s batch-64 loop, src/xsknf.c:654-672).  It pins the
restatement (csum_oracle.c) and generates tests/golden/.  It exists only where
it was built from a reference checkout: `available()` says whether it is here.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_ref", "libcsum_ref.so")
REFERENCE = os.environ.get("XSKNF_REFERENCE", "/root/reference")

REDIRECT = 0
DROP = 1

_lib = None


def build() -> bool:
    """Build the library if the reference checkout is present; True if it exists afterwards."""
    if os.path.isdir(REFERENCE):
        subprocess.run(["make", "-s", "-C", _HERE, "ref", f"REF={REFERENCE}"], check=True)
    return os.path.exists(LIB_PATH)


def available() -> bool:
    return os.path.exists(LIB_PATH)


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        lib = ctypes.CDLL(LIB_PATH)
        lib.ref_set_options.restype = None
        lib.ref_set_options.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint]
        lib.ref_packet_processor.restype = ctypes.c_int
        lib.ref_packet_processor.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint]
        lib.ref_process_batch.restype = None
        lib.ref_process_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_void_p, ctypes.c_uint32]
        lib.ref_time_batch.restype = ctypes.c_double
        lib.ref_time_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int]
        _lib = lib
    return _lib


def packet_processor(frame: bytearray, ingress=0, iters=1, action=REDIRECT, nif=1) -> int:
    """The reference function on one frame, in place."""
    lib = load()
    lib.ref_set_options(int(iters), int(action), int(nif))
    buf = (ctypes.c_uint8 * max(1, len(frame))).from_buffer(frame) if len(frame) else (ctypes.c_uint8 * 1)()
    return lib.ref_packet_processor(ctypes.addressof(buf), len(frame), ingress)


def process_batch(umem: np.ndarray, descs: np.ndarray, ingress=0, iters=1, action=REDIRECT, nif=1,
                  batch=64) -> np.ndarray:
    """The reference function over a host batch IN PLACE; returns int32 verdicts."""
    assert umem.dtype == np.uint8 and umem.flags.c_contiguous
    assert descs.flags.c_contiguous and descs.dtype.itemsize == 16
    lib = load()
    lib.ref_set_options(int(iters), int(action), int(nif))
    n = int(descs.shape[0])
    v = np.empty(n, dtype=np.int32)
    lib.ref_process_batch(umem.ctypes.data, descs.ctypes.data, n, ingress, v.ctypes.data, batch)
    return v


def _pin_mode(pin) -> int:
    """pin: False (unpinned), True / "first" (the first CPUs of the affinity
    mask), "last" (the last ones, away from the HIP runtime's threads)."""
    if pin == "last":
        return 2
    return 1 if pin else 0


def time_batch(umem, descs, iters=1, action=REDIRECT, nif=1, threads=1, reps=1, pin=True):
    lib = load()
    lib.ref_set_options(int(iters), int(action), int(nif))
    n = int(descs.shape[0])
    v = np.empty(n, dtype=np.int32)
    t = lib.ref_time_batch(umem.ctypes.data, descs.ctypes.data, n, v.ctypes.data, threads, reps,
                           _pin_mode(pin))
    if t < 0:
        raise RuntimeError("ref_time_batch failed")
    return t, v
