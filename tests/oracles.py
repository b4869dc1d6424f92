"""The CPU answer the full-size GPU parity tests compare with (test infrastructure).

`oracle/_ref/libcsum_ref.so` is the reference's own xsknf_packet_processor()
(checksummer_user.c:30-112 compiled from its verbatim lines; built by build()
wherever the reference checkout exists, it travels to the GPU box as a built
library).  The full-size runs are held against it, in process_batch_1if()'s
batch-64 loop (src/xsknf.c:654-672) split over threads.  It is required: a GPU
run without it fails (there is no quiet fall back to the restatement, which
tests/test_ref_pin.py holds equal to it on CPU).
"""
import numpy as np

from oracle import ref as R

KIND = "reference"


def require():
    """Fail loudly when the reference library is not here."""
    if not R.available():
        raise RuntimeError(f"{R.LIB_PATH} is missing: build it with `make oracle` in a container that holds the "
                           "reference checkout (build() does); the GPU parity tests compare with it, not with "
                           "the restatement")


def time_batch(umem, descs, threads=16, **kw):
    """In place over the host batch; returns (seconds, verdicts).

    The reference never sees a descriptor outside its UMEM: the kernel's rx
    validation drops it before the ring (and xsknf_gpu's boundary gives it -1,
    untouched, include/xsknf_gpu.h).  Such descriptors get -1 here and only the
    others go to the reference's function, whose pointer arithmetic
    (src/xsknf.c:659) would otherwise leave the buffer."""
    require()
    a = descs["addr"].astype(np.uint64)
    off = (a & np.uint64((1 << 48) - 1)) + (a >> np.uint64(48))
    size = np.uint64(umem.size)
    ok = (off <= size) & (descs["len"].astype(np.uint64) <= size - np.minimum(off, size))
    if ok.all():
        return R.time_batch(umem, descs, threads=threads, reps=1, pin=False, **kw)
    v = np.full(descs.shape[0], -1, dtype=np.int32)
    if ok.any():
        t, v[ok] = R.time_batch(umem, np.ascontiguousarray(descs[ok]), threads=threads, reps=1, pin=False, **kw)
    else:
        t = 0.0
    return t, v
