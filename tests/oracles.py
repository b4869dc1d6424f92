"""The CPU answer the full-size GPU parity tests compare with (test infrastructure).

Where `oracle/_ref/libcsum_ref.so` was built (the reference's own
xsknf_packet_processor(), checksummer_user.c:30-112 compiled from its verbatim
lines; it travels to the GPU box as a built library), the full-size runs are
held against the reference itself, in process_batch_1if()'s batch-64 loop
(src/xsknf.c:654-672) split over threads; elsewhere against the restatement
oracle/csum_oracle.c, which tests/test_ref_pin.py holds equal to it.
"""
from oracle import csum_oracle as O
from oracle import ref as R

KIND = "reference" if R.available() else "restatement"


def time_batch(umem, descs, threads=16, **kw):
    """In place over the host batch; returns (seconds, verdicts)."""
    if R.available():
        return R.time_batch(umem, descs, threads=threads, reps=1, pin=False, **kw)
    return O.c_time_batch(umem, descs, threads=threads, reps=1, **kw)
