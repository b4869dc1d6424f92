#!/usr/bin/env python3
"""End-to-end host-path rate (UMEM in host memory, pinned): the rate an AF_XDP
worker would see calling the GPU batch hook, PCIe included.

For each path (zerocopy / staged) and rx batch size, time back-to-back
synchronous xsknf_gpu_ctx_process_batch() calls over a host UMEM of 1500 B (or
--len) frames, and check one batch against the CPU oracle.

    python tools/e2e_bench.py [--frames 1048576] [--len 1500] [--batches 64,4096,65536,1048576]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from xsknf_amd import Checksummer, HostPath, frames  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--len", type=int, default=1500)
    ap.add_argument("--batches", default="64,1024,16384,262144,1048576")
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--paths", default="zerocopy,staged")
    a = ap.parse_args()
    b = frames.aligned_batch(a.frames, a.len)
    ref = None
    if a.check:
        from oracle import csum_oracle as O
        ref = b.copy()
        O.c_process_batch(ref.umem, ref.descs)
    cs = Checksummer(frame_len_hint=a.len)
    results = []
    for path in a.paths.split(","):
        umem = b.umem.copy()
        with HostPath(cs, umem, path=path, max_batch=max(int(x) for x in a.batches.split(","))) as hp:
            for bs in [int(x) for x in a.batches.split(",")]:
                bs = min(bs, a.frames)
                nb = a.frames // bs
                v = np.empty(bs, dtype=np.int32)
                hp.process_batch(b.descs[:bs], verdicts=v)   # warm-up
                done, t0 = 0, time.perf_counter()
                while time.perf_counter() - t0 < a.seconds or done == 0:
                    i = done % nb
                    hp.process_batch(b.descs[i * bs:(i + 1) * bs], verdicts=v)
                    done += 1
                dt = time.perf_counter() - t0
                fr = done * bs
                results.append({"path": path, "batch": bs, "calls": done,
                                "us_per_call": round(dt / done * 1e6, 2),
                                "mpps": round(fr / dt / 1e6, 3),
                                "gbs_checksummed": round(fr * a.len / dt / 1e9, 3)})
                print(json.dumps(results[-1]), flush=True)
            st = hp.stats()
        if ref is not None:
            # every frame was processed at least once; processing is idempotent
            ok = bool(np.array_equal(umem, ref.umem))
            print(json.dumps({"path": path, "umem_matches_oracle": ok, "stats": st}), flush=True)


if __name__ == "__main__":
    main()
