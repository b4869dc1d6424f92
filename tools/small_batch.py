#!/usr/bin/env python3
"""Latency of one synchronous small rx batch with the UMEM in pinned host memory
(the zero-copy host path's situation), per launch shape: which kernel mapping
keeps enough PCIe reads in flight when a batch is a few tiles.

    python tools/small_batch.py [--batches 64,256,1024,4096] [--shapes L,N,U,R,F[,K,W]:...]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from xsknf_amd import _lib, frames  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="64,256,1024,4096")
    ap.add_argument("--len", type=int, default=1500)
    ap.add_argument("--shapes", default="16,3,1,0,5,1,24:64,9,2,0,5:64,4,4,0,5:32,3,2,0,5:16,2,4,0,5:64,2,4,0,5")
    ap.add_argument("--calls", type=int, default=400)
    a = ap.parse_args()
    lib = _lib.load()
    nmax = max(int(x) for x in a.batches.split(","))
    b = frames.aligned_batch(nmax, a.len)
    umem = torch.from_numpy(b.umem).pin_memory()
    descs = torch.from_numpy(b.descs.view(np.uint8).reshape(-1, 16).copy()).pin_memory()
    verd = torch.empty(nmax, dtype=torch.int32).pin_memory()
    opts = _lib.CsumOpts(1, 0, 1, 0)
    # floor: an (almost) empty launch + synchronize on the same device
    x = torch.zeros(1, device="cuda")
    ts = []
    for i in range(a.calls + 20):
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        if i >= 20:
            ts.append(time.perf_counter() - t0)
    print(json.dumps({"null_launch_sync_us": round(statistics.median(ts) * 1e6, 2)}), flush=True)
    for n in (int(x) for x in a.batches.split(",")):
        for t in a.shapes.split(":"):
            s = tuple(int(y) for y in t.split(",")) + (0, 0)
            cfg = _lib.LaunchCfg(s[0], s[1], s[2], 8, s[3], s[4], s[5], s[6])

            def call():
                rc = lib.xsknf_gpu_checksum_batch_cfg(
                    ctypes.c_void_p(umem.data_ptr()), umem.numel(), ctypes.c_void_p(descs.data_ptr()), n, 0,
                    ctypes.byref(opts), ctypes.c_void_p(verd.data_ptr()), ctypes.byref(cfg), None)
                _lib.check(rc, f"shape {s}")
                torch.cuda.synchronize()

            for _ in range(20):
                call()
            ts = []
            for _ in range(a.calls):
                t0 = time.perf_counter()
                call()
                ts.append(time.perf_counter() - t0)
            med = statistics.median(ts)
            print(json.dumps({"batch": n, "shape": s[:7], "us_per_call": round(med * 1e6, 2),
                              "mpps": round(n / med / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
