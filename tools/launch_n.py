#!/usr/bin/env python3
"""Launch one checksummer shape N times on a rotated device-resident batch (for
rocprofv3 --pmc passes, where every dispatch of the run should be the same
configuration).

    python tools/launch_n.py --workload 570 --shape 16,2,2,0,3,1,24 --n 20 [--rotate 2]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from xsknf_amd import _lib, frames  # noqa: E402

WL = {"1500": (1500, "aligned"), "64": (64, "aligned"), "imix": ("imix", "aligned"), "570": (570, "aligned"),
      "jumbo": (9000, "unaligned")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="570")
    ap.add_argument("--shape", default="16,2,2,0,3,1,24")
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--rotate", type=int, default=2)
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--bpc", type=int, default=4)
    a = ap.parse_args()
    length, layout = WL[a.workload]
    dev = torch.device("cuda:0")
    K = max(1, a.rotate)
    lens = frames._lens(a.frames, length, np.random.default_rng(frames.SEED))
    umem, descs, _ = frames.device_batch(a.frames * K, np.tile(lens, K), layout=layout, device=dev)
    s = [int(x) for x in a.shape.split(",")] + [0] * 7
    c = _lib.LaunchCfg(s[0], s[1], s[2], a.bpc, s[3], s[4], s[5], s[6])
    lib = _lib.load()
    opts = _lib.CsumOpts(1, 0, 1, 0)
    verd = torch.empty(a.frames, dtype=torch.int32, device=dev)
    for i in range(a.n):
        rc = lib.xsknf_gpu_checksum_batch_cfg(ctypes.c_void_p(umem.data_ptr()), umem.numel(),
                                              ctypes.c_void_p(descs.data_ptr() + 16 * a.frames * (i % K)), a.frames,
                                              0, ctypes.byref(opts), ctypes.c_void_p(verd.data_ptr()), ctypes.byref(c),
                                              None)
        _lib.check(rc, "launch")
    torch.cuda.synchronize()
    print("ok", a.workload, a.shape, a.n)


if __name__ == "__main__":
    main()
