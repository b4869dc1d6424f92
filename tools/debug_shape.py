"""Run one launch shape of test_every_launch_shape_is_bit_exact and describe the
frames whose bytes differ from the oracle (GPU box; test infrastructure).

    python tools/debug_shape.py 64,2,1,0,0,1,4 [aligned|unaligned]
Set XSKNF_GPU_LIB to A/B another build of the library.
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import csum_oracle as O  # noqa: E402
from xsknf_amd import _lib, frames  # noqa: E402


def main():
    shape = tuple(int(x) for x in sys.argv[1].split(","))
    layout = sys.argv[2] if len(sys.argv) > 2 else "aligned"
    dev = torch.device("cuda:0")
    lib = _lib.load()
    rng = np.random.default_rng(sum(shape))
    lens = rng.integers(0, 3000, size=2500).astype(np.uint32)
    if layout == "aligned":
        b = frames.aligned_batch(2500, np.minimum(lens, 1792), chunk=2048, seed=sum(shape))
    else:
        b = frames.unaligned_batch(2500, lens, seed=sum(shape))
    frames.inject_edge_cases(b, 0.1)
    r = b.copy()
    ov = O.c_process_batch(r.umem, r.descs, ingress=1, iters=2, action=O.REDIRECT, nif=3)
    ou = r.umem
    kernel, window = (shape[5], shape[6]) if len(shape) > 5 else (0, 0)
    addrs = b.descs["addr"].astype(np.uint64)
    offs = ((addrs & np.uint64((1 << 48) - 1)) + (addrs >> np.uint64(48))).astype(np.int64)
    lens = b.descs["len"].astype(np.int64)
    for rep in range(3):
        umem = torch.from_numpy(b.umem).to(dev)
        descs = torch.from_numpy(b.descs.view(np.uint8).reshape(-1, 16).copy()).to(dev)
        v = torch.empty(b.n, dtype=torch.int32, device=dev)
        cfg = _lib.LaunchCfg(shape[0], shape[1], shape[2], 4, shape[3], shape[4], kernel, window)
        rc = lib.xsknf_gpu_checksum_batch_cfg(
            ctypes.c_void_p(umem.data_ptr()), umem.numel(), ctypes.c_void_p(descs.data_ptr()), b.n, 1,
            ctypes.byref(_lib.CsumOpts(2, O.REDIRECT, 3, 0)), ctypes.c_void_p(v.data_ptr()),
            ctypes.byref(cfg), None)
        torch.cuda.synchronize()
        gv, gu = v.cpu().numpy(), umem.cpu().numpy()
        vb = np.nonzero(gv != ov)[0]
        ub = np.nonzero(gu != ou)[0]
        print(f"rep {rep}: rc {rc}, {vb.size} verdicts and {ub.size} UMEM bytes differ")
        for pos in ub[:16]:
            owners = np.nonzero((offs <= pos) & (pos < offs + lens))[0]
            for i in owners[:2]:
                o, ln = int(offs[i]), int(lens[i])
                ihl = int(ou[o + 14] & 15) if ln > 14 else -1
                print(f"  byte {pos}: frame {i} (tile {i // 64}, lane {i % 64}) off {o} (mod16 {o % 16}) len {ln} "
                      f"ihl {ihl} at +{pos - o}: gpu {gu[pos]:02x} ref {ou[pos]:02x} orig {b.umem[pos]:02x} "
                      f"verdict {gv[i]}")
            if owners.size == 0:
                print(f"  byte {pos}: outside every frame: gpu {gu[pos]:02x} ref {ou[pos]:02x}")


if __name__ == "__main__":
    main()
