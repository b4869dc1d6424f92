"""Child process of test_gpu_parity.py::test_grid_sizing_on_a_smaller_device.

Runs one batch through the product path with XSKNF_GPU_CU_LIMIT set by the
parent (the library sizes its grids as on a device with that many CUs; the
variable is read once per process, so it needs a process of its own) and
prints one JSON line comparing every verdict and UMEM byte with the oracle.

    XSKNF_GPU_CU_LIMIT=4 python tests/cu_limit_child.py --frames 30720 --length 9000
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tests import oracles  # noqa: E402
from xsknf_amd import Checksummer, ChecksummerOptions, frames  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, required=True)
    ap.add_argument("--length", default="9000")
    ap.add_argument("--layout", default="unaligned")
    ap.add_argument("--mean", action="store_true", help="pass the batch's mean length too (static IMIX shape)")
    a = ap.parse_args()
    length = int(a.length) if a.length.isdigit() else a.length
    dev = torch.device("cuda:0")
    n = a.frames
    umem, descs, lens = frames.device_batch(n, length, layout=a.layout, device=dev, seed=n)
    host = umem.cpu().numpy()
    hd = descs.cpu().numpy().view(frames.DESC_DTYPE).reshape(-1).copy()
    frames.inject_edge_cases(frames.HostBatch(host, hd, a.layout), 0.01, seed=n + 1)
    umem.copy_(torch.from_numpy(host))
    descs.copy_(torch.from_numpy(hd.view(np.int64).reshape(n, 2)))
    # the batch's longest frame as the hint: the shape the product picks for it
    # (jumbo: the 8-wave pooled blocks with quarters)
    cs = Checksummer(ChecksummerOptions(), num_interfaces=1, frame_len_hint=int(lens.max()),
                     frame_len_mean=int(lens.mean()) if a.mean else 0)
    v = cs.process_batch(umem, descs)
    torch.cuda.synchronize()
    gv, gu = v.cpu().numpy(), umem.cpu().numpy()
    _, ov = oracles.time_batch(host, hd)
    from xsknf_amd import _lib
    print(json.dumps({"frames": n, "cus_limit": os.environ.get("XSKNF_GPU_CU_LIMIT"),
                      "pool_guard_trips": _lib.pool_guard_trips(),
                      "window_chunks": int(cs.launch_cfg().window_chunks),
                      "bad_verdicts": int((gv != ov).sum()), "bad_bytes": int((gu != host).sum())}))


if __name__ == "__main__":
    main()
