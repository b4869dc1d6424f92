#!/usr/bin/env python3
"""A/B the launch shapes of the checksummer kernel in ONE process (interleaved
rounds, median of per-round HIP-event timings), on device-resident batches.

    python tools/tune.py --workload 1500 --variants 32,3,2:32,3,1:64,2,1:32,3,1,3 [--bpc 8,4]

A variant is lanes_per_frame,chunks_per_lane,frames_per_group[,lds_ring[,fused_stores[,kernel,window]]]
(lds_ring must be 0: the LDS-DMA kernels were removed in round 5 and any other value is
-EINVAL; fused_stores 1 = single-pass stores;
kernel 1 = the split kernel with a `window`-chunk header window per lane).

Every variant's output (verdicts + whole UMEM) is compared with the default
shape's output, so a tuning run is also a cross-variant parity check.

--checks zero (default): the frames' checks are 0, so every check changes; the
timed launches alternate csum_iterations 1 and 2 per visit of a batch, so each
launch rewrites every check (a launch over frames the previous one left would
write nothing: the kernels skip checks a frame already holds).  --checks nic:
the checks a NIC's UDP offload writes (frames.offload_checks_device), all but
the carry-loss frames already right; the launches all use -i 1 (after the first
pass the carry-loss frames hold their value too: the same for every variant).
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from xsknf_amd import _lib, frames  # noqa: E402

WL = {
    "1500": (1500, "aligned"), "64": (64, "aligned"), "imix": ("imix", "aligned"),
    "jumbo": (9000, "unaligned"), "570": (570, "aligned"), "64u": (64, "unaligned"), "60u": (60, "unaligned"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="1500")
    ap.add_argument("--variants", default="")
    ap.add_argument("--bpc", default="0",
                    help="blocks per CU to try (comma list); 0 = the product's own choice for the default shape "
                         "(default_cfg), 8 (as many as fit) for the others")
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--checks", default="zero", choices=["zero", "nic"])
    ap.add_argument("--rotate", type=int, default=1,
                    help="batches the timed launches cycle through (bench.py's rotation: keeps a small-frame "
                         "batch out of the Infinity Cache between launches)")
    a = ap.parse_args()
    length, layout = WL[a.workload] if a.workload in WL else (int(a.workload), "aligned")
    dev = torch.device("cuda:0")
    K = max(1, a.rotate)
    base_lens = frames._lens(a.frames, length, __import__("numpy").random.default_rng(frames.SEED))
    umem0, descs_all, lens_all = frames.device_batch(a.frames * K, __import__("numpy").tile(base_lens, K),
                                                     layout=layout, device=dev)
    if a.checks == "nic":
        frames.offload_checks_device(umem0, descs_all)
    descs = descs_all[:a.frames]
    lens = lens_all[:a.frames]
    lib = _lib.load()
    opts = _lib.CsumOpts(1, 0, 1, 0)
    opts2 = _lib.CsumOpts(2, 0, 1, 0)
    n = a.frames
    hint = int(lens.max())
    dflt = _lib.LaunchCfg()
    lib.xsknf_gpu_launch_cfg_for_lens(hint, int(lens.mean()), ctypes.byref(dflt))   # the product's choice
    shapes = [(dflt.lanes_per_frame, dflt.chunks_per_lane, dflt.frames_per_group, dflt.lds_ring,
               dflt.fused_stores, dflt.kernel, dflt.window_chunks)]
    for t in [x for x in a.variants.split(":") if x]:
        s = tuple(int(y) for y in t.split(","))
        s = s + (0,) * (7 - len(s))
        if s not in shapes:
            shapes.append(s)
    bpcs = [int(x) for x in a.bpc.split(",")]
    cfgs = [(s, b if b else (dflt.blocks_per_cu if i == 0 else 8)) for i, s in enumerate(shapes) for b in bpcs]
    stream = torch.cuda.current_stream()
    umem = umem0.clone()
    verd = torch.empty(n, dtype=torch.int32, device=dev)

    rot = [0]

    def run(cfg, um, vv, j=0, alt=False):
        c = _lib.LaunchCfg(cfg[0][0], cfg[0][1], cfg[0][2], cfg[1], cfg[0][3], cfg[0][4], cfg[0][5], cfg[0][6])
        rc = lib.xsknf_gpu_checksum_batch_cfg(ctypes.c_void_p(um.data_ptr()), um.numel(),
                                              ctypes.c_void_p(descs_all.data_ptr() + 16 * n * j), n, 0,
                                              ctypes.byref(opts2 if alt else opts), ctypes.c_void_p(vv.data_ptr()),
                                              ctypes.byref(c), ctypes.c_void_p(stream.cuda_stream))
        _lib.check(rc, f"cfg {cfg}")

    # reference output = default shape on a fresh copy
    ref_u = umem0.clone()
    ref_v = torch.empty_like(verd)
    run(cfgs[0], ref_u, ref_v)
    torch.cuda.synchronize()
    times = {c: [] for c in cfgs}
    ok = {}
    for c in cfgs:
        u = umem0.clone()
        v = torch.empty_like(verd)
        run(c, u, v)
        torch.cuda.synchronize()
        ok[c] = bool(torch.equal(u, ref_u) and torch.equal(v, ref_v))
        del u, v
    for r in range(a.rounds):
        for c in cfgs:
            def visit():
                rot[0] += 1
                run(c, umem, verd, rot[0] % K, a.checks == "zero" and bool((rot[0] // K) & 1))
            for _ in range(2):
                visit()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.reps):
                visit()
            e1.record(stream)
            torch.cuda.synchronize()
            times[c].append(e0.elapsed_time(e1) / a.reps * 1e3)
    blen = int(lens.sum())
    alg = blen + n * 22
    for c in cfgs:
        med = statistics.median(times[c])
        print(json.dumps({"workload": a.workload, "checks": a.checks, "shape": c[0], "bpc": c[1], "us": round(med, 2),
                          "min_us": round(min(times[c]), 2),
                          "gbs_checksummed": round(blen / med / 1e3, 1),
                          "roofline_frac": round(alg / med / 1e3 / 8000, 4),
                          "mpps": round(n / med, 1), "matches_default": ok[c]}))


if __name__ == "__main__":
    main()
