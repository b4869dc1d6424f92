#!/usr/bin/env python3
"""Per-wave timeline of the split kernel (A/B instrument; `make tl` builds
build/tl/libxsknf_gpu.so with -DXSKNF_TIMELINE).

Each wave records the 100 MHz constant clock at its start, after its last
tile (stream done, its loads drained), and after its own patches, its tile
count, and the clock summed over its tiles in phase A's window loads, the rest
of phase A, and phase B.  The summary splits the launch into the stream and the patch
phase: when the first / median / last wave finished streaming, how long the
patches took per wave, and how much of the patch time overlapped other
waves' streams.

    XSKNF_GPU_LIB=build/tl/libxsknf_gpu.so python tools/timeline.py --workload 1500
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from xsknf_amd import _lib, frames  # noqa: E402

WL = {"1500": (1500, "aligned"), "imix": ("imix", "aligned"), "570": (570, "aligned"), "64": (64, "aligned"),
      "1024": (1024, "aligned"), "jumbo": (9000, "unaligned")}


def pct(x, q):
    return round(float(np.percentile(x, q)), 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="1500")
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--rotate", type=int, default=1)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variant", default="", help="lanes,chunks,u,ring,fused,kernel,window (default: product)")
    ap.add_argument("--bpc", type=int, default=0, help="blocks per CU asked for (0: the shape's own)")
    ap.add_argument("--same-checks", action="store_true",
                    help="every launch with -i 1 (after the first visit of a batch its checks are right and "
                         "nothing is written); default: alternate -i 1 / 2 per visit, so every check changes")
    a = ap.parse_args()
    length, layout = WL.get(a.workload, (int(a.workload) if a.workload.isdigit() else a.workload, "aligned"))
    dev = torch.device("cuda:0")
    K = max(1, a.rotate)
    base = frames._lens(a.frames, length, np.random.default_rng(frames.SEED))
    umem, descs_all, lens_all = frames.device_batch(a.frames * K, np.tile(base, K), layout=layout, device=dev)
    n = a.frames
    lib = _lib.load()
    if not hasattr(lib, "xsknf_gpu_ab_set_timeline"):
        raise SystemExit("not a timeline build: set XSKNF_GPU_LIB=build/tl/libxsknf_gpu.so")
    lib.xsknf_gpu_ab_set_timeline.argtypes = [ctypes.c_void_p]
    opts_by_iters = {1: _lib.CsumOpts(1, 0, 1, 0), 2: _lib.CsumOpts(2, 0, 1, 0)}
    cfg = _lib.LaunchCfg()
    lens = lens_all[:n]
    lib.xsknf_gpu_launch_cfg_for_lens(int(lens.max()), int(lens.mean()), ctypes.byref(cfg))
    if a.variant:
        v = [int(x) for x in a.variant.split(",")]
        cfg = _lib.LaunchCfg(v[0], v[1], v[2], 4, v[3], v[4], v[5], v[6])
    if a.bpc:
        cfg.blocks_per_cu = a.bpc
    verd = torch.empty(n, dtype=torch.int32, device=dev)
    tl = torch.zeros(8 * 65536, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()

    visits = [0] * K

    def run(j):
        # (the bench's worst case: each visit of a batch alternates -i 1 / 2, so every check changes)
        it = 1 if a.same_checks else 1 + visits[j] % 2
        visits[j] += 1
        rc = lib.xsknf_gpu_checksum_batch_cfg(ctypes.c_void_p(umem.data_ptr()), umem.numel(),
                                              ctypes.c_void_p(descs_all.data_ptr() + 16 * n * j), n, 0,
                                              ctypes.byref(opts_by_iters[it]), ctypes.c_void_p(verd.data_ptr()),
                                              ctypes.byref(cfg), ctypes.c_void_p(stream.cuda_stream))
        _lib.check(rc, "launch")

    _lib.check(lib.xsknf_gpu_ab_set_timeline(None), "timeline off")
    for j in range(10):
        run(j % K)
    torch.cuda.synchronize()
    rows = []
    for r in range(a.reps):
        tl.zero_()
        torch.cuda.synchronize()
        _lib.check(lib.xsknf_gpu_ab_set_timeline(ctypes.c_void_p(tl.data_ptr())), "timeline on")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        run(r % K)
        e1.record(stream)
        torch.cuda.synchronize()
        _lib.check(lib.xsknf_gpu_ab_set_timeline(None), "timeline off")
        t = tl.view(-1, 8).cpu().numpy()
        gw = np.nonzero(t[:, 0] != 0)[0]
        t = t[t[:, 0] != 0]
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        # waves per block (window + 32: one block per CU, 12 waves; 8 for jumbo's W = 4)
        wpb = 4
        if cfg.window_chunks & 32:   # one block per CU: split 12 waves (8 for jumbo's W = 4), lane 16
            wpb = (12 if (cfg.window_chunks & 15) == 8 else 8) if cfg.kernel == 1 else 16
        bslot, xcd, wvi = (gw // wpb) // cus, (gw // wpb) % 8, gw % 4
        blk = gw // wpb
        sd_us = (t[:, 1] - t[:, 0].min()) / 100.0
        nb = int(blk.max()) + 1
        bmax = np.full(nb, -1e9); bmin = np.full(nb, 1e9); bsum = np.zeros(nb); bcnt = np.zeros(nb)
        np.maximum.at(bmax, blk, sd_us); np.minimum.at(bmin, blk, sd_us)
        np.add.at(bsum, blk, sd_us); np.add.at(bcnt, blk, 1)
        ok = bcnt > 0
        bspread = (bmax - bmin)[ok]
        bmean = (bsum / np.maximum(bcnt, 1))[ok]
        cu = blk % cus
        csum = np.zeros(cus); ccnt = np.zeros(cus)
        np.add.at(csum, cu, sd_us); np.add.at(ccnt, cu, 1)
        cmean = (csum / np.maximum(ccnt, 1))[ccnt > 0]
        t0 = t[:, 0].min()
        start, sdone, pdone = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0, (t[:, 2] - t0) / 100.0   # us
        end = pdone.max()
        patch = pdone - sdone
        # patch time of waves while some other wave was still streaming
        last_stream = sdone.max()
        overl = np.clip(np.minimum(pdone, last_stream) - sdone, 0, None)
        tiles = t[:, 3]
        rows.append({
            "event_us": round(e0.elapsed_time(e1) * 1e3, 2), "waves": int(len(t)), "kernel_us": round(float(end), 2),
            "start_p99": pct(start, 99), "stream_done": [pct(sdone, 0), pct(sdone, 10), pct(sdone, 50),
                                                          pct(sdone, 90), pct(sdone, 100)],
            "patch_us": [pct(patch, 0), pct(patch, 50), pct(patch, 90), pct(patch, 100)],
            "patch_overlapping_stream_us_mean": round(float(overl.mean()), 2),
            "after_last_stream_us": round(float(end - last_stream), 2),
            "tiles": {int(k): int(v) for k, v in zip(*np.unique(tiles, return_counts=True))},
            "per_wave_us_phaseA_window_parse_B": [round(float(t[:, k].mean()) / 100.0, 2) for k in (4, 5, 6)],
            "stream_done_by_tiles": {int(k): pct(sdone[tiles == k], 50) for k in np.unique(tiles)},
            # wave index = block * 4 + wave: block slot on its CU (dispatch order) and XCD (block % 8)
            "stream_done_p50_max_by_block_slot": {int(b): [pct(sdone[bslot == b], 50), pct(sdone[bslot == b], 100)]
                                                  for b in np.unique(bslot)},
            "stream_done_p50_max_by_xcd": {int(x): [pct(sdone[xcd == x], 50), pct(sdone[xcd == x], 100)]
                                           for x in np.unique(xcd)},
            "stream_done_p50_by_simd": {int(w): pct(sdone[wvi == w], 50) for w in range(4)},
            # pooling potential: a block's 4 waves sharing their tiles would end near their mean
            "block_internal_spread_p50_p90": [pct(bspread, 50), pct(bspread, 90)],
            "stream_end_if_pooled_per_block": pct(bmean, 100),
            "stream_end_if_pooled_per_cu": pct(cmean, 100),
        })
    rows.sort(key=lambda x: x["kernel_us"])
    med = rows[len(rows) // 2]
    print(json.dumps({"workload": a.workload, "frames": n, "blocks_per_cu": cfg.blocks_per_cu, "cfg": [cfg.lanes_per_frame, cfg.chunks_per_lane, cfg.frames_per_group,
                                                      cfg.lds_ring, cfg.fused_stores, cfg.kernel, cfg.window_chunks],
                      "median": med, "kernel_us_all": [r["kernel_us"] for r in rows]}))


if __name__ == "__main__":
    main()
