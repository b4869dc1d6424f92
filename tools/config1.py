#!/usr/bin/env python3
"""Config 1: the checksummer NF over a veth pair, XDP skb mode, one worker.

BASELINE.json configs[0] / SURVEY.md 8(d) row 1.  Drives tools/build/xsk_veth
(make tools), which runs entirely inside its own network namespace:

  search   zero-loss rate search (reference tests/test-drop-cpu.py:99-122:
           -c DROP, loss <= 0.1 %), 64 B frames over 256 flows
  check    every frame of a mixed set (64..1514 B, edge cases) sent once with
           REDIRECT; the frames that come back must equal the oracle's output
           byte for byte, in order

The NF here is the reference per-frame path: the reference's own
xsknf_packet_processor() compiled from its verbatim lines (oracle/_ref, where
built; else the CPU restatement pinned to it; the harness's "nf" field says
which): this is the CPU reference configuration, run on the runtime of
include/xsknf.h.  Needs root (netns, XDP, AF_XDP); the GPU box
runs commands unprivileged, so this runs in the build container only.
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from xsknf_amd import frames as F  # noqa: E402

HARNESS = os.path.join(ROOT, "tools", "build", "xsk_veth")
SRC_MAC = bytes.fromhex("0a0000000001")


def write_frames(path: str, frames: list[bytes]) -> None:
    with open(path, "wb") as f:
        f.write(b"XSKF" + struct.pack("<I", len(frames)))
        for fr in frames:
            f.write(struct.pack("<I", len(fr)) + fr)


def read_frames(path: str) -> list[bytes]:
    with open(path, "rb") as f:
        data = f.read()
    assert data[:4] == b"XSKF"
    (n,) = struct.unpack_from("<I", data, 4)
    out, off = [], 8
    for _ in range(n):
        (ln,) = struct.unpack_from("<I", data, off)
        out.append(data[off + 4:off + 4 + ln])
        off += 4 + ln
    return out


def frames_64(n: int = 4096, seed: int = F.SEED) -> list[bytes]:
    """64 B Eth/IPv4/UDP, 256 flows, random payload."""
    rng = np.random.default_rng(seed)
    lens = np.full(n, 64, dtype=np.int64)
    hdr = F.headers(lens, rng.integers(0, 256, size=n))
    pay = rng.integers(0, 256, size=(n, 64 - F.HDR_LEN), dtype=np.uint8)
    return [bytes(hdr[i]) + bytes(pay[i]) for i in range(n)]


def frames_check(n: int = 3000, seed: int = F.SEED + 11) -> list[bytes]:
    """Mixed lengths 14..1514 and the edge cases the parity tests use."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(14, 1515, size=n)
    lens[: n // 4] = rng.choice([60, 64, 570, 1500, 1514], size=n // 4)
    hdr = F.headers(lens, rng.integers(0, 256, size=n))
    out = []
    for i in range(n):
        ln = int(lens[i])
        b = bytearray(bytes(hdr[i]) + rng.integers(0, 256, size=max(ln - F.HDR_LEN, 0),
                                                  dtype=np.uint8).tobytes())[:ln]
        kind = i % 17
        if kind == 3 and ln > 14:
            b[12:14] = b"\x86\xdd"              # not IPv4
        elif kind == 5 and ln > 23:
            b[23] = 6                           # TCP
        elif kind == 7 and ln > 14:
            b[14] = 0x46 + int(rng.integers(0, 9))   # ihl 6..14
        elif kind == 11 and ln > 40:
            b[40:42] = rng.integers(0, 256, size=2, dtype=np.uint8).tobytes()  # stale check
        out.append(bytes(b))
    return out


def oracle_outputs(frames: list[bytes], iterations: int) -> list[bytes]:
    """The frames the NF transmits back, as the oracle rewrites them: verdict -1
    (truncated headers, checksummer_user.c:43-55) drops a frame even in REDIRECT."""
    from oracle import csum_oracle as O
    out = []
    for fr in frames:
        buf = bytearray(fr)
        if O.c_packet_processor(buf, 0, iters=iterations, action=O.REDIRECT, nif=1) != -1:
            out.append(bytes(buf))
    return out


def run(args: list[str], timeout: float) -> dict:
    p = subprocess.run([HARNESS] + args, capture_output=True, text=True, timeout=timeout)
    line = p.stdout.strip().splitlines()[-1] if p.stdout.strip() else "{}"
    res = json.loads(line)
    res["exit"] = p.returncode
    if p.returncode not in (0,):
        res["stderr"] = p.stderr[-2000:]
    return res


def check(iterations: int = 1, n: int = 3000, extra: tuple = ()) -> dict:
    """extra: more harness flags (--two-phase, --poll, --batch B)."""
    sent = frames_check(n)
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        write_frames(fin, sent)
        res = run(["--frames", fin, "--check", fout, "--iterations", str(iterations), *extra], 120)
        if res.get("exit") != 0:
            return res
        back = [f for f in read_frames(fout) if f[6:12] == SRC_MAC]
    want = oracle_outputs(sent, iterations)
    res["ours_returned"] = len(back)
    res["expected"] = len(want)
    # in order: one worker, one queue, FIFO end to end
    res["mismatches"] = sum(1 for a, b in zip(back, want) if a != b) + abs(len(back) - len(want))
    return res


def search(iterations: int, max_mpps: float, step: float, trial_s: float, generators: int) -> dict:
    with tempfile.TemporaryDirectory() as d:
        fin = os.path.join(d, "in.bin")
        write_frames(fin, frames_64())
        res = run(["--frames", fin, "--search", "--iterations", str(iterations),
                   "--max-mpps", str(max_mpps), "--step-mpps", str(step), "--trial-s", str(trial_s),
                   "--generators", str(generators)], 600)
    res["frame_len"] = 64
    res["cpus_visible"] = os.cpu_count()
    return res


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("mode", choices=["check", "search"])
    ap.add_argument("--iterations", type=int, default=1)
    ap.add_argument("--max-mpps", type=float, default=4.0)
    ap.add_argument("--step-mpps", type=float, default=0.05)
    ap.add_argument("--trial-s", type=float, default=2.0)
    ap.add_argument("--generators", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.mode == "check":
        res = check(a.iterations)
    else:
        res = search(a.iterations, a.max_mpps, a.step_mpps, a.trial_s, a.generators)
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0 if res.get("exit") == 0 and res.get("mismatches", 0) == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
