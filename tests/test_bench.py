"""bench.py's measurement bookkeeping, on CPU (no GPU calls): the rotation that
keeps a pass out of the Infinity Cache, the iteration schedule that makes every
step rewrite every check of a base workload, the stream / batch pairing of
--streams, and the NIC workloads' shapes."""
import os

import numpy as np
import pytest

pytest.importorskip("torch")
import bench  # noqa: E402


class Args:
    rotate = 0
    rotate_bytes = 1 << 30
    streams = 1


def test_rotation_keeps_a_pass_past_the_infinity_cache():
    a = Args()
    assert bench.rotation(np.full(1 << 20, 1500, np.uint32), a) == 1
    k = bench.rotation(np.full(1 << 20, 64, np.uint32), a)
    touched = (1 << 20) * (64 + 20)
    assert k * touched >= a.rotate_bytes and (k - 1) * touched < a.rotate_bytes


@pytest.mark.parametrize("K", [1, 2, 3, 13])
def test_every_visit_of_a_batch_changes_its_checks(K):
    """Consecutive visits of the same batch use different iteration counts."""
    last = {}
    for it in range(10 * K):
        j, i = it % K, bench.iterations_of_step(it, K)
        if j in last:
            assert i != last[j]
        last[j] = i


@pytest.mark.parametrize("streams,lens,want", [(1, 64, (13, 1)), (2, 64, (14, 2)), (2, 1500, (2, 2)),
                                               (3, 1500, (3, 3))])
def test_batches_and_streams(streams, lens, want):
    a = Args()
    a.streams = streams
    K, S = bench.batches_and_streams("1500", np.full(1 << 20, lens, np.uint32), a)
    assert (K, S) == want
    assert K % S == 0                       # every visit of batch j goes to stream j % S
    for it in range(5 * K):
        assert (it % S) == (it % K) % S


def test_nic_workloads_time_one_stream_and_mirror_their_base():
    a = Args()
    a.streams = 2
    assert bench.batches_and_streams("1500-nic", np.full(16, 1500, np.uint32), a)[1] == 1
    for nic, base in bench.NIC.items():
        assert bench.WORKLOADS[nic][:3] == bench.WORKLOADS[base][:3]


@pytest.mark.parametrize("world", [2, 3, 8])
def test_check_fingerprint_of_shards_adds_up_to_the_whole(world):
    """--root-scatter holds the shards' all-reduced fingerprint against rank 0's
    single-GPU pass over the whole batch: with each shard's rebased descriptors
    and its span start as base, the shards' fingerprints sum to the whole's, and
    moving one check byte or swapping two frames' checks changes it."""
    import torch
    from xsknf_amd import frames
    from xsknf_amd.shard import rebase_descs, shard_by_bytes, shard_spans
    b = frames.unaligned_batch(3000, "imix", seed=51)
    umem = torch.from_numpy(b.umem.copy())
    whole_d = torch.from_numpy(b.descs.view(np.int64).reshape(-1, 2).copy())
    whole = bench.check_fingerprint(umem, whole_d, 0)
    ranges = shard_by_bytes(b.descs["len"], world)
    spans = shard_spans(b.descs, ranges, umem.numel())
    tot = [0, 0]
    for (lo, hi), (s0, s1) in zip(ranges, spans):
        d = torch.from_numpy(rebase_descs(b.descs[lo:hi], s0, umem.numel()).view(np.int64).reshape(-1, 2).copy())
        f = bench.check_fingerprint(umem[s0:s1], d, s0)
        tot = [tot[0] + f[0], tot[1] + f[1]]
    assert tot == whole
    offs = (b.descs["addr"] & ((1 << 48) - 1)) + (b.descs["addr"] >> 48)
    a, c = int(offs[10]) + 40, int(offs[20]) + 40
    if umem[a] == umem[c] and umem[a + 1] == umem[c + 1]:
        umem[a] ^= 1
    else:
        umem[a], umem[c] = umem[c].clone(), umem[a].clone()
        umem[a + 1], umem[c + 1] = umem[c + 1].clone(), umem[a + 1].clone()
    assert bench.check_fingerprint(umem, whole_d, 0) != whole


def test_cpu_baseline_windows_and_pinning():
    """cpu_baseline (kind "reference" where oracle/_ref is built, else the
    restatement) times three windows, reports their median with min / max, and
    pins one thread to the LAST CPU of the affinity mask, several threads to its
    last CPUs."""
    import os
    from xsknf_amd import frames
    b = frames.aligned_batch(2048, 1500, seed=61)
    res = {"sample": (b.umem.copy(), b.descs, b.n)}
    mask = sorted(os.sched_getaffinity(0))
    for threads in (1, min(2, len(mask))):
        c = bench.cpu_baseline(res, 0.3, threads, check=False)
        sp = c["spread"]
        assert sp["windows"] == 3 and sp["min"] <= c["value"] <= sp["max"]
        assert c["cores"] == threads and c["unit"] == "GB/s checksummed"
        assert c["pinned_to"] == bench._cpu_list(mask[-threads:])
        assert c["kind"] in ("reference", "port")
        assert c["mpps"] > 0


def test_cpu_list_ranges():
    assert bench._cpu_list([0, 1, 2, 3, 7, 9, 10]) == "0-3,7,9-10"
    assert bench._cpu_list([5]) == "5"


def test_lane_batch_workload_is_thirteen_batches():
    class A:
        frames = 1024
        config4_frames = 8192
    lens, span = bench.workload_lengths("64-13M", A, 1, 0)
    assert lens.shape[0] == 13 * 1024 and span is None and int(lens.max()) == 64


_LEG_CHILD = r"""
import os, sys, time
sys.path.insert(0, {root!r})
import bench
line = {{"metric": "m", "value": 1}}
def leg():
    os.write(1, b"RCCL version : banner\n")   # a library writing to fd 1, as RCCL's init does
    print("from python")
    if {sleep}:
        time.sleep({sleep})
    return {{"ok": True}}
line["c_host_multi"] = bench.bounded_leg(leg, {timeout}, line)
print(__import__("json").dumps(line), flush=True)
"""


@pytest.mark.parametrize("sleep,timeout", [(0, 30), (30, 1)])
def test_bounded_leg_keeps_stdout_to_one_line(sleep, timeout):
    """The `c_host_multi` leg (one process over every device of the node) runs
    last, its libraries' stdout (RCCL's version banner) goes to stderr, and if
    it hangs past the timeout the watchdog prints the line without it and the
    process exits 0: stdout always holds exactly one JSON line."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = _LEG_CHILD.format(root=root, sleep=sleep, timeout=timeout)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = p.stdout.strip().splitlines()
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert "RCCL version" in p.stderr and "from python" in p.stderr
    if sleep:
        assert "timed out" in out["c_host_multi"]["error"]
    else:
        assert out["c_host_multi"] == {"ok": True}
