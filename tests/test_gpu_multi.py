"""The multi-GPU path on the GPU box (BASELINE config 4).

* config 4 at full size on one GPU: the global 8,388,608-frame IMIX batch split
  into byte-balanced contiguous shards (xsknf_amd/shard.py), each shard copied
  into its own buffer with rebased descriptors -- exactly what a rank receives --
  and checksummed through the C ABI; every verdict and byte equals the oracle's
  pass over the whole batch;
* the root distribution (scatter_from_root) with two ranks on gloo, both on
  cuda:0, the HIP kernel run on the shards each rank received;
* `bench.py --gpus N` (N = 2, 4) started by hand on a one-GPU box starts its
  N ranks itself (gloo rehearsal), reports n_gpus = N, splits config 4 N ways
  and delivers every frame of the root distribution.

Processes are started from the forkserver of tests/conftest.py, never from this
(GPU-initialised) process.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle import csum_oracle as O
from tests import oracles
from xsknf_amd import Checksummer, frames
from xsknf_amd.shard import rebase_descs, shard_by_bytes, shard_spans

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
def test_config4_global_batch_in_byte_balanced_shards(dev):
    """BASELINE config 4: 8,388,608 IMIX frames (1 % edge cases), split 8 ways by
    bytes; each shard's span goes to its own buffer with rebased descriptors, as
    scatter_from_root delivers it; the union of the shards' results is the
    oracle's pass over the whole batch, byte for byte."""
    n, world = 8 << 20, 8
    umem, descs, _ = frames.device_batch(n, "imix", layout="aligned", device=dev)
    host = umem.cpu().numpy()
    hd = descs.cpu().numpy().view(frames.DESC_DTYPE).reshape(-1).copy()
    del descs
    b = frames.HostBatch(host, hd, "aligned")
    frames.inject_edge_cases(b, 0.01, seed=404)
    umem.copy_(torch.from_numpy(host))
    size = host.size
    ranges = shard_by_bytes(hd["len"], world)
    spans = shard_spans(hd, ranges, size)
    sums = [int(hd["len"][lo:hi].astype(np.int64).sum()) for lo, hi in ranges]
    assert max(sums) - min(sums) <= 2 * 1500
    gv = np.empty(n, dtype=np.int32)
    cs = Checksummer(frame_len_hint=1500)
    for (lo, hi), (b0, b1) in zip(ranges, spans):
        local = torch.empty(b1 - b0 + 16, dtype=torch.uint8, device=dev)   # a rank's receive buffer
        local[:b1 - b0].copy_(umem[b0:b1])
        ld = rebase_descs(hd[lo:hi], b0, size)
        ldt = torch.from_numpy(ld.view(np.int64).reshape(-1, 2).copy()).to(dev)
        gv[lo:hi] = cs.process_batch(local, ldt).cpu().numpy()
        umem[b0:b1].copy_(local[:b1 - b0])
        del local, ldt
    torch.cuda.synchronize()
    gu = umem.cpu().numpy()                                    # before the CPU oracle
    _, ov = oracles.time_batch(host, hd)      # in place over the whole batch
    assert np.array_equal(gv, ov)
    assert np.array_equal(gu, host)
    assert (ov == -1).sum() > 0 and (ov == 0).sum() > 0.98 * n


def _c_host_multi_run(dev, host, hd, layout, edge_seed=None, mean=0, action=0, nif=1):
    """The global batch through the C host's multi-device calls over every visible
    device (include/xsknf_gpu.h xsknf_gpu_multi_*: ncclCommInitAll, grouped
    ncclSend / ncclRecv from device 0 -- the root's own shard as a send to itself
    --, a launch per device, the counter ncclAllReduce); checked against the
    reference's own pass over the whole batch: every verdict, every byte of every
    shard's span, and the all-reduced counters."""
    from xsknf_amd import ChecksummerOptions, multi
    ndev = torch.cuda.device_count()
    umem = torch.from_numpy(host).to(dev)
    size = host.size
    torch.cuda.synchronize()
    with multi.MultiDevice(range(ndev)) as m:
        secs = m.scatter(0, umem.data_ptr(), size, hd)
        del umem
        ms = m.process(ChecksummerOptions(action=action), num_interfaces=nif, frame_len_max=int(hd["len"].max()),
                       frame_len_mean=mean)
        cnt = m.counters()
        shards = []
        for k in range(ndev):
            info = m.shard_info(k)
            su, sv = m.fetch(k)
            shards.append((info, su, sv))
    ref = host.copy()
    _, ov = oracles.time_batch(ref, hd, action=action, nif=nif)
    ranges = shard_by_bytes(hd["len"], ndev)
    spans = shard_spans(hd, ranges, size)
    for k, (info, su, sv) in enumerate(shards):
        assert (info["frame_lo"], info["frame_hi"]) == ranges[k]
        assert (info["span_lo"], info["span_hi"]) == spans[k]
        assert info["device"] == k
        lo, hi = ranges[k]
        assert np.array_equal(sv, ov[lo:hi]), f"shard {k} verdicts"
        assert np.array_equal(su, ref[spans[k][0]:spans[k][1]]), f"shard {k} bytes"
    assert cnt == multi.expected_counters(ref, hd, ov)
    return secs, ms, cnt, ndev


@pytest.mark.slow
def test_c_host_multi_device_config4(dev):
    """BASELINE config 4 (8,388,608 IMIX frames, aligned 2 KiB chunks, 1 % edge
    cases) through the C host's multi-device path, over
    every device of the box (one on the GPU box: the root's shard moves by an
    RCCL send to itself), bit-exact against the reference's own function over the
    whole batch; the all-reduced counters equal the host's."""
    n = 8 << 20
    b = frames.aligned_batch(n, "imix", seed=frames.SEED)
    frames.inject_edge_cases(b, 0.01, seed=405)
    secs, ms, cnt, ndev = _c_host_multi_run(dev, b.umem, b.descs, "aligned", mean=int(b.descs["len"].mean()))
    assert cnt["frames"] == n and cnt["forward"] > 0.98 * n and cnt["drop"] > 0
    assert secs > 0 and len(ms) == ndev and all(t > 0 for t in ms)
    print(f"c-host multi: {ndev} device(s), scatter {secs * 1e3:.1f} ms, process {ms} ms")


@pytest.mark.parametrize("case", ["unaligned-edges", "jumbo", "out-of-range", "drop-2if", "one-frame"])
def test_c_host_multi_device_cases(dev, case):
    """Smaller batches through the same path: packed unaligned frames (odd starts)
    with 10 % edge cases, jumbo frames, descriptors outside the UMEM (verdict -1,
    no byte), DROP with two interfaces, a single frame."""
    action, nif = 0, 1
    if case == "unaligned-edges":
        b = frames.unaligned_batch(20000, "imix", seed=51)
        frames.inject_edge_cases(b, 0.1, seed=52)
    elif case == "jumbo":
        b = frames.unaligned_batch(3000, 9000, seed=53)
    elif case == "out-of-range":
        b = frames.aligned_batch(5000, "imix", seed=54)
        b.descs["addr"][::37] += np.uint64(1 << 40)
    elif case == "drop-2if":
        b = frames.aligned_batch(5000, 1500, seed=55)
        action, nif = 1, 2
    else:
        b = frames.aligned_batch(1, 570, seed=56)
    _c_host_multi_run(dev, b.umem, b.descs, b.layout, action=action, nif=nif)


def _c_host_packed_round_trip(dev, host, hd, action=0, nif=1, iters=1, mean=0, base_off=0, process_first=False):
    """The global batch out and back through the C host's multi-device calls over
    every visible device: xsknf_gpu_multi_scatter_packed (each shard's frames
    packed into 16-byte slots on the root, then grouped ncclSend / ncclRecv),
    xsknf_gpu_multi_return (each device's records-only pass, its records sent to
    the root, applied there).  Checked: every shard holds exactly its frames'
    bytes before the pass; afterwards the root's UMEM and verdicts equal the
    reference's own pass over the whole batch, byte for byte."""
    from xsknf_amd import ChecksummerOptions, _lib, multi
    ndev = torch.cuda.device_count()
    # the root's UMEM `base_off` bytes into its allocation (a base that is not
    # 16-byte aligned: frames whose first 16-byte chunk starts before it)
    big = torch.zeros(host.size + base_off + 64, dtype=torch.uint8, device=dev)
    umem = big[base_off:base_off + host.size]
    umem.copy_(torch.from_numpy(host))
    n = hd.shape[0]
    v = torch.full((max(n, 1),), 0x7eadbeef, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    a = hd["addr"].astype(np.uint64)
    off = ((a & np.uint64((1 << 48) - 1)) + (a >> np.uint64(48))).astype(np.int64)
    ln = hd["len"].astype(np.int64)
    inr = (off <= host.size) & (ln <= host.size - np.minimum(off, host.size))
    rng = np.random.default_rng(n)
    with multi.MultiDevice(range(ndev)) as m:
        secs = m.scatter_packed(0, umem.data_ptr(), umem.numel(), hd)
        moved = 0
        for k in range(ndev):
            info = m.shard_info(k)
            assert info["flags"] == _lib.SHARD_PACKED and info["device"] == k
            su, sv, sd = m.fetch(k, descs=True)
            lo, hi = info["frame_lo"], info["frame_hi"]
            moved += su.size
            assert np.array_equal(sd["len"], hd["len"][lo:hi]) and np.array_equal(sd["options"], hd["options"][lo:hi])
            idx = np.arange(lo, hi)
            if idx.size > 3000:
                idx = np.sort(rng.choice(idx, 3000, replace=False))
            for f in idx:
                if not inr[f]:
                    assert sd["addr"][f - lo] >= su.size
                    continue
                p, L = int(sd["addr"][f - lo]), int(ln[f])
                assert p % 16 == (umem.data_ptr() + int(off[f])) % 16
                assert np.array_equal(su[p:p + L], host[off[f]:off[f] + L]), f"frame {f} packed bytes"
        if process_first:
            # the shards checksummed in place first: a return now would describe a
            # second pass, so it is refused (-EBUSY) until the batch is scattered again
            m.process(ChecksummerOptions(action=action, csum_iterations=iters), num_interfaces=nif,
                      frame_len_max=int(hd["len"].max()) if n else 0)
            with pytest.raises(_lib.XsknfGpuError, match="rc=-16"):
                m.return_results(umem.data_ptr(), v.data_ptr())
            m.scatter_packed(0, umem.data_ptr(), umem.numel(), hd)
        ms, secs2 = m.return_results(umem.data_ptr(), v.data_ptr(), ChecksummerOptions(action=action,
                                                                                         csum_iterations=iters),
                                     num_interfaces=nif, frame_len_max=int(hd["len"].max()) if n else 0,
                                     frame_len_mean=mean)
        with pytest.raises(_lib.XsknfGpuError):
            m.counters()   # -EOPNOTSUPP after a packed scatter
    ref = host.copy()
    _, ov = oracles.time_batch(ref, hd, action=action, nif=nif, iters=iters)
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy()[:n], ov), "verdicts"
    assert np.array_equal(umem.cpu().numpy(), ref), "root UMEM"
    return secs, secs2, ms, moved


@pytest.mark.slow
def test_c_host_packed_round_trip_config4(dev):
    """BASELINE config 4 (8,388,608 IMIX frames in 2 KiB chunks, 1 % edge cases)
    out of the root packed and back as records: the root's UMEM and verdicts equal
    the reference's pass over the whole batch, and the packed shards moved ~1/5
    of the span bytes (the 2 KiB chunks' gaps stay home)."""
    n = 8 << 20
    b = frames.aligned_batch(n, "imix", seed=frames.SEED)
    frames.inject_edge_cases(b, 0.01, seed=406)
    secs, secs2, ms, moved = _c_host_packed_round_trip(dev, b.umem, b.descs, mean=int(b.descs["len"].mean()))
    frame_bytes = int(b.descs["len"].astype(np.int64).sum())
    assert frame_bytes <= moved < 1.1 * frame_bytes + 16 * n
    print(f"c-host packed: moved {moved / 1e9:.2f} GB for {frame_bytes / 1e9:.2f} GB of frames "
          f"(span {b.umem.size / 1e9:.1f} GB), scatter {secs * 1e3:.1f} ms, return {secs2 * 1e3:.1f} ms, pass {ms} ms")


@pytest.mark.parametrize("case", ["unaligned-edges", "jumbo", "out-of-range", "drop-2if", "one-frame", "64B-iter3",
                                  "ihl-overlap", "empty", "odd-base-and-end", "processed-first"])
def test_c_host_packed_round_trip_cases(dev, case):
    """Packed frames at odd addresses (unaligned UMEM, 10 % edge cases), jumbo
    frames, descriptors outside the UMEM, DROP with two interfaces, one frame,
    64-B frames (the lane kernel's records) with 3 iterations, frames whose UDP
    header overlaps the IP header (ihl 2 / 3), an empty batch."""
    action, nif, iters = 0, 1, 1
    if case == "unaligned-edges":
        b = frames.unaligned_batch(20000, "imix", seed=61)
        frames.inject_edge_cases(b, 0.1, seed=62)
    elif case == "jumbo":
        b = frames.unaligned_batch(3000, 9000, seed=63)
    elif case == "out-of-range":
        b = frames.aligned_batch(5000, "imix", seed=64)
        b.descs["addr"][::37] += np.uint64(1 << 40)
    elif case == "drop-2if":
        b = frames.aligned_batch(5000, 1500, seed=65)
        action, nif = 1, 2
    elif case == "one-frame":
        b = frames.aligned_batch(1, 570, seed=66)
    elif case == "64B-iter3":
        b = frames.aligned_batch(30000, 64, seed=67)
        iters = 3
    elif case == "ihl-overlap":
        b = frames.unaligned_batch(4000, "imix", seed=68)
        frames.inject_edge_cases(b, 0.3, seed=69)
    elif case == "processed-first":
        b = frames.aligned_batch(20000, "imix", seed=72)
        frames.inject_edge_cases(b, 0.05, seed=73)
        _c_host_packed_round_trip(dev, b.umem, b.descs, process_first=True)
        return
    elif case == "empty":
        b = frames.aligned_batch(1, 570, seed=70)
        b = frames.HostBatch(b.umem, b.descs[:0].copy(), b.layout)
    else:
        # packed frames from the UMEM's first byte to its last, the UMEM 7 bytes
        # into its allocation: the first and last 16-byte chunks reach outside it
        b = frames.unaligned_batch(3000, "imix", seed=71)
        a = b.descs["addr"]
        off = (a & np.uint64((1 << 48) - 1)) + (a >> np.uint64(48))
        b.descs["addr"] = off - off[0]          # (aligned-mode addresses: plain offsets)
        end = int((b.descs["addr"] + b.descs["len"]).max())
        umem = b.umem[int(off[0]):int(off[0]) + end].copy()
        _c_host_packed_round_trip(dev, umem, b.descs, base_off=7)
        return
    _c_host_packed_round_trip(dev, b.umem, b.descs, action=action, nif=nif, iters=iters)


def _run_tool(cmd, timeout):
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout, p.stderr


@pytest.mark.parametrize("frames_n", [1, 65537, 1 << 20])
def test_c_host_tool_config4_shape(dev, clean_ctx, frames_n):
    """tools/multi_config4.c: a C host drives the multi-device calls itself
    (xsknf_gpu_multi_create / _scatter / _process / _counters, then
    _scatter_packed / _return), over every device of the box, on an IMIX batch in
    config 4's layout; its own check against the CPU oracle -- the all-reduced
    counters, the root's UMEM and verdicts after the return -- must hold.  (Run
    from the forkserver, never from this GPU-initialised process.)"""
    tool = os.path.join(ROOT, "tools", "build", "multi_config4")
    if not os.path.exists(tool):
        pytest.fail(f"{tool} is not built (make tools)")
    with clean_ctx.Pool(1) as pool:
        rc, out, err = pool.apply(_run_tool, ([tool, str(frames_n)], 300))
    assert rc == 0, (out, err[-2000:])
    r = json.loads(out.strip().splitlines()[-1])
    assert r["frames"] == frames_n and r["counters_match"] and r["root_umem_match"] and r["verdicts_match"]
    assert r["frame_bytes"] <= r["packed_bytes"] <= r["frame_bytes"] + 31 * frames_n


def _scatter_rank(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    from xsknf_amd.shard import scatter_from_root
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    umem = descs = ranges = None
    if rank == 0:
        b = frames.unaligned_batch(6000, "imix", seed=31)
        frames.inject_edge_cases(b, 0.05, seed=32)
        umem, descs = torch.from_numpy(b.umem.copy()), b.descs
        ranges = shard_by_bytes(b.descs["len"], world)
    lu, ld, (b0, b1) = scatter_from_root(dist, umem, descs, ranges, rank, world, "cpu")
    dev = torch.device("cuda:0")
    lu, ld = lu.to(dev), ld.to(dev)
    v = Checksummer(frame_len_hint=1500).process_batch(lu, ld)
    torch.cuda.synchronize()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), b0=b0, b1=b1, umem=lu[:b1 - b0].cpu().numpy(),
             v=v.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_root_scatter_two_ranks_hip_kernel(dev, clean_ctx, tmp_path):
    """scatter_from_root over gloo with two ranks on cuda:0; each rank runs the
    HIP kernel on the shard it received; bytes and verdicts equal the oracle's
    pass over the whole batch on the root."""
    world, port = 2, _free_port()
    procs = [clean_ctx.Process(target=_scatter_rank, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    b = frames.unaligned_batch(6000, "imix", seed=31)
    frames.inject_edge_cases(b, 0.05, seed=32)
    ranges = shard_by_bytes(b.descs["len"], world)
    full = b.umem.copy()
    fv = O.c_process_batch(full, b.descs)
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        lo, hi = ranges[r]
        assert np.array_equal(z["v"], fv[lo:hi]), f"rank {r} verdicts"
        assert np.array_equal(z["umem"], full[int(z["b0"]):int(z["b1"])]), f"rank {r} bytes"


def _run(cmd, env, timeout):
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout, p.stderr


@pytest.mark.parametrize("world", [2, 4])
def test_bench_gpus_n_starts_its_ranks(dev, clean_ctx, world):
    """`python bench.py --gpus N` (no torch.distributed.run around it) starts N
    ranks itself (the reference's one worker per queue, src/xsknf.c:1046-1100);
    on a one-GPU box they rehearse over gloo; rank 0 reports n_gpus = N and
    every rank's frames, config 4's global batch is split N ways by bytes (rank
    0 holds exactly shard_by_bytes' first range), and the root distribution
    delivers every frame and matches the single-GPU pass."""
    from xsknf_amd import frames as F
    from xsknf_amd.shard import shard_by_bytes
    env = dict(os.environ)
    if torch.cuda.device_count() < world:
        env["XSKNF_BENCH_BACKEND"] = "gloo"
    c4 = 131072
    cmd = [sys.executable, "bench.py", "--gpus", str(world), "--steps", "3", "--warmup", "1", "--frames", "65536",
           "--secondary", "config4", "--config4-frames", str(c4), "--cpu-seconds", "0", "--kernel-steps", "0",
           "--min-warmup-s", "0"]
    with clean_ctx.Pool(1) as pool:
        rc, out, err = pool.apply(_run, (cmd, env, 400))
    assert rc == 0, err[-3000:]
    line = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == world
    assert line["config"]["global_batch"] == world * 65536
    assert line["verdicts"]["forward"] == world * 65536
    assert line["secondary"]["config4"]["frames"] == c4
    glens = F.imix_lengths(c4, np.random.default_rng(F.SEED))
    assert line["secondary"]["config4"]["rank0_shard"] == list(shard_by_bytes(glens, world)[0])
    assert line["roofline"]["frac"] > 0
    # self-checking multi-rank line: the backend saw every rank, and the root
    # distribution ran by default and delivered every frame
    assert line["dist"]["ranks_seen"] == world and line["dist"]["world_size"] == world
    assert line["dist"]["frames_allreduced"] == world * 65536
    # every rank's own step is in the line (a straggler is visible), consistent with the max
    pr = line["dist"]["per_rank"]
    assert len(pr["step_us"]) == world and len(pr["wall_ms_per_step"]) == world
    assert pr["frames"] == [65536] * world and all(x > 0 for x in pr["gbs_checksummed"])
    assert line["dist"]["step_us_max"] == max(pr["step_us"]) and line["dist"]["step_us_min"] == min(pr["step_us"])
    assert line["dist"]["step_spread"] >= 1.0
    assert line["dist"]["sum_of_rank_rates_gbs"] >= line["dist"]["per_rank_gbs_mean"] > 0
    assert abs(line["ms_per_step"] - max(pr["wall_ms_per_step"])) <= 1e-3 * max(1.0, line["ms_per_step"])
    # both time bases of the roofline, named
    assert 0 < line["roofline"]["frac_wall"] and "frac_wall" in line["roofline"]["basis"]
    assert line["root_scatter"]["frames_total"] == world * 65536
    assert line["root_scatter"]["vs_single_gpu"]["match"] is True
    assert line["root_scatter"]["rfc_check"]["violations"] == 0


def test_rccl_collectives_on_one_gpu(dev, clean_ctx):
    """The RCCL branch of bench.py on the MI355X itself: one rank under
    torch.distributed.run with XSKNF_BENCH_DIST=1 brings the "nccl" process
    group up (init_process_group(device_id=...)), and the run goes through the
    same collectives as at N > 1 -- barriers, device-tensor all-reduces, the
    root distribution's broadcast (`shard.scatter_from_root`, device tensors)
    and the HIP kernel on the shard it hands back, checked against the
    single-GPU pass by the fingerprint.  (N > 1 over xGMI needs a multi-GPU
    node: the driver's SCALE run.)"""
    port = _free_port()
    env = dict(os.environ, XSKNF_BENCH_DIST="1")
    env.pop("XSKNF_BENCH_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={port}", "bench.py", "--gpus", "1", "--steps", "3",
           "--warmup", "1", "--frames", "65536", "--secondary", "", "--cpu-seconds", "0", "--kernel-steps", "0",
           "--min-warmup-s", "0", "--no-probes"]
    with clean_ctx.Pool(1) as pool:
        rc, out, err = pool.apply(_run, (cmd, env, 400))
    assert rc == 0, err[-3000:]
    line = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])
    assert line["dist"]["backend"] == "nccl"
    assert line["dist"]["collective_device"] == "cuda"
    assert line["dist"]["ranks_seen"] == 1 and line["dist"]["world_size"] == 1
    assert line["dist"]["frames_allreduced"] == 65536
    assert line["root_scatter"]["frames_total"] == 65536
    assert line["root_scatter"]["vs_single_gpu"]["match"] is True
    assert line["root_scatter"]["rfc_check"]["violations"] == 0
