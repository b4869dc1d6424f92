#!/usr/bin/env python3
"""Device-resident throughput of the checksummer batch path (BASELINE.json metric).

One step = one pass of the hot path (xsknf_packet_processor over every frame of
one rx batch, checksummer_user.c:30-112, as the per-frame loop of
src/xsknf.c:654-672 calls it) over a batch already resident in HBM.
Default workload = BASELINE config 3: 1,048,576 frames of 1500 B per GPU in an
aligned UMEM (2048 B chunks, data at +256).  Each rank processes its own batch
(frames shard with no exchange, as one xsknf worker per NIC queue does,
src/xsknf.c:1046-1100), so `scaling` is weak and `value` is the aggregate.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload 1500|64|imix|jumbo]

--gpus N > 1 without a torch.distributed.run environment starts the N ranks
itself (one process per GPU, RCCL); the parent never touches the GPU.  On a box
with fewer than N GPUs the ranks share the devices over gloo (a rehearsal of
the N-rank path, marked `rehearsal` in the line).  Rank 0 prints ONE JSON line.

Secondary workloads (timed after the primary, reported under `secondary`, each
with its step fraction, kernel and committed PMC traffic): 64 B (config 2), a
1M-frame IMIX batch (config 4's per-GPU shard), 9000 B jumbo frames in an
unaligned UMEM (config 5), and config 4 -- the global 8,388,608-frame IMIX batch
split into byte-balanced contiguous shards, one per rank (all of it on one GPU
at N = 1, exactly config 4's 8-way split at N = 8); the NIC-checksummed variants
(`*-nic`); and `64-13M`, config 2's frames as one 13M-frame batch (one
lane-kernel launch instead of 13: what a 64 B step costs without its launch's
ramp and drain).

At world 1 the line ends with `c_host_multi`: config 4 through the C host's
multi-device calls over every visible device of this one process (span
scatter, in-place steps, all-reduced counters; then the frames-only packed
scatter and the results' return, checked byte for byte against one device's
pass), run last behind a watchdog so that it cannot cost the line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

# pageable host copies through HIP's own staging buffers, not by locking the
# caller's pages (the runtime path behind the GPU suite's faults);
# before the first HIP call
os.environ.setdefault("GPU_PINNED_MIN_XFER_SIZE", "1048576")

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from xsknf_amd import Checksummer, ChecksummerOptions, frames  # noqa: E402
from xsknf_amd.shard import shard_by_bytes  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
DESC_BYTES, VERDICT_BYTES, CHECK_BYTES = 16, 4, 2
CONFIG4_FRAMES = 8 * (1 << 20)  # BASELINE config 4: 8,388,608 IMIX frames over the node

WORKLOADS = {
    # name: (length, layout, chunk, description)
    "1500": (1500, "aligned", 2048, "BASELINE config 3: 1500 B frames, aligned UMEM 2048 B chunks, data at +256"),
    "64": (64, "aligned", 2048, "BASELINE config 2: 64 B frames, aligned UMEM 2048 B chunks, data at +256"),
    "570": (570, "aligned", 2048, "IMIX's middle size class alone: 570 B frames, aligned UMEM 2048 B chunks"),
    "imix": ("imix", "aligned", 2048, "IMIX 64/570/1500 B (7:4:1), 1M frames per GPU, aligned 2048 B chunks"),
    "jumbo": (9000, "unaligned", 0, "BASELINE config 5: 9000 B frames, unaligned-chunk UMEM, ~50% odd starts"),
    "64-13M": (64, "aligned", 2048, "BASELINE config 2's frames (64 B, aligned UMEM 2048 B chunks) as ONE batch of "
                                    "13 x the per-GPU frames: one lane-kernel launch, one ramp and drain for all of it"),
    "config4": ("imix", "aligned", 2048,
                "BASELINE config 4: 8,388,608 IMIX 64/570/1500 B frames (7:4:1) split into byte-balanced "
                "contiguous shards, one per GPU, aligned 2048 B chunks"),
}
# The same batches with the UDP checksums a NIC's transmit offload fills in, as
# the reference's own traffic carries them (tests/gen-traffic.lua:120,
# bufs:offloadUdpChecksums()): the checksummer computes the value the frame
# already holds for all but the frames whose single fold loses a carry
# (checksummer_user.c:105-106), and the kernels leave those frames untouched.
# The base workloads (checks 0 in every frame, so every check changes) are the
# worst case and stay the headline.
NIC = {"1500-nic": "1500", "imix-nic": "imix", "64-nic": "64", "jumbo-nic": "jumbo"}
for _k, _b in NIC.items():
    _l, _lay, _c, _d = WORKLOADS[_b]
    WORKLOADS[_k] = (_l, _lay, _c, _d + "; UDP checksums as a NIC offload writes them (gen-traffic.lua:120)")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--workload", default="1500", choices=sorted(WORKLOADS))
    p.add_argument("--frames", type=int, default=1 << 20, help="frames per GPU (config4: global frames "
                   f"= {CONFIG4_FRAMES} unless --config4-frames)")
    p.add_argument("--config4-frames", type=int, default=CONFIG4_FRAMES)
    p.add_argument("--secondary", default="64,imix,jumbo,config4,1500-nic,imix-nic,64-nic,jumbo-nic,64-13M",
                   help="comma list of extra workloads timed after the primary ('' = none)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=1)
    p.add_argument("--cpu-all-cores", type=int, default=-1,
                   help="threads for the all-cores CPU leg (-1 = the process's CPUs, at most 16; 0 = skip)")
    p.add_argument("--min-warmup-s", type=float, default=0.1,
                   help="keep warming up (untimed) until this much time has passed")
    p.add_argument("--primary-warmup-s", type=float, default=1.0,
                   help="the same for the primary workload (1500 B on one box: 278.4 us after 3 s of warmup "
                        "twice, 278.4 and 281.5 after 0.1 s)")
    p.add_argument("--no-root-scatter", action="store_true",
                   help="N > 1: skip the distribution of a root-resident global IMIX batch (SURVEY 8(e) "
                        "collective 1, reported as `root_scatter`; timed by default when N > 1)")
    p.add_argument("--no-probes", action="store_true", help="skip the read / step-floor probes")
    p.add_argument("--no-c-host-multi", action="store_true",
                   help="world 1: skip config 4 through the C host's multi-device calls (`c_host_multi`)")
    p.add_argument("--c-host-multi-timeout", type=float, default=240.0,
                   help="seconds before the `c_host_multi` leg is abandoned (the line is printed without it)")
    p.add_argument("--no-verify", action="store_true",
                   help="skip the RFC receive-side check of the primary and config4 outputs (rfc_check)")
    p.add_argument("--rotate", type=int, default=0,
                   help="batches the steps cycle through (0 = enough to exceed --rotate-bytes)")
    p.add_argument("--rotate-bytes", type=int, default=1 << 30)
    p.add_argument("--streams", type=int, default=1,
                   help="launch streams the steps rotate over (batches are independent: with 2, one batch's "
                        "launch starts while the previous one drains; needs >= 2 rotated batches)")
    p.add_argument("--kernel-steps", type=int, default=50,
                   help="launches of the summing kernel alone (records only), reported beside the step")
    return p.parse_args()


# ---- rank launch --------------------------------------------------------------

def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """`--gpus N` (N > 1) outside a torch.distributed.run environment: start the
    N ranks as a child torch.distributed.run and return its exit code.  This
    process only counts devices (torch.cuda.device_count() does not initialise
    the GPU) and never execs: the ranks are a child process."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    env = dict(os.environ)
    ndev = torch.cuda.device_count()
    if ndev < args.gpus and "XSKNF_BENCH_BACKEND" not in env:
        env["XSKNF_BENCH_BACKEND"] = "gloo"
        print(f"bench: {args.gpus} ranks on {ndev} GPU(s): gloo rehearsal, ranks share devices",
              file=sys.stderr)
    env.setdefault("OMP_NUM_THREADS", "4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd, env=env)


_DIST = False   # a process group is up (world > 1, or XSKNF_BENCH_DIST=1 at world 1)


def dist_setup(args):
    """One process per GPU (torch.distributed.run env).  XSKNF_BENCH_BACKEND=gloo
    rehearses the N > 1 path on fewer GPUs (ranks share devices round robin);
    the default is nccl (RCCL), one rank per GPU.  XSKNF_BENCH_DIST=1 brings the
    process group up at world 1 too, so that the collectives (RCCL's init,
    barrier, device-tensor all-reduces and broadcast, the root-distribution leg)
    run on a one-GPU box exactly as at N > 1."""
    global _DIST
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("XSKNF_BENCH_BACKEND", "nccl")
    ndev = max(1, torch.cuda.device_count())
    if backend != "nccl":
        local %= ndev
    _DIST = world > 1 or (os.environ.get("XSKNF_BENCH_DIST") == "1" and "MASTER_ADDR" in os.environ)
    if _DIST:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using {world}", file=sys.stderr)
    rehearsal = None
    if world > 1 and backend != "nccl":
        rehearsal = f"{backend}: {world} ranks on {min(world, ndev)} GPU(s); timings are contended, not a scaling point"
    return world, rank, torch.device("cuda", local), rehearsal


def barrier(world):
    if _DIST:
        dist.barrier()
    torch.cuda.synchronize()


def coll_device():
    """Where collective operands live: HBM for RCCL, host memory for gloo."""
    return "cuda" if os.environ.get("XSKNF_BENCH_BACKEND", "nccl") == "nccl" else "cpu"


def allreduce_max(x: float, world: int) -> float:
    if not _DIST:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allgather_f64(vals, world):
    """Every rank's `vals` (a list of floats), as a list per rank (rank order)."""
    t = torch.tensor(vals, dtype=torch.float64, device=coll_device())
    if not _DIST:
        return [t.tolist()]
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [p.tolist() for p in parts]


def allreduce_sum_i64(vals, world):
    t = torch.tensor(vals, dtype=torch.int64, device=coll_device())
    if _DIST:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(x) for x in t.tolist()]


# ---- one workload ---------------------------------------------------------------

def workload_lengths(name, args, world, rank):
    """This rank's frame lengths (and, for config4, its [lo, hi) of the global batch)."""
    length, layout, chunk, _ = WORKLOADS[name]
    if name == "config4":
        glens = frames.imix_lengths(args.config4_frames, np.random.default_rng(frames.SEED))
        lo, hi = shard_by_bytes(glens, world)[rank]
        return glens[lo:hi].astype(np.uint32), (lo, hi)
    n = args.frames * (13 if name == "64-13M" else 1)
    return frames._lens(n, length, np.random.default_rng(frames.SEED + rank)), None


def rotation(lens: np.ndarray, args) -> int:
    """Batches the steps cycle through: enough that what one pass touches (the
    frames' 64-B sectors, descriptors, verdicts) times K exceeds --rotate-bytes,
    so a step never finds the previous pass's bytes in the 256 MiB Infinity
    Cache -- a 1M-frame 64 B batch touches 84 MB, and re-reading it step after
    step would be served partly on-die.  A 1500 B batch (1.6 GB) needs K = 1."""
    if args.rotate > 0:
        return args.rotate
    touched = int(((lens.astype(np.int64) + 63) // 64 * 64).sum()) + 20 * lens.shape[0]
    return int(min(16, max(1, -(-args.rotate_bytes // max(1, touched)))))


def batches_and_streams(name, lens_in, args):
    """(K rotated batches, S launch streams).  With S > 1, steps in flight
    together own distinct batches and every visit of a batch goes to the same
    stream (K a multiple of S), so the visits of a batch stay ordered.  NIC
    workloads time each step by its own events: one stream."""
    K = rotation(lens_in, args)
    S = args.streams if name not in NIC else 1
    if S > 1:
        K = -(-max(K, S) // S) * S
    return K, S


def iterations_of_step(it: int, K: int) -> int:
    """csum_iterations of step `it` of a base workload: each visit of a batch
    (step it touches batch it % K) alternates 1 and 2, so every check the
    previous visit wrote changes again."""
    return 1 + ((it // K) & 1)


def time_workload(name, args, world, rank, dev, seed, primary):
    length, layout, chunk, desc = WORKLOADS[name]
    lens_in, span = workload_lengths(name, args, world, rank)
    n = int(lens_in.shape[0])
    K, S = batches_and_streams(name, lens_in, args)
    # K batches of the same shape in one UMEM (batch j = frames [j*n, (j+1)*n)),
    # step i processes batch i % K
    umem, descs, lens = frames.device_batch(n * K, np.tile(lens_in, K), layout=layout, chunk=chunk or frames.CHUNK,
                                            seed=seed, device=dev)
    if name in NIC:
        frames.offload_checks_device(umem, descs)
    # the caller knows its batch: longest frame and mean length (xsknf_gpu_checksum_batch_lens)
    hint, mean = int(lens.max()), int(lens_in.mean())
    cs = Checksummer(ChecksummerOptions(), num_interfaces=1, frame_len_hint=hint, frame_len_mean=mean)
    # A frame that already holds the check the kernel computes is left untouched
    # (include/xsknf_gpu.h), so a pass over a batch the previous pass just
    # checksummed would write nothing.  Every step must see its frames as they
    # arrive (inputs reset between repeats):
    # * base workloads (checks 0, every one changes): each visit of a batch
    #   alternates csum_iterations 1 and 2, so every check the previous visit
    #   wrote changes again -- the step's work is that of fresh frames (the
    #   kernel's cost does not depend on the iteration count: closed form);
    # * NIC workloads: the checks a step changes (the carry-loss frames, 0.005 %
    #   of 64 B frames to 3.7 % of jumbo frames) are put back after it on the
    #   launch stream, and each step is timed by its own HIP events around its
    #   launch only (the put-back is test scaffolding: an index_put and its
    #   launch gap, ~7 us per step; putting them back on a side stream while the
    #   next batch ran instead measured slower, its cross-stream waits sitting
    #   between the steps).
    cs_alt = Checksummer(ChecksummerOptions(csum_iterations=2), num_interfaces=1, frame_len_hint=hint,
                         frame_len_mean=mean)
    nic = name in NIC
    verdicts = torch.empty(n * K, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    umem_ptr, umem_size = umem.data_ptr(), umem.numel()
    descs_ptrs = [descs.data_ptr() + 16 * n * j for j in range(K)]
    v_ptrs = [verdicts.data_ptr() + 4 * n * j for j in range(K)]
    batch_bytes = [int(lens[j * n:(j + 1) * n].sum()) for j in range(K)]

    # a bounded host sample of the ORIGINAL frames for the CPU baseline leg
    sample = None
    if primary and rank == 0 and world == 1 and args.cpu_seconds > 0:
        k = min(n, 1 << 16)
        dk = descs[:k].cpu().numpy().view(frames.DESC_DTYPE).reshape(-1)
        offs = (dk["addr"] & np.uint64((1 << 48) - 1)) + (dk["addr"] >> np.uint64(48))
        hi = int((offs + dk["len"]).max())
        sample = (umem[:hi].cpu().numpy(), dk, k)

    restore = []   # NIC: per batch, (UMEM positions, NIC bytes) of the checks a pass changes
    if nic:
        addr = descs[:, 0]
        starts = (addr & ((1 << 48) - 1)) + ((addr >> 48) & 0xFFFF)
        at = torch.stack([starts + 40, starts + 41], 1).reshape(-1).clamp_(max=umem_size - 1)
        orig = umem[at]
        for j in range(K):
            cs.process_batch_ptr(umem_ptr, umem_size, descs_ptrs[j], n, v_ptrs[j], 0, stream.cuda_stream)
        for j in range(K):
            sl = slice(2 * n * j, 2 * n * (j + 1))
            ch = umem[at[sl]] != orig[sl]
            restore.append((at[sl][ch].clone(), orig[sl][ch].clone()))
            umem[restore[j][0]] = restore[j][1]
        del addr, starts, at, orig
        torch.cuda.synchronize()

    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    it = [0]
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps if nic else 0)]

    def step():
        j = it[0] % K
        c = cs_alt if (not nic and iterations_of_step(it[0], K) == 2) else cs
        if nic:
            evs[it[0] % len(evs)][0].record(stream)
        c.process_batch_ptr(umem_ptr, umem_size, descs_ptrs[j], n, v_ptrs[j], 0, streams[it[0] % S].cuda_stream)
        if nic:
            evs[it[0] % len(evs)][1].record(stream)
            if restore[j][0].numel():
                umem[restore[j][0]] = restore[j][1]   # this batch's changed checks, back as the NIC wrote them
        it[0] += 1

    # W untimed warmup steps, continued until at least --min-warmup-s of
    # warmup has run: measured on MI355X, 10 steps (3 ms) leave the step ~3 %
    # slower than after 30 ms (clocks still ramping)
    t_w = time.perf_counter()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    warm_s = max(args.min_warmup_s, args.primary_warmup_s if primary else 0.0)
    while time.perf_counter() - t_w < warm_s:
        for _ in range(10):
            step()
        torch.cuda.synchronize()
    barrier(world)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    first = it[0]
    ev0.record(stream)
    for st in streams[1:]:
        st.wait_event(ev0)
    for _ in range(args.steps):
        step()
    for st in streams[1:]:
        e = torch.cuda.Event()
        e.record(st)
        stream.wait_event(e)
    ev1.record(stream)
    barrier(world)
    wall = time.perf_counter() - t0
    # frame bytes of the timed steps (the K batches differ slightly in length mix)
    bytes_len = sum(batch_bytes[i % K] for i in range(first, first + args.steps)) // args.steps
    # NIC: the last args.steps steps were the timed ones, each between its own events
    step_ms = (sum(a.elapsed_time(b) for a, b in evs) if nic else ev0.elapsed_time(ev1)) / args.steps
    wall_max = allreduce_max(wall, world)
    step_ms_max = allreduce_max(step_ms, world)
    # every rank's own step (HIP events) and wall time, and its bytes: a straggler
    # rank shows in the line (dist.per_rank), not only in the max
    per_rank = allgather_f64([step_ms, wall / args.steps * 1e3, float(bytes_len), float(n)], world)
    if not nic:
        # leave batch 0 as one -i 1 pass leaves it (the CPU leg checks it)
        cs.process_batch_ptr(umem_ptr, umem_size, descs_ptrs[0], n, v_ptrs[0], 0, stream.cuda_stream)
        torch.cuda.synchronize()

    # the summing kernel alone, for reference beside the step: records-only
    # mode (include/xsknf_gpu.h fused_stores = 3), same shape, same stream, HIP
    # events around K launches (it only reads the UMEM).  For frames >= 1024 B
    # it is exactly the step's first kernel; a single-kernel shape (checks
    # in-line, fused_stores mode 1) has no second kernel: its step IS the kernel.
    import ctypes
    from xsknf_amd import _lib
    lib = _lib.load()
    cfg = cs.launch_cfg()
    # one launch per step: every check in-line (mode 1), or deferred and patched
    # in the same launch once the waves' streams are done (+16, split kernel)
    single_kernel = (cfg.fused_stores & 3) == 1 or bool(cfg.fused_stores & 16)
    stores = ("checks in-line" if (cfg.fused_stores & 3) == 1 else
              ("checks deferred, patched from the block's queue by waves done streaming"
               if cfg.kernel == 1 and cfg.window_chunks & 32 else
               "checks deferred, each wave patches its own tiles") if cfg.fused_stores & 16 else
              "checks deferred to a scatter_checks launch")
    family = ("checksum_kernel_split" if cfg.kernel == 1 else
              "checksum_kernel_lane" if cfg.lanes_per_frame == 1 else "checksum_kernel")
    if cfg.kernel == 1 and cfg.window_chunks & 32:
        family += ", one block per CU, tile pool"
    k_ms = None
    if args.kernel_steps > 0 and (cfg.fused_stores & 3) != 1:
        cfg.fused_stores = 3
        rec = torch.empty(n, dtype=torch.int32, device=dev)
        opts = cs.csum_opts()

        kit = [0]

        def kstep():
            j = kit[0] % K
            kit[0] += 1
            rc = lib.xsknf_gpu_checksum_batch_cfg(
                ctypes.c_void_p(umem_ptr), umem_size, ctypes.c_void_p(descs_ptrs[j]), n, 0, ctypes.byref(opts),
                ctypes.c_void_p(rec.data_ptr()), ctypes.byref(cfg), ctypes.c_void_p(stream.cuda_stream))
            _lib.check(rc, "records-only launch")

        for _ in range(3):
            kstep()
        barrier(world)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.kernel_steps):
            kstep()
        e1.record(stream)
        barrier(world)
        k_ms = e0.elapsed_time(e1) / args.kernel_steps
        del rec

    vh = verdicts[:n].cpu().numpy()
    counters = allreduce_sum_i64([n, bytes_len, int((vh == -1).sum()), int((vh >= 0).sum())], world)
    # batch 0 has just had a -i 1 pass (NIC workloads: every pass is -i 1)
    rfc = rfc_verify(umem, descs, n, world) if (primary or name == "config4") and not args.no_verify else None
    shape = {"lanes_per_frame": cfg.lanes_per_frame, "chunks_per_lane": cfg.chunks_per_lane,
             "items_in_flight": cfg.frames_per_group, "window_chunks": cfg.window_chunks & 15,
             "tile_pool": bool(cfg.kernel == 1 and cfg.window_chunks & 32),
             "frame_len_max": hint, "frame_len_mean": mean}
    return dict(name=name, desc=desc, n=n, K=K, lens=lens, bytes_len=bytes_len, step_ms=step_ms, stores=stores,
                rfc=rfc,
                shape=shape,
                step_ms_max=step_ms_max, per_rank=per_rank,
                sum_ms=k_ms, single_kernel=single_kernel, family=family, wall_max=wall_max, counters=counters,
                umem=umem, descs=descs, verdicts=verdicts, sample=sample, layout=layout, chunk=chunk, span=span)


def root_scatter_leg(args, world, rank, dev):
    """SURVEY.md 8(e), collective 1 (and BASELINE config 4's shape): the global
    batch -- `--frames` x world IMIX frames, packed (unaligned-mode) -- starts in
    rank 0's HBM; each rank receives its byte-balanced contiguous shard (one
    span + its descriptors, point-to-point over xGMI, all ranks at once) and
    checksums it.  Reported separately from `value`: the device-resident metric
    excludes the distribution, and in the reference frames arrive per NIC queue."""
    from xsknf_amd.shard import scatter_from_root
    n_total = args.frames * world
    umem = descs = ranges = ref = None
    if rank == 0:
        umem, dt, lens = frames.device_batch(n_total, "imix", layout="unaligned", seed=frames.SEED, device=dev)
        descs = dt.cpu().numpy().view(frames.DESC_DTYPE).reshape(-1)
        ranges = shard_by_bytes(lens, world)
        # the single-GPU answer the shards are checked against: the whole batch
        # through one Checksummer on rank 0, after the timed region
        ref = (umem.clone(), dt)
    cdev = coll_device()
    if cdev == "cpu" and umem is not None:     # gloo rehearsal: host tensors
        umem = umem.cpu()
    barrier(world)
    t0 = time.perf_counter()
    lu, ld, (b0, b1) = scatter_from_root(dist, umem, descs, ranges, rank, world, cdev)
    if cdev == "cuda":
        torch.cuda.synchronize()
    barrier(world)
    t_move = allreduce_max(time.perf_counter() - t0, world)
    if cdev == "cpu":
        lu, ld = lu.to(dev), ld.to(dev)
    n_local = ld.shape[0]
    # alternating csum_iterations 1 / 2: every pass changes every check (a pass
    # over frames the previous pass left would write nothing, time_workload)
    css = [Checksummer(ChecksummerOptions(csum_iterations=i), num_interfaces=1, frame_len_hint=1500)
           for i in (1, 2)]
    stream = torch.cuda.current_stream(dev)
    for i in range(3):
        v = css[i & 1].process_batch(lu, ld)
    barrier(world)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    reps = 10
    for i in range(reps):
        v = css[(i + 1) & 1].process_batch(lu, ld)
    e1.record(stream)
    barrier(world)
    step_s = allreduce_max(e0.elapsed_time(e1) / reps / 1e3, world)
    dl = ld.cpu().numpy().view(frames.DESC_DTYPE).reshape(-1)
    vh = v.cpu().numpy()
    rfc = None if args.no_verify else rfc_verify(lu, ld, n_local, world)   # the last pass was -i 1
    moved = (b1 - b0 + 16 * n_local) if rank != 0 else 0
    fp = check_fingerprint(lu, ld, b0)
    tot = allreduce_sum_i64([n_local, int(dl["len"].astype(np.int64).sum()), moved,
                             int((vh == -1).sum()), int((vh >= 0).sum())] + fp, world)
    if rank == 0 and tot[0] != n_total:
        raise RuntimeError(f"root scatter: {tot[0]} frames arrived of {n_total}")
    single = None
    if rank == 0:
        ru, rd = ref
        rv = css[0].process_batch(ru, rd).cpu().numpy()
        rfp = check_fingerprint(ru, rd, 0)
        sharded = {"checks_sum": tot[5], "checks_weighted": tot[6], "drop": tot[3], "forward": tot[4]}
        whole = {"checks_sum": rfp[0], "checks_weighted": rfp[1],
                 "drop": int((rv == -1).sum()), "forward": int((rv >= 0).sum())}
        single = {"match": sharded == whole, "sharded": sharded, "single_gpu": whole,
                  "fingerprint": "sum of every frame's written check, and the same weighted by its "
                                 "global UMEM offset mod 65521 + 1; verdict counts"}
        del ref, ru, rd
    return {"frames_total": tot[0], "frame_bytes_total": tot[1], "bytes_moved": tot[2],
            "scatter_ms": round(t_move * 1e3, 3),
            "scatter_GBps": round(tot[2] / t_move / 1e9, 1) if t_move > 0 else None,
            "checksum_step_us_max": round(step_s * 1e6, 2),
            "gbs_checksummed": round(tot[1] / step_s / 1e9, 1),
            "verdicts": {"drop": tot[3], "forward": tot[4]},
            "rfc_check": rfc,
            "vs_single_gpu": single,
            "layout": "IMIX 64/570/1500 (7:4:1) packed, unaligned-mode descriptors; shards by bytes"}


def c_host_multi_leg(args, dev, reps=10):
    """BASELINE config 4 through the C host's multi-device calls (include/xsknf_gpu.h
    xsknf_gpu_multi_*, xsknf_amd/csrc/multi.hip) in THIS one process, over every
    visible device (XSKNF_BENCH_MULTI_DEVICES caps it): the global IMIX batch in
    device 0's HBM, split by bytes, every shard moved by grouped RCCL ncclSend /
    ncclRecv (device 0's own shard as a send to itself), checksummed on every
    device at once, the counters summed by ncclAllReduce and held against one
    device's pass over the whole batch.  At world 1 only (the ranks of
    `--gpus N` are the one-process-per-GPU path); on a one-GPU box it runs at
    N = 1."""
    from xsknf_amd import multi
    ndev = torch.cuda.device_count()
    if os.environ.get("XSKNF_BENCH_MULTI_DEVICES"):
        ndev = max(1, min(ndev, int(os.environ["XSKNF_BENCH_MULTI_DEVICES"])))
    n = args.config4_frames
    umem, dt, lens = frames.device_batch(n, "imix", layout="aligned", chunk=frames.CHUNK, seed=frames.SEED,
                                         device=dev)
    hd = dt.cpu().numpy().view(frames.DESC_DTYPE).reshape(-1).copy()
    mean = int(lens.mean())
    total = int(lens.astype(np.int64).sum())
    opts = [ChecksummerOptions(csum_iterations=i) for i in (1, 2)]
    pristine = umem.clone()          # for one device's pass over the whole batch, the reference answer
    with multi.MultiDevice(range(ndev)) as m:
        scat = [m.scatter(0, umem.data_ptr(), umem.numel(), hd) for _ in range(3)]
        moved = sum(m.shard_info(k)["span_hi"] - m.shard_info(k)["span_lo"] + 16 * (m.shard_info(k)["frame_hi"] -
                    m.shard_info(k)["frame_lo"]) for k in range(ndev))
        for i in range(3):
            m.process(opts[i & 1], frame_len_max=1500, frame_len_mean=mean)
        steps = [m.process(opts[(i + 1) & 1], frame_len_max=1500, frame_len_mean=mean) for i in range(reps)]
        m.process(opts[0], frame_len_max=1500, frame_len_mean=mean)   # the last pass -i 1
        cnt = m.counters()
        infos = [m.shard_info(k) for k in range(ndev)]
        # out and back: the frames packed on the root (their bytes only), every
        # device's records-only pass, the records applied to the root's UMEM
        # (xsknf_gpu_multi_scatter_packed / _return); -i 1, so the root's UMEM
        # and verdicts must equal one device's -i 1 pass over the whole batch
        pk = [m.scatter_packed(0, umem.data_ptr(), umem.numel(), hd) for _ in range(3)]
        pk_moved = sum(m.shard_info(k)["span_hi"] - m.shard_info(k)["span_lo"] for k in range(ndev)) + 16 * n
        vret = torch.empty(n, dtype=torch.int32, device=dev)
        rets = [m.return_results(umem.data_ptr(), vret.data_ptr(), opts[0], frame_len_max=1500, frame_len_mean=mean)
                for _ in range(3)]
        # the hot path in place on the packed shards (after the return: a shard
        # whose checks a pass wrote would send no records for them)
        for i in range(3):
            m.process(opts[i & 1], frame_len_max=1500, frame_len_mean=mean)
        psteps = [m.process(opts[(i + 1) & 1], frame_len_max=1500, frame_len_mean=mean) for i in range(reps)]
    # one device's pass over the whole batch, -i 1, and its counters on the device
    v = Checksummer(ChecksummerOptions(), num_interfaces=1, frame_len_hint=1500, frame_len_mean=mean).process_batch(
        pristine, dt)
    fp = check_fingerprint(pristine, dt, 0)
    single = {"frames": n, "bytes": total, "drop": int((v == -1).sum()), "forward": int((v >= 0).sum()),
              "checks_sum": fp[0], "checks_weighted": fp[1]}
    round_trip_match = bool(torch.equal(umem, pristine)) and bool(torch.equal(vret, v))
    t_pk = sorted(pk)[1]
    t_ret = sorted(r[1] for r in rets)[1]
    pass_us = [round(sorted(r[0][k] for r in rets)[1] * 1e3, 2) for k in range(ndev)]
    packed = {"scatter_ms": round(t_pk * 1e3, 3), "scatter_bytes": pk_moved,
              "scatter_GBps": round(pk_moved / t_pk / 1e9, 1),
              "return_ms": round(t_ret * 1e3, 3), "return_bytes": 4 * n,
              "records_pass_us_per_device": pass_us,
              "round_trip_ms": round((t_pk + t_ret) * 1e3, 3),
              "step_us_on_packed_shards": round(sorted(max(st) for st in psteps)[len(psteps) // 2] * 1e3, 2),
              "match": round_trip_match,
              "what": "frames packed into 16-byte slots on device 0 (its own shard straight into its shard buffer, "
                      "the others' sent by grouped ncclSend / ncclRecv; scatter_bytes: every shard's packed bytes); "
                      "each device's records-only pass; 4 B per frame back; the checks applied to device 0's UMEM -- "
                      "match: device 0's UMEM and verdicts equal one device's pass over the whole batch, every "
                      "byte (medians of 3)"}
    del umem, dt, v, pristine, vret
    per_dev = [sorted(st[k] for st in steps)[len(steps) // 2] for k in range(ndev)]
    step_max = sorted(max(st) for st in steps)[len(steps) // 2]
    t_scat = sorted(scat)[1]
    return {"devices": ndev, "frames": n, "frame_bytes": total,
            "shards": [{"device": x["device"], "frames": [x["frame_lo"], x["frame_hi"]],
                        "bytes": x["frame_bytes"]} for x in infos],
            "scatter_ms": round(t_scat * 1e3, 3), "scatter_bytes": moved,
            "scatter_GBps": round(moved / t_scat / 1e9, 1),
            "step_us_per_device": [round(t * 1e3, 2) for t in per_dev],
            "step_us": round(step_max * 1e3, 2),
            "gbs_checksummed": round(total / (step_max / 1e3) / 1e9, 1),
            "mpps": round(n / (step_max / 1e3) / 1e6, 1),
            "counters": cnt, "single_gpu": single, "match": cnt == single, "packed_round_trip": packed,
            "api": "xsknf_gpu_multi_create (ncclCommInitAll) / _scatter (grouped ncclSend / ncclRecv from device "
                   "0) / _process (a stream per device) / _counters (ncclAllReduce); medians of "
                   f"{reps} steps, each the slowest device's HIP-event time"}


def bounded_leg(fn, seconds, line):
    """Run one optional leg with a watchdog: its result, {"error": ...} if it
    raised, and if it has not returned after `seconds` the bench line is printed
    with {"error": "timed out"} in its place and the process exits 0 (the
    primary's figures stand; the exit ends whatever the leg left on the GPU)."""
    done = threading.Event()
    # what the leg's libraries print to stdout (RCCL's version banner at
    # communicator init) goes to stderr: stdout carries the one JSON line
    sys.stdout.flush()
    saved, py_stdout = os.dup(1), sys.stdout
    os.dup2(2, 1)
    sys.stdout = sys.stderr

    def watchdog():
        if not done.wait(seconds):
            os.dup2(saved, 1)
            line["c_host_multi"] = {"error": f"timed out after {seconds} s (the line was printed by the watchdog)"}
            py_stdout.write(json.dumps(line) + "\n")
            py_stdout.flush()
            os._exit(0)

    threading.Thread(target=watchdog, daemon=True).start()
    try:
        return fn()
    except Exception as e:   # reported in the line; the primary's figures stand
        return {"error": f"{type(e).__name__}: {e}"}
    finally:
        done.set()
        sys.stdout = py_stdout
        os.dup2(saved, 1)
        os.close(saved)


def check_fingerprint(umem, descs, base):
    """[sum of the written checks, the same weighted by (global offset mod 65521) + 1]
    over the well-formed-length frames of one batch (device tensors; `base` =
    the batch's offset in the global UMEM), so that a sharded run can be held
    against the single-GPU run of the whole batch."""
    d = descs.view(torch.int64).reshape(-1, 2)
    addr = d[:, 0]
    off = (addr & ((1 << 48) - 1)) + (addr >> 48)
    ok = (d[:, 1] & 0xFFFFFFFF) >= 42
    off = off[ok]
    c = umem[off + 40].to(torch.int64) | (umem[off + 41].to(torch.int64) << 8)
    w = (off + base) % 65521 + 1
    return [int(c.sum()), int((c * w).sum())]


def rfc_verify(umem, descs, n, world):
    """Every well-formed frame's written check passes the RFC 768 / 1071
    receive-side verification (tests/rfc1071.py, written from the RFC, no
    restatement of the checksummer): V = 0xFFFF, or 0x0001 where the reference's
    single fold (checksummer_user.c:105-106) drops a carry.  A size-independent
    property of the full batch after its last -i 1 pass; all-reduced over the
    ranks: [frames checked, violations, carry-loss frames]."""
    from tests import rfc1071
    d = descs[:n].cpu().numpy().view(frames.DESC_DTYPE).reshape(-1)
    offs = ((d["addr"] & np.uint64((1 << 48) - 1)) + (d["addr"] >> np.uint64(48))).astype(np.int64)
    idx, V = rfc1071.verify(umem, offs, d["len"].astype(np.int64))
    c = allreduce_sum_i64([int(idx.size), int(((V != 0xFFFF) & (V != 0x0001)).sum()), int((V == 0x0001).sum())],
                          world)
    return {"frames_checked": c[0], "violations": c[1], "carry_loss_frames": c[2],
            "property": "RFC 768/1071 receive-side sum of every well-formed frame = 0xFFFF (0x0001 where the "
                        "single fold drops a carry), after the workload's last -i 1 pass"}


# ---- CPU baseline, probes, traffic -----------------------------------------------

def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_list(cpus) -> str:
    """A CPU set as ranges ("0-15,32")."""
    out, run = [], []
    for c in sorted(cpus):
        if run and c == run[-1] + 1:
            run.append(c)
            continue
        if run:
            out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
        run = [c]
    if run:
        out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
    return ",".join(out)


def cpu_baseline(res, budget_s, threads, check=True, windows=3):
    """The reference's own xsknf_packet_processor() (oracle/_ref: its verbatim
    text compiled gcc -O2 -flto, kind "reference") -- or, where that library was
    not built, the C restatement (kind "port") -- timed on host cores in a
    process_batch_1if-shaped loop over a bounded sample of the same workload;
    also checks the GPU result on that sample.

    `windows` timed windows of budget_s / windows each; `value` is their
    median, `spread` their min / max.  One thread is pinned to the LAST CPU of
    the process's affinity mask (the reference's tests pin the NF to one core,
    tests/test-drop-cpu.py:79; the first CPU of the mask is where the HIP
    runtime's threads of this process tend to run); several threads take the
    mask's last `threads` CPUs."""
    from oracle import csum_oracle as O
    from oracle import ref as R

    kind = "reference" if R.available() else "port"
    timer = R.time_batch if kind == "reference" else O.c_time_batch
    process = R.process_batch if kind == "reference" else O.c_process_batch
    umem_host, descs_host, k = res["sample"]
    lens = descs_host["len"].astype(np.int64)
    work = umem_host.copy()
    t1, v = timer(work, descs_host, threads=threads, reps=1, pin="last")
    reps = max(1, int(budget_s / windows / max(t1, 1e-6)))
    rates, secs = [], 0.0
    for _ in range(max(1, windows)):
        t, v = timer(work, descs_host, threads=threads, reps=reps, pin="last")
        rates.append(lens.sum() * reps / t / 1e9)
        secs += t
    gbs = float(np.median(rates))
    # checker: GPU output on the sample frames == the CPU path's output (single
    # pass; reprocessing is idempotent because the check is cleared before summing)
    match = None
    if check:
        process(umem_host, descs_host)
        hi = umem_host.shape[0]
        g_umem = res["umem"][:hi].cpu().numpy()
        g_v = res["verdicts"][:k].cpu().numpy()
        match = bool(np.array_equal(g_v, v) and np.array_equal(g_umem, umem_host))
    mask = sorted(os.sched_getaffinity(0))
    used = mask[-threads:] if threads <= len(mask) else mask
    frames_per_gb = k / lens.sum()
    return {"value": round(gbs, 4), "unit": "GB/s checksummed", "cores": threads,
            "spread": {"min": round(float(min(rates)), 4), "max": round(float(max(rates)), 4),
                       "windows": len(rates), "statistic": "median of the windows"},
            "kind": kind, "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "affinity_mask": _cpu_list(mask), "pinned_to": _cpu_list(used),
            "mpps": round(gbs * frames_per_gb * 1e3, 4),
            "sample": f"{k} frames of the same workload ({lens.sum() / 1e6:.1f} MB) x {reps} passes per window, "
                      f"{len(rates)} windows, {secs:.1f} s, process_batch_1if-shaped loop (batch 64), "
                      + ("1 core pinned to the last CPU of the mask" if threads == 1 else
                         f"{threads} threads on {threads} of the box's {len(mask)}-CPU share"),
            "gpu_matches_oracle_on_sample": match,
            "code": "oracle/_ref/libcsum_ref.so: reference checksummer_user.c:30-112 verbatim, gcc -O2 -flto"
                    if kind == "reference" else "oracle/csum_oracle.c (restatement), gcc -O2 -flto"}


def probes_for(res, reps=20):
    """bare memory patterns measured beside the kernels, on the
    batch just measured (all K rotated batches at once, so the probes read cold
    bytes too; tools/hbm_probe.hip in library form, built by `make tools`):
      * read: the fastest bare read of the same frame bytes -- the chunk-stride /
        packed-span shapes for uniform batches, and for any batch the
        descriptor-driven shape (each frame's 16-B chunks from its descriptor,
        64-frame tiles per wave, lanes round robin over the tile's chunks);
      * step floor: the step's whole memory pattern with no arithmetic -- every
        frame's bytes read, every check's 64-B sector rewritten (unchanged) in
        the stream or deferred to each wave's end, whichever is faster, and a
        4-byte verdict written per frame.
    Ratios are probe time / kernel time: < 1 means the kernel is slower than
    the bare pattern, > 1 that the kernel's own access pattern beats the probe
    (it does at 1500 B, so there the probe is a reference, not a ceiling)."""
    import ctypes
    path = os.path.join(ROOT, "tools", "build", "libhbm_probe.so")
    if not os.path.exists(path):
        return None
    lens = res["lens"]
    K = res["K"]
    n_all = res["n"] * K
    umem = res["umem"]
    try:
        lib = ctypes.CDLL(path)
        lib.hbm_probe_read_us.restype = ctypes.c_double
        lib.hbm_probe_read_us.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                          ctypes.c_uint64, ctypes.c_int]
        lib.hbm_probe_desc_us.restype = ctypes.c_double
        lib.hbm_probe_desc_us.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_uint32]
    except (OSError, AttributeError):
        return None
    torch.cuda.synchronize()
    shapes = {}
    # (the chunk-stride and span shapes read everything in one launch: only for
    # unrotated batches, where that is one batch per launch as the kernels run)
    if K > 1:
        pass
    elif res["layout"] == "aligned" and int(lens.min()) == int(lens.max()):
        shapes["chunk_stride"] = lib.hbm_probe_read_us(ctypes.c_void_p(umem.data_ptr()), n_all,
                                                       res["chunk"] or frames.CHUNK, frames.HEADROOM,
                                                       int(lens[0]), reps)
    elif res["layout"] != "aligned":
        shapes["packed_span"] = lib.hbm_probe_read_us(ctypes.c_void_p(umem.data_ptr()), 1, 0, 0,
                                                      umem.numel() // 16 * 16, reps)
    dargs = (ctypes.c_void_p(umem.data_ptr()), umem.numel(), ctypes.c_void_p(res["descs"].data_ptr()), n_all)
    # one launch per batch of at most 1M frames, as the kernels run (launch gaps and ramps included)
    per = min(res["n"], 1 << 20)
    shapes["descriptors"] = lib.hbm_probe_desc_us(*dargs, 0, reps, per)
    shapes = {k: v / K for k, v in shapes.items() if v > 0}
    if not shapes:
        return None
    best = min(shapes, key=shapes.get)
    us = shapes[best]
    # the step writes a 4-byte verdict per frame as well (modes 3 / 4); 1 / 2 without it, for reference
    floors = {k: lib.hbm_probe_desc_us(*dargs, m, reps, per) / K
              for k, m in (("in_stream", 3), ("deferred", 4), ("in_stream_no_verdicts", 1),
                           ("deferred_no_verdicts", 2))}
    floors = {k: v for k, v in floors.items() if v > 0}
    out = {"read_us": round(us, 2), "read_frame_GBps": round(res["bytes_len"] / us / 1e3, 1),
           "read_shape": best, "read_shapes_us": {k: round(v, 2) for k, v in shapes.items()},
           "probe": "tools/hbm_probe.hip: fastest read shape over the same frame bytes, nothing written"}
    if floors:
        fb = min((k for k in floors if "no_verdicts" not in k), key=floors.get, default=min(floors, key=floors.get))
        out["step_floor_us"] = round(floors[fb], 2)
        out["step_floor_shape"] = fb
        out["step_floor_shapes_us"] = {k: round(v, 2) for k, v in floors.items()}
        out["step_vs_floor_probe"] = round(floors[fb] / (res["step_ms"] * 1e3), 4)
    k_ms = res["sum_ms"] if res["sum_ms"] is not None else None
    if k_ms:
        out["summing_kernel_vs_read_probe"] = round(us / (k_ms * 1e3), 4)
    return out


def traffic_for(name):
    """HBM bytes of one step (every kernel of every launch of it) from the
    committed rocprofv3 PMC passes (tools/traffic.py ->
    profiles/traffic_<workload>.json), or None."""
    p = os.path.join(ROOT, "profiles", f"traffic_{name}.json")
    if os.path.exists(p):
        try:
            t = json.load(open(p))
        except (OSError, ValueError):
            return None
        return t.get("hbm_bytes_per_step", t.get("hbm_bytes_per_launch"))
    return None


def step_summary(r, steps):
    total_frames, total_bytes = r["counters"][0], r["counters"][1]
    t = r["step_ms_max"] / 1e3
    alg = total_bytes + total_frames * (DESC_BYTES + VERDICT_BYTES + CHECK_BYTES)
    out = {"frames": total_frames, "mpps": round(total_frames / t / 1e6, 2),
           "gbs_checksummed": round(total_bytes / t / 1e9, 2), "step_us": round(r["step_ms_max"] * 1e3, 2),
           "step_frac": round(alg / t / 1e9 / HBM_PEAK_GBS / max(1, r.get("world", 1)), 4),
           "wall_ms_per_step": round(r["wall_max"] / steps * 1e3, 4), "rotated_batches": r["K"]}
    if r["span"] is not None:
        out["rank0_shard"] = list(r["span"])
    out["summing_kernel_alone_us"] = round(r["sum_ms"] * 1e3, 2) if r["sum_ms"] is not None else None
    out["probes"] = r.get("probes")
    out["kernel"] = f"{r['family']} ({r['stores']})"
    out["launch_shape"] = r["shape"]
    out["traffic"] = traffic_for(r["name"])
    if r.get("rfc") is not None:
        out["rfc_check"] = r["rfc"]
    return out


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    world, rank, dev, rehearsal = dist_setup(args)
    torch.cuda.set_device(dev)
    seed = frames.SEED + rank
    prim = time_workload(args.workload, args, world, rank, dev, seed, primary=True)
    sec = {}
    for name in [s for s in args.secondary.split(",") if s and s != args.workload]:
        r = time_workload(name, args, world, rank, dev, seed, primary=False)
        r["world"] = world
        if world == 1 and not args.no_probes and name not in NIC:   # same bytes as the base workload
            r["probes"] = probes_for(r)
        sec[name] = step_summary(r, args.steps)
        del r
        # A workload's freed buffers stay in torch's cache for the next one: a
        # batch allocated from the driver again after a 27 GB free (the 64 B
        # workload's 13 rotated batches) streams slower than the same batch in
        # memory allocated first -- jumbo 1474 vs 1452-1456 us, config 4 910 vs
        # 887, IMIX 113.5 vs 110.8; the 13M-frame 64 B batch the other way, 640
        # vs 659 (profiles/r05/ab/ab_bench_alloc_*.jsonl): every workload runs
        # on first-allocated memory, as an NF's UMEM, allocated once at start.  (XSKNF_BENCH_EMPTY_CACHE=1: the
        # round-4 behaviour, for A/B.)
        if os.environ.get("XSKNF_BENCH_EMPTY_CACHE"):
            torch.cuda.empty_cache()

    root_scatter = root_scatter_leg(args, world, rank, dev) if (_DIST and not args.no_root_scatter) else None
    # what the collectives saw: every rank contributes 1 (so a SCALE line shows
    # that the backend really had N ranks), and the frames summed over ranks
    dist_info = None
    if _DIST:
        seen = allreduce_sum_i64([1], world)[0]
        pr = prim["per_rank"]
        steps_us = [round(r[0] * 1e3, 2) for r in pr]
        walls_ms = [round(r[1], 4) for r in pr]
        rates = [r[2] / (r[0] / 1e3) / 1e9 for r in pr]          # each rank's GB/s on its own step
        dist_info = {"ranks_seen": seen, "backend": str(dist.get_backend()), "world_size": dist.get_world_size(),
                     "frames_allreduced": prim["counters"][0],
                     "per_rank": {"step_us": steps_us, "wall_ms_per_step": walls_ms,
                                  "gbs_checksummed": [round(x, 1) for x in rates],
                                  "frames": [int(r[3]) for r in pr]},
                     "step_us_min": min(steps_us), "step_us_max": max(steps_us),
                     "step_spread": round(max(steps_us) / min(steps_us), 4) if min(steps_us) > 0 else None,
                     # the rate one rank reaches alone (its N = 1 equivalent), and the sum of the
                     # ranks' own rates: value / that sum < 1 is what the max-over-ranks clock cost
                     "per_rank_gbs_mean": round(sum(rates) / len(rates), 1),
                     "sum_of_rank_rates_gbs": round(sum(rates), 1),
                     "collective_device": coll_device(),
                     "collectives": "barrier + max-time and counter all-reduces after the timed region; "
                                    "root_scatter: broadcast + point-to-point isend/irecv"}

    total_frames, total_bytes, n_drop, n_fwd = prim["counters"]
    step_s = prim["wall_max"] / args.steps          # wall clock, max over ranks: `value`
    value = total_bytes / step_s / 1e9
    mpps = total_frames / step_s / 1e6
    # roofline: the whole step on this rank -- every frame byte,
    # its 16 B descriptor read, its 4 B verdict and 2 B check writes -- over the
    # step's HIP-event time on the launch stream (both kernels of the step)
    step_k_s = prim["step_ms"] / 1e3
    step_alg = prim["bytes_len"] + prim["n"] * (DESC_BYTES + VERDICT_BYTES + CHECK_BYTES)
    achieved = step_alg / step_k_s / 1e9
    kernel_alone = None
    if prim["sum_ms"] is not None:
        alg_k = prim["bytes_len"] + prim["n"] * (DESC_BYTES + VERDICT_BYTES)
        kernel_alone = {"kernel": f"{prim['family']} (records only, launched alone, back to back)",
                        "us": round(prim["sum_ms"] * 1e3, 2), "alg_bytes": alg_k,
                        "achieved": round(alg_k / (prim["sum_ms"] / 1e3) / 1e9, 1),
                        "frac": round(alg_k / (prim["sum_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
    # the same bytes over `value`'s clock (wall time around the K steps, max over ranks, per rank)
    achieved_wall = step_alg / step_s / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic_for(args.workload),
            "basis": "frac / achieved: whole step (SURVEY.md 8(d)), sum(len + 22) per batch on rank 0 / the "
                     "step's HIP-event time on the launch stream (the kernels' own time); frac_wall / "
                     "achieved_wall: the same bytes over value's time base (wall clock around the timed steps, "
                     "max over ranks); traffic = FETCH_SIZE/WRITE_SIZE of every kernel of one step",
            "achieved_wall": round(achieved_wall, 1), "frac_wall": round(achieved_wall / HBM_PEAK_GBS, 4),
            "kernels": f"{prim['family']} ({prim['stores']})", "launch_shape": prim["shape"],
            "alg_bytes_per_step": step_alg, "step_us": round(step_k_s * 1e6, 2),
            "summing_kernel_alone": kernel_alone,
            "probes": None if args.no_probes else probes_for(prim)}
    cpu = None
    if rank == 0 and prim["sample"] is not None:
        cpu = cpu_baseline(prim, args.cpu_seconds, args.cpu_threads)
        n_all = args.cpu_all_cores
        if n_all < 0:
            n_all = min(16, len(os.sched_getaffinity(0)))
        if n_all > 1:
            allc = cpu_baseline(prim, args.cpu_seconds / 2, n_all, check=False)
            cpu["all_cores"] = {k: allc[k] for k in ("value", "unit", "cores", "mpps", "spread", "pinned_to",
                                                     "sample")}
    if rank == 0:
        length, layout, chunk, desc = WORKLOADS[args.workload]
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "GB/s checksummed",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "min_warmup_s": args.min_warmup_s,
            "primary_warmup_s": args.primary_warmup_s,
            "ms_per_step": round(step_s * 1e3, 4), "kernel_steps": args.kernel_steps,
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u16 words summed in u32", "data": "synthetic",
            "mpps": round(mpps, 2),
            "config": {"workload": desc, "frames_per_gpu": prim["n"], "frame_len": length,
                       "layout": layout, "global_batch": total_frames, "rotated_batches": prim["K"],
                       "parallelism": f"shard{world} (independent frames, no exchange)"},
            "roofline": roof, "cpu_baseline": cpu, "secondary": sec,
            "verdicts": {"drop": n_drop, "forward": n_fwd},
            "rfc_check": prim["rfc"],
        }
        if rehearsal:
            out["config"]["rehearsal"] = rehearsal
        if root_scatter is not None:
            out["root_scatter"] = root_scatter
        if dist_info is not None:
            out["dist"] = dist_info
        if world == 1 and not args.no_c_host_multi:
            # last, and bounded: on a node of several GPUs this is one process
            # driving all of them over RCCL; a hang there must not cost the line
            out["c_host_multi"] = bounded_leg(lambda: c_host_multi_leg(args, dev), args.c_host_multi_timeout, out)
        print(json.dumps(out), flush=True)
    if _DIST:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
