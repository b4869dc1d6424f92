"""The AF_XDP runtime (include/xsknf.h, libxsknf.so) on CPU.

The NF here is the reference per-frame path (the oracle's
xsknf_packet_processor-shaped callback), so these tests check the runtime's
datapath -- rx batches, verdict routing, fill / tx / completion recycling,
multi-interface forwarding and cross-UMEM copies (src/xsknf.c:409-742) --
against the oracle applied frame by frame.  Emulated queues ("emu<k>") play
the kernel's part; tests/test_gpu_runtime.py runs the same loop with the GPU
hook, and test_veth_config1 runs real AF_XDP sockets over a veth pair.
"""
import ctypes
import errno
import os
import subprocess
import sys
import time

import numpy as np
import pytest

from oracle import csum_oracle as O
from xsknf_amd import runtime as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import config1  # noqa: E402


def test_header_matches_binding_and_exports():
    from test_capi import declared_functions
    declared = set(declared_functions("xsknf.h", "XSKNF_API"))
    assert declared == set(R.EXPORTED_SYMBOLS)
    out = subprocess.run(["nm", "-D", "--defined-only", R.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert exported == declared          # nothing else leaks out of the library


def test_struct_layouts_match_the_header(tmp_path):
    """ctypes mirrors == what the C compiler lays out for include/xsknf.h (the
    reference's src/xsknf.h:25-59 member order; 13 counters, statistics.c:8)."""
    src = tmp_path / "layout.c"
    fields = [f for f, _ in R.Config._fields_]
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "xsknf.h"\nint main(void){\n'
                   'printf("%zu %zu\\n", sizeof(struct xsknf_config), sizeof(struct xsknf_socket_stats));\n'
                   + "".join(f'printf("%zu\\n", offsetof(struct xsknf_config, {f}));\n' for f in fields)
                   + "return 0;}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert int(out[0]) == ctypes.sizeof(R.Config)
    assert int(out[1]) == ctypes.sizeof(R.SocketStats) == 13 * 8
    assert [int(x) for x in out[2:]] == [getattr(R.Config, f).offset for f in fields]


def nf_oracle(iterations=1, action=O.REDIRECT, nif=1):
    lib = O.load()
    lib.oracle_nf_set_options.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32]
    lib.oracle_nf_set_options(iterations, action, nif)
    return ctypes.cast(lib.oracle_nf_packet_processor, ctypes.c_void_p).value


def expected(frames, ingress=0, iterations=1, action=O.REDIRECT, nif=1):
    """Oracle verdict and rewritten bytes of every frame."""
    out = []
    for f in frames:
        b = bytearray(f)
        v = O.c_packet_processor(b, ingress, iters=iterations, action=action, nif=nif)
        out.append((v, bytes(b)))
    return out


def pump(rt, plan, n_if=1, timeout=30.0):
    """Emulated kernel: deliver plan[iface] frames on each iface, collect every tx.

    Returns {iface: [frames transmitted on it]} once the workers have received
    everything and nothing more comes out."""
    sent = {i: 0 for i in range(n_if)}
    got = {i: [] for i in range(n_if)}
    total = sum(len(v) for v in plan.values())
    t_end = time.time() + timeout
    quiet_since = None
    while time.time() < t_end:
        progress = False
        for i, frames in plan.items():
            if sent[i] < len(frames):
                k = rt.deliver(frames[sent[i]:sent[i] + 512], iface=i)
                sent[i] += k
                progress |= k > 0
        for i in range(n_if):
            out = rt.transmit(iface=i)
            got[i].extend(out)
            progress |= bool(out)
        assert rt.worker_error() == 0
        rx = sum(rt.stats(0, i)["rx_npkts"] for i in range(n_if))
        if all(sent[i] == len(plan[i]) for i in plan) and rx == total:
            if progress:
                quiet_since = None
            elif quiet_since is None:
                quiet_since = time.time()
            elif time.time() - quiet_since > 0.2:
                return got
        time.sleep(0.0005)
    raise AssertionError(f"timeout: sent {sent}, rx {rx}/{total}")


@pytest.fixture
def frames():
    return config1.frames_check(6000)


def test_redirect_round_trip_matches_oracle(frames):
    with R.Runtime(R.make_config(["emu0"])) as rt:
        rt.set_packet_processor(nf_oracle())
        rt.start()
        got = pump(rt, {0: frames})[0]
        st = rt.stats()
    want = [b for v, b in expected(frames) if v != -1]
    assert len(got) == len(want)
    assert got == want                      # byte exact, in order
    assert st["rx_npkts"] == len(frames)    # > 4096: frames were recycled
    assert st["tx_npkts"] <= len(want)


def test_drop_recycles_every_frame(frames):
    n = 3 * R.FRAMES_PER_SOCKET + 17
    fr = (frames * 3)[:n]
    with R.Runtime(R.make_config(["emu0"])) as rt:
        rt.set_packet_processor(nf_oracle(action=O.DROP))
        rt.start()
        got = pump(rt, {0: fr})[0]
        st = rt.stats()
    # DROP: -1 for every IPv4/UDP frame; non-IPv4 / non-UDP still return 0 (tx)
    want = [b for v, b in expected(fr, action=O.DROP) if v != -1]
    assert got == want
    assert st["rx_npkts"] == n


@pytest.mark.parametrize("bind", [(0, 0), (R.XDP_COPY, R.XDP_ZEROCOPY)], ids=["shared-umem", "two-umems"])
def test_two_interfaces_forward_to_the_next(frames, bind):
    f0, f1 = frames[:2500], frames[2500:5000]
    cfg = R.make_config(["emu0", "emu1"], bind=list(bind))
    with R.Runtime(cfg) as rt:
        rt.set_packet_processor(nf_oracle(nif=2))
        rt.start()
        got = pump(rt, {0: f0, 1: f1}, n_if=2)
        b0, b1 = rt.umem(0, 0)[0], rt.umem(0, 1)[0]
    assert (b0 == b1) == (bind == (0, 0))
    # verdict (ingress + 1) % 2: emu0's frames leave on emu1 and vice versa;
    # non-IPv4 / non-UDP frames return 0 -> leave on emu0
    e0, e1 = expected(f0, 0, nif=2), expected(f1, 1, nif=2)
    out0 = [b for v, b in e0 if v == 0] + [b for v, b in e1 if v == 0]
    out1 = [b for v, b in e0 if v == 1] + [b for v, b in e1 if v == 1]
    assert sorted(got[0]) == sorted(out0)
    assert sorted(got[1]) == sorted(out1)


def test_unaligned_chunks(frames):
    cfg = R.make_config(["emu0"], unaligned=True, frame_size=3000)   # not a power of two
    with R.Runtime(cfg) as rt:
        rt.set_packet_processor(nf_oracle(iterations=3))
        rt.start()
        got = pump(rt, {0: frames[:5000]})[0]
    assert got == [b for v, b in expected(frames[:5000], iterations=3) if v != -1]


@pytest.mark.parametrize("batch", [1, 255, 256, 2048])
def test_batch_sizes(frames, batch):
    with R.Runtime(R.make_config(["emu0"], batch_size=batch)) as rt:
        rt.set_packet_processor(nf_oracle())
        rt.start()
        got = pump(rt, {0: frames[:5000]})[0]
    assert got == [b for v, b in expected(frames[:5000]) if v != -1]


def test_poll_mode_on_emulated_queues(frames):
    with R.Runtime(R.make_config(["emu0"], poll=True)) as rt:
        rt.set_packet_processor(nf_oracle())
        rt.start()
        got = pump(rt, {0: frames[:1000]})[0]
        assert rt.stats()["opt_polls"] > 0
    assert got == [b for v, b in expected(frames[:1000]) if v != -1]


def nf_oracle_async(iterations=1, action=O.REDIRECT, nif=1):
    """The oracle as a two-phase hook: submit records, complete computes (oracle/csum_oracle.c)."""
    lib = O.load()
    nf_oracle(iterations, action, nif)
    lib.oracle_nf_async_reset()
    return (ctypes.cast(lib.oracle_nf_batch_submit, ctypes.c_void_p).value,
            ctypes.cast(lib.oracle_nf_batch_complete, ctypes.c_void_p).value)


def async_stats(worker=0):
    lib = O.load()
    sub, ovl = ctypes.c_uint64(), ctypes.c_uint64()
    lib.oracle_nf_async_stats.argtypes = [ctypes.c_uint, ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.POINTER(ctypes.c_uint64)]
    lib.oracle_nf_async_stats(worker, ctypes.byref(sub), ctypes.byref(ovl))
    return sub.value, ovl.value


@pytest.mark.parametrize("batch,depth", [(1, 1), (64, 1), (2048, 1), (64, 3), (7, 4), (64, 8), (5, 8)])
def test_async_hook_round_trip(frames, batch, depth):
    """Two-phase hook: batch k is routed only after its complete, while batch k+1
    (.. k+depth) is in flight; output identical to the per-frame path, in order."""
    with R.Runtime(R.make_config(["emu0"], batch_size=batch)) as rt:
        rt.set_batch_processor_async(*nf_oracle_async(iterations=2))
        rt.set_batch_depth(depth)
        rt.start()
        got = pump(rt, {0: frames})[0]
        st = rt.stats()
    assert got == [b for v, b in expected(frames, iterations=2) if v != -1]
    assert st["rx_npkts"] == len(frames)
    submits, overlapped = async_stats()
    assert submits >= len(frames) // batch
    if batch <= 64:                           # pump delivers 512 at a time: several batches per delivery
        assert overlapped > 0                 # a batch was submitted while one was in flight


@pytest.mark.parametrize("bind", [(0, 0), (R.XDP_COPY, R.XDP_ZEROCOPY)], ids=["shared-umem", "two-umems"])
def test_async_hook_two_interfaces(frames, bind):
    f0, f1 = frames[:2500], frames[2500:5000]
    cfg = R.make_config(["emu0", "emu1"], bind=list(bind), batch_size=128)
    with R.Runtime(cfg) as rt:
        rt.set_batch_processor_async(*nf_oracle_async(nif=2))
        rt.start()
        got = pump(rt, {0: f0, 1: f1}, n_if=2)
    e0, e1 = expected(f0, 0, nif=2), expected(f1, 1, nif=2)
    assert sorted(got[0]) == sorted([b for v, b in e0 + e1 if v == 0])
    assert sorted(got[1]) == sorted([b for v, b in e0 + e1 if v == 1])


def test_async_hook_stop_and_restart_loses_no_frame(frames):
    """A stop completes the batch in flight; after a restart the socket still has
    its whole frame budget (more frames than a socket owns go through)."""
    first, second = frames[:1500], (frames * 2)[:3 * R.FRAMES_PER_SOCKET + 5]
    with R.Runtime(R.make_config(["emu0"], batch_size=256)) as rt:
        rt.set_batch_processor_async(*nf_oracle_async(action=O.DROP))
        rt.start()
        got1 = pump(rt, {0: first})[0]
        assert rt.stop() == 0
        rt.start()
        n0 = rt.stats()["rx_npkts"]
        sent, got2 = 0, []
        t_end = time.time() + 30
        while (sent < len(second) or rt.stats()["rx_npkts"] - n0 < len(second)) and time.time() < t_end:
            sent += rt.deliver(second[sent:sent + 512])
            got2.extend(rt.transmit())
            time.sleep(0.0005)
        time.sleep(0.2)
        got2.extend(rt.transmit())
        assert rt.worker_error() == 0
        assert rt.stats()["rx_npkts"] - n0 == len(second)
    assert got1 == [b for v, b in expected(first, action=O.DROP) if v != -1]
    assert got2 == [b for v, b in expected(second, action=O.DROP) if v != -1]


def test_init_and_start_errors():
    lib = R.load()
    assert lib.xsknf_set_batch_depth(0) == -errno.EINVAL
    assert lib.xsknf_set_batch_depth(9) == -errno.EINVAL
    assert lib.xsknf_set_batch_processor_async(ctypes.c_void_p(1), None, None) == -errno.EINVAL
    cfg = R.make_config(["emu0"])
    cfg.working_mode = R.MODE_XDP
    assert lib.xsknf_init(ctypes.byref(cfg), None) == -errno.EOPNOTSUPP
    assert lib.xsknf_init(ctypes.byref(R.make_config(["no-such-if0"])), None) == -errno.ENODEV
    assert lib.xsknf_init(ctypes.byref(R.make_config(["emu0"], frame_size=3000)), None) == -errno.EINVAL
    assert lib.xsknf_init(ctypes.byref(R.make_config(["emu0"], workers=0)), None) == -errno.EINVAL
    with R.Runtime(R.make_config(["emu0"])) as rt:
        # a second init while one is live
        assert lib.xsknf_init(ctypes.byref(R.make_config(["emu0"])), None) == -errno.EINVAL
        # no NF registered and none linked in
        assert lib.xsknf_start_workers() == -errno.ENOENT
        st = R.SocketStats()
        assert lib.xsknf_get_socket_stats(1, 0, ctypes.byref(st)) == -errno.EINVAL
        assert lib.xsknf_emu_deliver(0, 0, None, None, 1, 64) == -errno.EINVAL
        too_big = np.zeros(4096, dtype=np.uint8)
        ln = np.array([4096 - 255], dtype=np.uint32)         # > frame_size - headroom
        assert lib.xsknf_emu_deliver(0, 0, too_big.ctypes.data, ln.ctypes.data, 1, 4096) == -errno.EINVAL
    assert lib.xsknf_cleanup() == 0                        # idempotent


def _c_parse(argv):
    lib = R.load()
    libc = ctypes.CDLL(None)
    ctypes.c_int.in_dll(libc, "optind").value = 0        # fresh getopt scan
    args = [a.encode() for a in argv]
    arr = (ctypes.c_char_p * (len(args) + 1))(*args, None)
    cfg = R.Config()
    assert lib.xsknf_parse_args(len(args), arr, ctypes.byref(cfg)) == 0
    names = [cfg.interfaces[i].decode() for i in range(cfg.num_interfaces)]
    return cfg, names


@pytest.mark.parametrize("argv,want", [
    (["nf", "-i", "eth0"], dict(names=["eth0"], workers=1, batch=64, poll=0, busy=0, unaligned=0, fs=4096,
                                skb=False, bind=[""])),
    (["nf", "-i", "eth0:c", "-i", "eth1:z", "-S", "-b", "128", "-w", "2", "-p"],
     dict(names=["eth0", "eth1"], workers=2, batch=128, poll=1, busy=0, unaligned=0, fs=4096, skb=True,
          bind=["copy", "zerocopy"])),
    (["nf", "--iface=ens1f0", "--unaligned", "--frame-size=3000", "--busy-poll", "-M", "AF_XDP"],
     dict(names=["ens1f0"], workers=1, batch=64, poll=0, busy=1, unaligned=1, fs=3000, skb=False, bind=[""])),
    (["nf", "-i", "veth0", "-f", "2048", "--", "-c", "DROP", "-i", "5"],
     dict(names=["veth0"], workers=1, batch=64, poll=0, busy=0, unaligned=0, fs=2048, skb=False, bind=[""])),
])
def test_parse_args_defaults_and_options(argv, want):
    """src/xsknf.c:777-874 (defaults :46-52), and runtime.parse_args binding the same C parser."""
    bound, _ = R.parse_args(argv[1:], prog="nf")
    for cfg, names in (_c_parse(argv), (bound, [bound.interfaces[i].decode() for i in range(bound.num_interfaces)])):
        assert names == want["names"]
        assert cfg.workers == want["workers"] and cfg.batch_size == want["batch"]
        assert cfg.poll == want["poll"] and cfg.busy_poll == want["busy"]
        assert cfg.unaligned_chunks == want["unaligned"] and cfg.xsk_frame_size == want["fs"]
        assert bool(cfg.xdp_flags & R.XDP_FLAGS_SKB_MODE) == want["skb"]
        assert cfg.xdp_flags & R.XDP_FLAGS_DRV_MODE == (0 if want["skb"] else R.XDP_FLAGS_DRV_MODE)
        for i, mode in enumerate(want["bind"]):
            wantf = R.XDP_USE_NEED_WAKEUP | {"": 0, "copy": R.XDP_COPY, "zerocopy": R.XDP_ZEROCOPY}[mode]
            assert cfg.bind_flags[i] == wantf
        assert cfg.ebpf_filename == b"nf_kern.o" and cfg.xdp_progname == b"handle_xdp"


@pytest.mark.parametrize("argv", [["nf"], ["nf", "-i", "eth0:x"], ["nf", "-i", "e0", "-M", "FOO"],
                                  ["nf", "-i", "e0", "-w", "0"], ["nf", "-i", "e0", "-f", "3000"]])
def test_parse_args_errors_exit_like_the_reference(argv):
    code = ("import ctypes,sys; sys.path.insert(0, %r); from xsknf_amd import runtime as R; "
            "lib=R.load(); a=[x.encode() for x in %r]; arr=(ctypes.c_char_p*(len(a)+1))(*a, None); "
            "lib.xsknf_parse_args(len(a), arr, ctypes.byref(R.Config())); print('returned')") % (ROOT, argv)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 1 and "returned" not in p.stdout
    assert "xsknf library options" in p.stderr


def _veth_available():
    if os.geteuid() != 0 or not os.path.exists(config1.HARNESS):
        return False
    p = subprocess.run(["unshare", "-n", "true"], capture_output=True)
    return p.returncode == 0


@pytest.mark.skipif(not _veth_available(), reason="needs root, netns and tools/build/xsk_veth (make tools)")
def test_veth_config1_is_bit_exact():
    """Real AF_XDP sockets (skb mode, copy) over a veth pair in a private netns."""
    res = config1.check(iterations=2, n=1500)
    assert res["exit"] == 0, res
    assert res["worker_error"] == 0
    assert res["expected"] > 1300 and res["mismatches"] == 0, res


@pytest.mark.parametrize("extra", [("--two-phase",), ("--two-phase", "--poll"), ("--poll",)],
                         ids=["two-phase", "two-phase-poll", "poll"])
def test_veth_config1_hooks_and_poll(extra):
    """Real AF_XDP sockets: the two-phase hook keeps a batch in flight across worker
    passes, and with poll() a pass never blocks while one is out (the last batch
    still comes back)."""
    res = config1.check(iterations=1, n=1200, extra=extra)
    assert res["exit"] == 0, res
    assert res["worker_error"] == 0
    assert res["expected"] > 1000 and res["mismatches"] == 0, res
