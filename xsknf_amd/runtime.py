"""ctypes binding of the AF_XDP runtime, include/xsknf.h (xsknf_amd/lib/libxsknf.so).

The runtime mirrors the reference library (src/xsknf.c): workers, UMEM,
AF_XDP sockets, rx batches -> NF -> fill / tx rings.  The NF is either a
per-frame C callback (xsknf_packet_processor semantics) or a batch hook; the
GPU checksummer hook is ``libxsknf_gpu``'s ``xsknf_gpu_hook_process``
(:class:`GpuHook`).

Interfaces named ``emu<k>`` are emulated queues whose kernel side is driven
from here (:meth:`Runtime.deliver` / :meth:`Runtime.transmit`), so the whole
worker loop runs without AF_XDP privileges (the GPU box) and deterministically
in tests.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libxsknf.so")

EXPORTED_SYMBOLS = (
    "xsknf_parse_args", "xsknf_init", "xsknf_cleanup", "xsknf_start_workers", "xsknf_stop_workers",
    "xsknf_get_socket_stats", "xsknf_set_packet_processor", "xsknf_set_batch_processor",
    "xsknf_set_batch_processor_async", "xsknf_set_batch_depth",
    "xsknf_get_umem", "xsknf_worker_error", "xsknf_emu_deliver", "xsknf_emu_transmit",
)

XSKNF_MAX_INTERFACES = 32
XSKNF_MAX_WORKERS = 32
MODE_AF_XDP, MODE_XDP, MODE_COMBINED = 0x1, 0x2, 0x3
# linux/if_xdp.h, linux/if_link.h
XDP_COPY, XDP_ZEROCOPY, XDP_USE_NEED_WAKEUP = 1 << 1, 1 << 2, 1 << 3
XDP_FLAGS_UPDATE_IF_NOEXIST, XDP_FLAGS_SKB_MODE, XDP_FLAGS_DRV_MODE = 1 << 0, 1 << 1, 1 << 2
FRAMES_PER_SOCKET = 4096
XDP_HEADROOM = 256


class Config(ctypes.Structure):
    """struct xsknf_config (include/xsknf.h, = src/xsknf.h:25-40)."""

    _fields_ = [
        ("interfaces", ctypes.c_char_p * XSKNF_MAX_INTERFACES),
        ("bind_flags", ctypes.c_uint32 * XSKNF_MAX_INTERFACES),
        ("num_interfaces", ctypes.c_uint),
        ("workers", ctypes.c_uint),
        ("working_mode", ctypes.c_uint),
        ("xdp_flags", ctypes.c_uint32),
        ("batch_size", ctypes.c_uint32),
        ("poll", ctypes.c_int),
        ("unaligned_chunks", ctypes.c_int),
        ("xsk_frame_size", ctypes.c_int),
        ("busy_poll", ctypes.c_int),
        ("ebpf_filename", ctypes.c_char * 256),
        ("xdp_progname", ctypes.c_char * 256),
        ("tc_progname", ctypes.c_char * 256),
    ]


class SocketStats(ctypes.Structure):
    """struct xsknf_socket_stats: 13 unsigned longs (src/xsknf.h:42-59)."""

    _fields_ = [(n, ctypes.c_ulong) for n in (
        "rx_npkts", "tx_npkts", "rx_dropped_npkts", "rx_invalid_npkts", "tx_invalid_npkts",
        "rx_full_npkts", "rx_fill_empty_npkts", "tx_empty_npkts", "rx_empty_polls",
        "fill_fail_polls", "tx_wakeup_sendtos", "tx_trigger_sendtos", "opt_polls")]

    def as_dict(self) -> dict:
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class RuntimeError_(RuntimeError):
    pass


_lib_rt = None


def load() -> ctypes.CDLL:
    global _lib_rt
    if _lib_rt is not None:
        return _lib_rt
    if not os.path.exists(LIB_PATH):
        raise RuntimeError_(f"{LIB_PATH} is missing: build it with `make`")
    lib = ctypes.CDLL(LIB_PATH)
    lib.xsknf_parse_args.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(Config)]
    lib.xsknf_init.argtypes = [ctypes.POINTER(Config), ctypes.c_void_p]
    lib.xsknf_cleanup.argtypes = []
    lib.xsknf_start_workers.argtypes = []
    lib.xsknf_stop_workers.argtypes = []
    lib.xsknf_get_socket_stats.argtypes = [ctypes.c_uint, ctypes.c_uint, ctypes.POINTER(SocketStats)]
    lib.xsknf_set_packet_processor.argtypes = [ctypes.c_void_p]
    lib.xsknf_set_batch_processor.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.xsknf_set_batch_processor_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.xsknf_set_batch_depth.argtypes = [ctypes.c_uint]
    lib.xsknf_get_umem.argtypes = [ctypes.c_uint, ctypes.c_uint, ctypes.POINTER(ctypes.c_void_p),
                                   ctypes.POINTER(ctypes.c_uint64)]
    lib.xsknf_worker_error.argtypes = [ctypes.c_uint]
    lib.xsknf_emu_deliver.argtypes = [ctypes.c_uint, ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_uint32, ctypes.c_uint32]
    lib.xsknf_emu_transmit.argtypes = [ctypes.c_uint, ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.c_uint32]
    for name in EXPORTED_SYMBOLS:
        getattr(lib, name).restype = ctypes.c_int
    _lib_rt = lib
    return lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError_(f"{what} failed: rc={rc} ({os.strerror(-rc) if rc < 0 else rc})")


def parse_args(argv: Sequence[str], prog: str = "checksummer") -> Tuple[Config, List[str]]:
    """The runtime's own C xsknf_parse_args() (the reference's src/xsknf.c:777-874,
    getopt "i:pSf:ub:BM:w:" up to `--`): returns the struct xsknf_config and the
    application's arguments after `--`.  As in the reference, an invalid option
    prints the error and the usage and calls exit(1): the whole process ends."""
    lib = load()
    args = [prog, *argv]
    bufs = [ctypes.create_string_buffer(a.encode()) for a in args]
    arr = (ctypes.c_char_p * (len(args) + 1))()
    for i, b in enumerate(bufs):
        arr[i] = ctypes.cast(b, ctypes.c_char_p)
    libc = ctypes.CDLL(None)
    ctypes.c_int.in_dll(libc, "optind").value = 0        # glibc: full getopt re-initialisation
    cfg = Config()
    _check(lib.xsknf_parse_args(len(args), arr, ctypes.byref(cfg)), "xsknf_parse_args")
    cfg._argv_bufs = bufs                               # cfg.interfaces points into them
    optind = ctypes.c_int.in_dll(libc, "optind").value
    app = [arr[i].decode() for i in range(optind, len(args))]
    return cfg, app


def make_config(interfaces: Sequence[str], *, workers: int = 1, batch_size: int = 64,
                frame_size: int = 4096, unaligned: bool = False, skb_mode: bool = False,
                bind: Optional[Sequence[int]] = None, poll: bool = False) -> Config:
    """A struct xsknf_config as xsknf_parse_args would build it for these options."""
    c = Config()
    c._names = [s.encode() for s in interfaces]          # keep the strings alive
    for i, n in enumerate(c._names):
        c.interfaces[i] = n
        c.bind_flags[i] = XDP_USE_NEED_WAKEUP | (bind[i] if bind else 0)
    c.num_interfaces = len(interfaces)
    c.workers = workers
    c.working_mode = MODE_AF_XDP
    c.xdp_flags = XDP_FLAGS_UPDATE_IF_NOEXIST | (XDP_FLAGS_SKB_MODE if skb_mode else XDP_FLAGS_DRV_MODE)
    c.batch_size = batch_size
    c.poll = int(poll)
    c.unaligned_chunks = int(unaligned)
    c.xsk_frame_size = frame_size
    return c


class Runtime:
    """One xsknf_init() .. xsknf_cleanup() lifetime (the library is a singleton)."""

    def __init__(self, config: Config):
        self.lib = load()
        self.config = config
        _check(self.lib.xsknf_init(ctypes.byref(config), None), "xsknf_init")
        self.started = False

    # -- NF selection -------------------------------------------------------
    def set_packet_processor(self, fn_ptr: int) -> None:
        _check(self.lib.xsknf_set_packet_processor(ctypes.c_void_p(fn_ptr)), "set_packet_processor")

    def set_batch_processor(self, fn_ptr: Optional[int], user: Optional[int] = None) -> None:
        _check(self.lib.xsknf_set_batch_processor(ctypes.c_void_p(fn_ptr), ctypes.c_void_p(user)),
               "set_batch_processor")

    def set_batch_processor_async(self, submit_ptr: int, complete_ptr: int, user: Optional[int] = None) -> None:
        """The two-phase hook (xsknf_batch_submit_fn / xsknf_batch_complete_fn): one batch
        in flight per worker while the next is received."""
        _check(self.lib.xsknf_set_batch_processor_async(ctypes.c_void_p(submit_ptr), ctypes.c_void_p(complete_ptr),
                                                        ctypes.c_void_p(user)), "set_batch_processor_async")

    def set_batch_depth(self, depth: int) -> None:
        _check(self.lib.xsknf_set_batch_depth(depth), "set_batch_depth")

    # -- lifecycle ----------------------------------------------------------
    def start(self) -> None:
        _check(self.lib.xsknf_start_workers(), "xsknf_start_workers")
        self.started = True

    def stop(self) -> int:
        rc = self.lib.xsknf_stop_workers()
        self.started = False
        return rc

    def close(self) -> int:
        rc = self.lib.xsknf_cleanup()
        self.started = False
        # clear the NF so a later Runtime does not inherit it
        self.lib.xsknf_set_batch_processor(None, None)
        self.lib.xsknf_set_packet_processor(None)
        self.lib.xsknf_set_batch_depth(1)
        return rc

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- queries ------------------------------------------------------------
    def stats(self, worker: int = 0, iface: int = 0) -> dict:
        s = SocketStats()
        _check(self.lib.xsknf_get_socket_stats(worker, iface, ctypes.byref(s)), "get_socket_stats")
        return s.as_dict()

    def umem(self, worker: int = 0, iface: int = 0):
        p, n = ctypes.c_void_p(), ctypes.c_uint64()
        _check(self.lib.xsknf_get_umem(worker, iface, ctypes.byref(p), ctypes.byref(n)), "get_umem")
        return p.value, n.value

    def worker_error(self, worker: int = 0) -> int:
        return self.lib.xsknf_worker_error(worker)

    # -- emulated queues: the kernel's side ----------------------------------
    def deliver(self, frames: List[bytes], worker: int = 0, iface: int = 0) -> int:
        """Post as many of `frames` as the fill / rx rings allow; returns the count."""
        if not frames:
            return 0
        stride = max(len(f) for f in frames) or 1
        buf = np.zeros((len(frames), stride), dtype=np.uint8)
        lens = np.zeros(len(frames), dtype=np.uint32)
        for i, f in enumerate(frames):
            buf[i, :len(f)] = np.frombuffer(f, dtype=np.uint8)
            lens[i] = len(f)
        rc = self.lib.xsknf_emu_deliver(worker, iface, buf.ctypes.data, lens.ctypes.data, len(frames), stride)
        if rc < 0:
            _check(rc, "emu_deliver")
        return rc

    def transmit(self, max_frames: int = 4096, worker: int = 0, iface: int = 0,
                 stride: int = 10240) -> List[bytes]:
        out = np.zeros((max_frames, stride), dtype=np.uint8)
        lens = np.zeros(max_frames, dtype=np.uint32)
        rc = self.lib.xsknf_emu_transmit(worker, iface, out.ctypes.data, lens.ctypes.data, max_frames, stride)
        if rc < 0:
            _check(rc, "emu_transmit")
        return [out[i, :min(int(lens[i]), stride)].tobytes() for i in range(rc)]


class GpuHook:
    """The checksummer batch hook of libxsknf_gpu (xsknf_gpu_hook_*) for a Runtime."""

    def __init__(self, *, iterations: int = 1, action: int = _lib.ACTION_REDIRECT, num_interfaces: int = 1,
                 workers: int = 1, path: int = _lib.PATH_ZEROCOPY, max_batch: int = 64,
                 frame_len_hint: int = 4096):
        self.lib = _lib.load()
        self.opts = _lib.CsumOpts(iterations, action, num_interfaces, 0)
        h = ctypes.c_void_p()
        _lib.check(self.lib.xsknf_gpu_hook_create(ctypes.byref(h), ctypes.byref(self.opts), workers, path,
                                                  max_batch, frame_len_hint), "xsknf_gpu_hook_create")
        self.handle = h.value
        self.workers = workers

    @property
    def fn_ptr(self) -> int:
        return ctypes.cast(self.lib.xsknf_gpu_hook_process, ctypes.c_void_p).value

    @property
    def submit_ptr(self) -> int:
        return ctypes.cast(self.lib.xsknf_gpu_hook_submit, ctypes.c_void_p).value

    @property
    def complete_ptr(self) -> int:
        return ctypes.cast(self.lib.xsknf_gpu_hook_complete, ctypes.c_void_p).value

    def stats(self, worker: int = 0) -> dict:
        s = _lib.CtxStats()
        _lib.check(self.lib.xsknf_gpu_hook_get_stats(self.handle, worker, ctypes.byref(s)), "hook_get_stats")
        return {"batches": s.batches, "frames": s.frames, "bytes_h2d": s.bytes_h2d, "bytes_d2h": s.bytes_d2h}

    def destroy(self) -> None:
        if self.handle:
            self.lib.xsknf_gpu_hook_destroy(self.handle)
            self.handle = None
