"""ctypes binding of the C ABI declared in include/xsknf_gpu.h.

The product path is the gfx950 library ``xsknf_amd/lib/libxsknf_gpu.so`` built
by ``make`` (or ``__graft_entry__.build()``).  There is no fallback: if the
library is missing or fails to load, importing the binding raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# XSKNF_GPU_LIB: an alternative build of the same library (A/B experiments)
LIB_PATH = os.environ.get("XSKNF_GPU_LIB") or os.path.join(_HERE, "lib", "libxsknf_gpu.so")

# Every symbol include/xsknf_gpu.h declares (checked by tests/test_capi.py).
EXPORTED_SYMBOLS = (
    "xsknf_gpu_version",
    "xsknf_gpu_device_count",
    "xsknf_gpu_checksum_batch",
    "xsknf_gpu_last_error",
    "xsknf_gpu_pool_guard_trips",
    "xsknf_gpu_default_launch_cfg",
    "xsknf_gpu_checksum_batch_cfg",
    "xsknf_gpu_checksum_batch_lens",
    "xsknf_gpu_launch_cfg_for_lens",
    "xsknf_gpu_ctx_create",
    "xsknf_gpu_ctx_register_umem",
    "xsknf_gpu_ctx_process_batch",
    "xsknf_gpu_ctx_submit",
    "xsknf_gpu_ctx_wait",
    "xsknf_gpu_ctx_get_stats",
    "xsknf_gpu_ctx_destroy",
    "xsknf_gpu_hook_create",
    "xsknf_gpu_hook_process",
    "xsknf_gpu_hook_submit",
    "xsknf_gpu_hook_complete",
    "xsknf_gpu_hook_get_stats",
    "xsknf_gpu_hook_destroy",
    "xsknf_gpu_shard_plan",
    "xsknf_gpu_shard_rebase",
    "xsknf_gpu_shard_pack_plan",
    "xsknf_gpu_multi_create",
    "xsknf_gpu_multi_scatter",
    "xsknf_gpu_multi_scatter_packed",
    "xsknf_gpu_multi_return",
    "xsknf_gpu_multi_process",
    "xsknf_gpu_multi_counters",
    "xsknf_gpu_multi_shard_info",
    "xsknf_gpu_multi_fetch",
    "xsknf_gpu_multi_destroy",
)

MULTI_COUNTERS = 6   # XSKNF_GPU_MULTI_COUNTERS

PATH_ZEROCOPY = 0
PATH_STAGED = 1
PATH_RESIDENT = 2

ACTION_REDIRECT = 0
ACTION_DROP = 1


class CsumOpts(ctypes.Structure):
    """struct xsknf_csum_opts (include/xsknf_gpu.h)."""

    _fields_ = [
        ("csum_iterations", ctypes.c_int32),
        ("action", ctypes.c_int32),
        ("num_interfaces", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
    ]


class LaunchCfg(ctypes.Structure):
    """struct xsknf_gpu_launch_cfg (include/xsknf_gpu.h)."""

    _fields_ = [
        ("lanes_per_frame", ctypes.c_int32),
        ("chunks_per_lane", ctypes.c_int32),
        ("frames_per_group", ctypes.c_int32),
        ("blocks_per_cu", ctypes.c_int32),
        ("lds_ring", ctypes.c_int32),
        ("fused_stores", ctypes.c_int32),
        ("kernel", ctypes.c_int32),          # XSKNF_GPU_KERNEL_AUTO 0 / _SPLIT 1
        ("window_chunks", ctypes.c_int32),   # split kernel header window
    ]


class CtxStats(ctypes.Structure):
    """struct xsknf_gpu_ctx_stats (include/xsknf_gpu.h)."""

    _fields_ = [("batches", ctypes.c_uint64), ("frames", ctypes.c_uint64),
                ("bytes_h2d", ctypes.c_uint64), ("bytes_d2h", ctypes.c_uint64),
                ("resident_batches", ctypes.c_uint64), ("resident_launches", ctypes.c_uint64)]


SHARD_PACKED = 1   # XSKNF_GPU_SHARD_PACKED


class ShardInfo(ctypes.Structure):
    """struct xsknf_gpu_shard_info (include/xsknf_gpu.h)."""

    _fields_ = [("device", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("frame_lo", ctypes.c_uint64), ("frame_hi", ctypes.c_uint64),
                ("span_lo", ctypes.c_uint64), ("span_hi", ctypes.c_uint64),
                ("frame_bytes", ctypes.c_uint64),
                ("umem", ctypes.c_void_p), ("descs", ctypes.c_void_p), ("verdicts", ctypes.c_void_p)]


class XsknfGpuError(RuntimeError):
    pass


_lib = None


def _one_hip_runtime() -> None:
    """Bind the library to torch's HIP runtime when torch is installed.

    libxsknf_gpu.so needs libamdhip64.so.7 (RUNPATH /opt/rocm).  Loaded after
    torch, that name resolves to the HIP runtime torch bundles, and the process
    has one.  Loaded BEFORE torch, it pulls in /opt/rocm's runtime and torch
    then loads its own (libtorch_hip needs `libamdhip64.so`, a different name):
    two HIP and two HSA runtimes in one process, where torch.cuda.synchronize()
    does not wait for this library's launches and torch's stream handles mean
    nothing to it.  Importing torch first rules that out."""
    try:
        import torch  # noqa: F401
    except ImportError:     # a torch-free process (C tools, the NF binary) has one runtime anyway
        pass


def load() -> ctypes.CDLL:
    """Load the gfx950 library once; raise loudly if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    _one_hip_runtime()
    if not os.path.exists(LIB_PATH):
        raise XsknfGpuError(
            f"{LIB_PATH} is missing: build it with `make` or __graft_entry__.build(); "
            "there is no CPU fallback for the checksummer batch path")
    lib = ctypes.CDLL(LIB_PATH)
    lib.xsknf_gpu_version.restype = ctypes.c_uint32
    lib.xsknf_gpu_version.argtypes = []
    lib.xsknf_gpu_device_count.restype = ctypes.c_int
    lib.xsknf_gpu_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
    lib.xsknf_gpu_last_error.restype = ctypes.c_char_p
    lib.xsknf_gpu_last_error.argtypes = []
    lib.xsknf_gpu_checksum_batch.restype = ctypes.c_int
    lib.xsknf_gpu_checksum_batch.argtypes = [
        ctypes.c_void_p, ctypes.c_uint64,   # umem, umem_size
        ctypes.c_void_p, ctypes.c_uint32,   # descs, n
        ctypes.c_uint32,                    # ingress_ifindex
        ctypes.POINTER(CsumOpts),           # opts
        ctypes.c_void_p,                    # verdicts
        ctypes.c_uint32,                    # frame_len_hint
        ctypes.c_void_p,                    # stream
    ]
    lib.xsknf_gpu_default_launch_cfg.restype = ctypes.c_int
    lib.xsknf_gpu_default_launch_cfg.argtypes = [ctypes.c_uint32, ctypes.POINTER(LaunchCfg)]
    lib.xsknf_gpu_checksum_batch_lens.restype = ctypes.c_int
    lib.xsknf_gpu_checksum_batch_lens.argtypes = [
        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
        ctypes.POINTER(CsumOpts), ctypes.c_void_p,
        ctypes.c_uint32, ctypes.c_uint32,   # frame_len_max, frame_len_mean
        ctypes.c_void_p,
    ]
    lib.xsknf_gpu_launch_cfg_for_lens.restype = ctypes.c_int
    lib.xsknf_gpu_launch_cfg_for_lens.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(LaunchCfg)]
    lib.xsknf_gpu_checksum_batch_cfg.restype = ctypes.c_int
    lib.xsknf_gpu_checksum_batch_cfg.argtypes = [
        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
        ctypes.POINTER(CsumOpts), ctypes.c_void_p, ctypes.POINTER(LaunchCfg), ctypes.c_void_p,
    ]
    lib.xsknf_gpu_ctx_create.restype = ctypes.c_int
    lib.xsknf_gpu_ctx_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int,
                                         ctypes.c_uint32, ctypes.c_uint32]
    lib.xsknf_gpu_ctx_register_umem.restype = ctypes.c_int
    lib.xsknf_gpu_ctx_register_umem.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    lib.xsknf_gpu_ctx_process_batch.restype = ctypes.c_int
    lib.xsknf_gpu_ctx_process_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                ctypes.c_uint32, ctypes.POINTER(CsumOpts),
                                                ctypes.c_void_p]
    lib.xsknf_gpu_ctx_submit.restype = ctypes.c_int
    lib.xsknf_gpu_ctx_submit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.POINTER(CsumOpts), ctypes.c_void_p,
                                         ctypes.POINTER(ctypes.c_uint64)]
    lib.xsknf_gpu_ctx_wait.restype = ctypes.c_int
    lib.xsknf_gpu_ctx_wait.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    lib.xsknf_gpu_ctx_get_stats.restype = ctypes.c_int
    lib.xsknf_gpu_ctx_get_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(CtxStats)]
    lib.xsknf_gpu_ctx_destroy.restype = ctypes.c_int
    lib.xsknf_gpu_ctx_destroy.argtypes = [ctypes.c_void_p]
    lib.xsknf_gpu_hook_create.restype = ctypes.c_int
    lib.xsknf_gpu_hook_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(CsumOpts),
                                          ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32]
    lib.xsknf_gpu_hook_process.restype = ctypes.c_int
    lib.xsknf_gpu_hook_process.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64,
                                           ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    lib.xsknf_gpu_hook_submit.restype = ctypes.c_int
    lib.xsknf_gpu_hook_submit.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64,
                                          ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_uint64)]
    lib.xsknf_gpu_hook_complete.restype = ctypes.c_int
    lib.xsknf_gpu_hook_complete.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
    lib.xsknf_gpu_hook_get_stats.restype = ctypes.c_int
    lib.xsknf_gpu_hook_get_stats.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(CtxStats)]
    lib.xsknf_gpu_hook_destroy.restype = ctypes.c_int
    lib.xsknf_gpu_hook_destroy.argtypes = [ctypes.c_void_p]
    u64, vp = ctypes.c_uint64, ctypes.c_void_p
    lib.xsknf_gpu_shard_plan.restype = ctypes.c_int
    lib.xsknf_gpu_shard_plan.argtypes = [vp, u64, u64, ctypes.c_uint32, vp, vp]
    lib.xsknf_gpu_shard_rebase.restype = ctypes.c_int
    lib.xsknf_gpu_shard_rebase.argtypes = [vp, u64, u64, u64, vp]
    lib.xsknf_gpu_multi_create.restype = ctypes.c_int
    lib.xsknf_gpu_shard_pack_plan.restype = ctypes.c_int
    lib.xsknf_gpu_shard_pack_plan.argtypes = [vp, u64, u64, u64, ctypes.c_uint32, vp, vp, vp]
    lib.xsknf_gpu_multi_create.argtypes = [ctypes.POINTER(vp), vp, ctypes.c_int]
    lib.xsknf_gpu_multi_scatter.restype = ctypes.c_int
    lib.xsknf_gpu_multi_scatter.argtypes = [vp, ctypes.c_int, vp, u64, vp, u64, ctypes.POINTER(ctypes.c_double)]
    lib.xsknf_gpu_multi_process.restype = ctypes.c_int
    lib.xsknf_gpu_multi_scatter_packed.restype = ctypes.c_int
    lib.xsknf_gpu_multi_scatter_packed.argtypes = [vp, ctypes.c_int, vp, u64, vp, u64, ctypes.POINTER(ctypes.c_double)]
    lib.xsknf_gpu_multi_return.restype = ctypes.c_int
    lib.xsknf_gpu_multi_return.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(CsumOpts), ctypes.c_uint32,
                                           ctypes.c_uint32, vp, vp, vp, ctypes.POINTER(ctypes.c_double)]
    lib.xsknf_gpu_multi_process.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(CsumOpts), ctypes.c_uint32,
                                            ctypes.c_uint32, vp]
    lib.xsknf_gpu_multi_counters.restype = ctypes.c_int
    lib.xsknf_gpu_multi_counters.argtypes = [vp, vp]
    lib.xsknf_gpu_multi_shard_info.restype = ctypes.c_int
    lib.xsknf_gpu_multi_shard_info.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ShardInfo)]
    lib.xsknf_gpu_multi_fetch.restype = ctypes.c_int
    lib.xsknf_gpu_multi_fetch.argtypes = [vp, ctypes.c_int, vp, vp, vp]
    lib.xsknf_gpu_multi_destroy.restype = ctypes.c_int
    lib.xsknf_gpu_multi_destroy.argtypes = [vp]
    lib.xsknf_gpu_pool_guard_trips.restype = ctypes.c_int
    lib.xsknf_gpu_pool_guard_trips.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
    _lib = lib
    return lib


def pool_guard_trips(reset: bool = False) -> int:
    """Waves of the pooled split kernel on the current device that found a unit
    no wave claimed (include/xsknf_gpu.h xsknf_gpu_pool_guard_trips; 0 unless
    the library's grid bound is wrong)."""
    t = ctypes.c_uint32(0)
    check(load().xsknf_gpu_pool_guard_trips(ctypes.byref(t), 1 if reset else 0), "xsknf_gpu_pool_guard_trips")
    return int(t.value)


def last_error() -> str:
    return load().xsknf_gpu_last_error().decode(errors="replace")


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise XsknfGpuError(f"{what} failed: rc={rc} ({os.strerror(-rc) if rc < 0 else rc}); "
                            f"last HIP error: {last_error()!r}")
