// host_path.hip -- the batch hook with the UMEM in host memory.
//
// In the reference, an AF_XDP worker (src/xsknf.c:716-742) peeks up to
// batch_size rx descriptors and calls xsknf_packet_processor() on each frame,
// in place in the worker's mmap'd UMEM (src/xsknf.c:654-672, :958/:975).  This
// context is what such a worker holds to run that loop on the GPU instead:
// host UMEM registered once, then one synchronous call per rx batch with the
// descriptors and verdicts in host arrays.
//
// ZEROCOPY: the UMEM is pinned and mapped into the device address space; the
//   kernel reads the frames and writes the check bytes over PCIe, in place.
//   Checks are written in-line (fused stores): a deferred sector rewrite would
//   re-read sectors over PCIe.
// STAGED: the byte span of the batch's frames is copied to a device mirror of
//   the UMEM (hipMemcpyAsync from pinned memory), summed in HBM with every
//   check deferred, and only the 4-byte per-frame records come back; the host
//   then writes each frame's 2 check bytes itself.  Copying the span back
//   instead would overwrite frames outside the batch that the kernel / NIC may
//   be filling concurrently (fill-ring frames), so it never does.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <new>

#include "../../include/xsknf_gpu.h"
#include "checksummer_internal.h"

struct xsknf_gpu_ctx {
  int device = 0;
  int path = XSKNF_GPU_PATH_ZEROCOPY;
  uint32_t max_batch = 0;
  uint32_t hint = 0;
  hipStream_t stream = nullptr;
  uint8_t *umem_host = nullptr;
  uint64_t umem_size = 0;
  uint8_t *umem_dev = nullptr;        // mapped host pointer (ZEROCOPY) or device mirror (STAGED)
  bool registered = false;
  xsknf_gpu_desc *descs_dev = nullptr;
  int32_t *verdicts_dev = nullptr;
  xsknf_gpu_desc *descs_pinned = nullptr;
  int32_t *verdicts_pinned = nullptr;
  xsknf_gpu_desc *descs_mapped = nullptr;   // device views of the pinned arrays (direct mode)
  int32_t *verdicts_mapped = nullptr;
  xsknf_gpu_ctx_stats stats = {};
};

// Direct mode (the default): the kernel reads the descriptors from, and
// writes the verdicts / records to, the pinned host arrays themselves, so a
// call is one launch and one synchronize -- no H2D descriptor copy and no D2H
// verdict copy, each a separate DMA command with its own latency (a batch of 64
// frames: 39 us per call with both copies).  -DXSKNF_CTX_COPY_ARRAYS keeps the
// copies (A/B builds).
#ifdef XSKNF_CTX_COPY_ARRAYS
constexpr bool kDirect = false;
#else
constexpr bool kDirect = true;
#endif

namespace {

int fail(hipError_t e, const char *where) {
  xsknf_gpu::set_error(e, where);
  return -EIO;
}

uint64_t umem_offset(uint64_t addr) {
  return (addr & XSKNF_GPU_UNALIGNED_BUF_ADDR_MASK) + (addr >> XSKNF_GPU_UNALIGNED_BUF_OFFSET_SHIFT);
}

void release(xsknf_gpu_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->registered) (void)hipHostUnregister(c->umem_host);
  if (c->path == XSKNF_GPU_PATH_STAGED && c->umem_dev) (void)hipFree(c->umem_dev);
  if (c->descs_dev) (void)hipFree(c->descs_dev);
  if (c->verdicts_dev) (void)hipFree(c->verdicts_dev);
  if (c->descs_pinned) (void)hipHostFree(c->descs_pinned);
  if (c->verdicts_pinned) (void)hipHostFree(c->verdicts_pinned);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

}  // namespace

extern "C" {

int xsknf_gpu_ctx_create(struct xsknf_gpu_ctx **out, int device, int path, uint32_t max_batch,
                         uint32_t frame_len_hint) {
  if (!out || max_batch == 0) return -EINVAL;
  if (path != XSKNF_GPU_PATH_ZEROCOPY && path != XSKNF_GPU_PATH_STAGED) return -EINVAL;
  *out = nullptr;
  xsknf_gpu_ctx *c = new (std::nothrow) xsknf_gpu_ctx;
  if (!c) return -ENOMEM;
  c->device = device;
  c->path = path;
  c->max_batch = max_batch;
  c->hint = frame_len_hint;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&c->descs_dev, sizeof(xsknf_gpu_desc) * max_batch);
  if (e == hipSuccess) e = hipMalloc(&c->verdicts_dev, sizeof(int32_t) * max_batch);
  if (e == hipSuccess) e = hipHostMalloc(&c->descs_pinned, sizeof(xsknf_gpu_desc) * max_batch, hipHostMallocDefault);
  if (e == hipSuccess) e = hipHostMalloc(&c->verdicts_pinned, sizeof(int32_t) * max_batch, hipHostMallocDefault);
  if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&c->descs_mapped), c->descs_pinned, 0);
  if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&c->verdicts_mapped), c->verdicts_pinned, 0);
  if (e != hipSuccess) {
    const int rc = fail(e, "xsknf_gpu_ctx_create");
    release(c);
    return rc;
  }
  *out = c;
  return 0;
}

int xsknf_gpu_ctx_register_umem(struct xsknf_gpu_ctx *c, void *umem, uint64_t size) {
  if (!c || !umem || size == 0 || c->registered) return -EINVAL;
  hipError_t e = hipSetDevice(c->device);
  const unsigned flags = c->path == XSKNF_GPU_PATH_ZEROCOPY ? hipHostRegisterMapped : hipHostRegisterDefault;
  if (e == hipSuccess) e = hipHostRegister(umem, size, flags);
  if (e != hipSuccess) return fail(e, "hipHostRegister(umem)");
  c->registered = true;
  c->umem_host = static_cast<uint8_t *>(umem);
  c->umem_size = size;
  if (c->path == XSKNF_GPU_PATH_ZEROCOPY) {
    void *dp = nullptr;
    e = hipHostGetDevicePointer(&dp, umem, 0);
    c->umem_dev = static_cast<uint8_t *>(dp);
  } else {
    e = hipMalloc(&c->umem_dev, size);
  }
  if (e != hipSuccess) {
    (void)hipHostUnregister(umem);
    c->registered = false;
    c->umem_dev = nullptr;
    return fail(e, "xsknf_gpu_ctx_register_umem");
  }
  return 0;
}

int xsknf_gpu_ctx_process_batch(struct xsknf_gpu_ctx *c, const struct xsknf_gpu_desc *descs, uint32_t n,
                                uint32_t ingress_ifindex, const struct xsknf_csum_opts *opts,
                                int32_t *verdicts) {
  using namespace xsknf_gpu;
  if (!c || !c->registered || n > c->max_batch) return -EINVAL;
  if (n == 0) return 0;
  if (!descs || !verdicts) return -EINVAL;
  KernelArgs a;
  int rc = prepare(a, c->umem_dev, c->umem_size, kDirect ? c->descs_mapped : c->descs_dev, n, ingress_ifindex,
                   opts, kDirect ? c->verdicts_mapped : c->verdicts_dev);
  if (rc != 0) return rc < 0 ? rc : 0;
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) return fail(e, "hipSetDevice");

  memcpy(c->descs_pinned, descs, sizeof(xsknf_gpu_desc) * n);
  if (!kDirect) {
    e = hipMemcpyAsync(c->descs_dev, c->descs_pinned, sizeof(xsknf_gpu_desc) * n, hipMemcpyHostToDevice,
                       c->stream);
    if (e != hipSuccess) return fail(e, "hipMemcpyAsync(descs)");
  }
  c->stats.bytes_h2d += sizeof(xsknf_gpu_desc) * n;

  xsknf_gpu_launch_cfg cfg;
  default_cfg(c->hint ? c->hint : 2048u, cfg);
  if (c->path == XSKNF_GPU_PATH_ZEROCOPY && n <= 2048) {
    // A small batch is a few 64-frame tiles: the split kernel would read it
    // over PCIe with a few waves.  The group kernel spreads it over many
    // (4 or 2 frames per wave), so more reads are in flight
    // (tools/small_batch.py, 1500 B: 64 frames 44.8 -> 18.8 us per call,
    // 256: 46.8 -> 24.1, 1024: 51.0 -> 45.0; equal from 4096).
    cfg.kernel = XSKNF_GPU_KERNEL_AUTO;
    cfg.window_chunks = 0;
    cfg.lds_ring = 0;
    cfg.lanes_per_frame = n <= 256 ? 32 : 64;
    cfg.chunks_per_lane = n <= 256 ? 3 : 2;
    cfg.frames_per_group = n <= 256 ? 2 : 4;
  }
  if (c->path == XSKNF_GPU_PATH_STAGED) {
    // byte span of the batch's (in-range) frames
    uint64_t lo = UINT64_MAX, hi = 0;
    for (uint32_t i = 0; i < n; ++i) {
      const uint64_t off = umem_offset(descs[i].addr);
      if (off > c->umem_size || descs[i].len > c->umem_size - off) continue;
      lo = off < lo ? off : lo;
      hi = off + descs[i].len > hi ? off + descs[i].len : hi;
    }
    if (hi > lo) {
      e = hipMemcpyAsync(c->umem_dev + lo, c->umem_host + lo, hi - lo, hipMemcpyHostToDevice, c->stream);
      if (e != hipSuccess) return fail(e, "hipMemcpyAsync(umem span)");
      c->stats.bytes_h2d += hi - lo;
    }
    cfg.fused_stores = 3;   // records only: the checks are applied on the host below
  } else {
    cfg.fused_stores = 1;   // in place over PCIe, ...
    a.sector_stores = 0;    // ... as 2-byte writes (byte enables; no RMW in host memory)
  }
  rc = run(a, cfg, c->stream);
  if (rc != 0) return rc;
  e = kDirect ? hipSuccess
              : hipMemcpyAsync(c->verdicts_pinned, c->verdicts_dev, sizeof(int32_t) * n, hipMemcpyDeviceToHost,
                               c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return fail(e, "verdict copy-back");
  c->stats.bytes_d2h += sizeof(int32_t) * n;

  if (c->path == XSKNF_GPU_PATH_STAGED) {
    // checksummer_user.c:108 on the host: the 2 check bytes of every summed frame
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t r = static_cast<uint32_t>(c->verdicts_pinned[i]);
      if ((r & kRecTagMask) == kRecTag) {
        uint8_t *p = c->umem_host + umem_offset(descs[i].addr) + ((r >> 16) & 0x7f) + 6;
        p[0] = static_cast<uint8_t>(r);
        p[1] = static_cast<uint8_t>(r >> 8);
        verdicts[i] = a.fwd_verdict;
      } else {
        verdicts[i] = static_cast<int32_t>(r);
      }
    }
  } else {
    memcpy(verdicts, c->verdicts_pinned, sizeof(int32_t) * n);
  }
  c->stats.batches += 1;
  c->stats.frames += n;
  return 0;
}

int xsknf_gpu_ctx_get_stats(const struct xsknf_gpu_ctx *c, struct xsknf_gpu_ctx_stats *stats) {
  if (!c || !stats) return -EINVAL;
  *stats = c->stats;
  return 0;
}

int xsknf_gpu_ctx_destroy(struct xsknf_gpu_ctx *c) {
  if (!c) return -EINVAL;
  release(c);
  return 0;
}

}  // extern "C"

// ---- batch hook: one context per (worker, UMEM) ------------------------------

namespace {

constexpr int kUmemsPerWorker = 2;  // a worker's zero-copy and copy-mode UMEMs

struct HookSlot {
  void *umem = nullptr;
  xsknf_gpu_ctx *ctx = nullptr;
};

struct HookWorker {
  HookSlot slot[kUmemsPerWorker];
} __attribute__((aligned(64)));   // workers write their own slots only

}  // namespace

struct xsknf_gpu_hook {
  xsknf_csum_opts opts = {};
  uint32_t workers = 0;
  int path = XSKNF_GPU_PATH_ZEROCOPY;
  uint32_t max_batch = 0;
  uint32_t hint = 0;
  int devices = 1;
  HookWorker *w = nullptr;
};

extern "C" {

int xsknf_gpu_hook_create(struct xsknf_gpu_hook **out, const struct xsknf_csum_opts *opts, uint32_t workers,
                          int path, uint32_t max_batch, uint32_t frame_len_hint) {
  if (!out || !opts || workers == 0 || max_batch == 0) return -EINVAL;
  if (path != XSKNF_GPU_PATH_ZEROCOPY && path != XSKNF_GPU_PATH_STAGED) return -EINVAL;
  if (opts->action != XSKNF_CSUM_ACTION_REDIRECT && opts->action != XSKNF_CSUM_ACTION_DROP) return -EINVAL;
  *out = nullptr;
  int devices = 0;
  hipError_t e = hipGetDeviceCount(&devices);
  if (e != hipSuccess) return fail(e, "hipGetDeviceCount");
  if (devices < 1) return -ENODEV;
  xsknf_gpu_hook *h = new (std::nothrow) xsknf_gpu_hook;
  if (!h) return -ENOMEM;
  h->w = new (std::nothrow) HookWorker[workers];
  if (!h->w) {
    delete h;
    return -ENOMEM;
  }
  h->opts = *opts;
  h->workers = workers;
  h->path = path;
  h->max_batch = max_batch;
  h->hint = frame_len_hint;
  h->devices = devices;
  *out = h;
  return 0;
}

int xsknf_gpu_hook_process(void *hook, uint32_t worker_idx, void *umem, uint64_t umem_size,
                           const struct xsknf_gpu_desc *descs, uint32_t n, uint32_t ingress_ifindex,
                           int32_t *verdicts) {
  xsknf_gpu_hook *h = static_cast<xsknf_gpu_hook *>(hook);
  if (!h || worker_idx >= h->workers || !umem || umem_size == 0) return -EINVAL;
  if (n > h->max_batch) return -EINVAL;
  HookWorker &w = h->w[worker_idx];
  xsknf_gpu_ctx *ctx = nullptr;
  for (HookSlot &s : w.slot) {
    if (s.umem == umem) {
      ctx = s.ctx;
      break;
    }
  }
  if (!ctx) {
    HookSlot *free_slot = nullptr;
    for (HookSlot &s : w.slot) {
      if (!s.umem) {
        free_slot = &s;
        break;
      }
    }
    if (!free_slot) return -ENOSPC;
    int rc = xsknf_gpu_ctx_create(&ctx, static_cast<int>(worker_idx % static_cast<uint32_t>(h->devices)),
                                  h->path, h->max_batch, h->hint);
    if (rc) return rc;
    rc = xsknf_gpu_ctx_register_umem(ctx, umem, umem_size);
    if (rc) {
      xsknf_gpu_ctx_destroy(ctx);
      return rc;
    }
    free_slot->umem = umem;
    free_slot->ctx = ctx;
  }
  return xsknf_gpu_ctx_process_batch(ctx, descs, n, ingress_ifindex, &h->opts, verdicts);
}

int xsknf_gpu_hook_get_stats(const struct xsknf_gpu_hook *h, uint32_t worker_idx, struct xsknf_gpu_ctx_stats *stats) {
  if (!h || !stats || worker_idx >= h->workers) return -EINVAL;
  *stats = {};
  for (const HookSlot &s : h->w[worker_idx].slot) {
    if (!s.ctx) continue;
    stats->batches += s.ctx->stats.batches;
    stats->frames += s.ctx->stats.frames;
    stats->bytes_h2d += s.ctx->stats.bytes_h2d;
    stats->bytes_d2h += s.ctx->stats.bytes_d2h;
  }
  return 0;
}

int xsknf_gpu_hook_destroy(struct xsknf_gpu_hook *h) {
  if (!h) return -EINVAL;
  for (uint32_t i = 0; i < h->workers; ++i)
    for (HookSlot &s : h->w[i].slot)
      if (s.ctx) release(s.ctx);
  delete[] h->w;
  delete h;
  return 0;
}

}  // extern "C"
