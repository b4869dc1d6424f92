// multi.hip -- one process over N devices: config 4's global batch, sharded.
//
// The reference scales one worker per NIC queue (src/xsknf.c:992, the worker
// loop started per queue at :1046-1100): frames never cross workers, so its
// parallelism is independent batches.  On a node of MI355X the same holds per
// device, and the per-worker hook (host_path.hip: worker w on device
// w % devices) is that model.  This file adds what a C host needs when a
// global batch starts on ONE device (BASELINE config 4):
//
//   * xsknf_gpu_shard_plan  -- contiguous descriptor ranges balanced by frame
//     bytes (the kernel is HBM-bound: bytes set each device's time), and the
//     UMEM byte span of each range; the same cuts as xsknf_amd/shard.py.
//   * xsknf_gpu_multi_create -- one RCCL communicator per device
//     (ncclCommInitAll: one process drives every device), a stream each.
//   * xsknf_gpu_multi_scatter -- each shard moved from the root device as ONE
//     span of UMEM bytes plus its rebased descriptors, by grouped ncclSend /
//     ncclRecv: every peer's transfer at once, each on its own xGMI link (the
//     root's own shard too, as a send to itself, so the path is the same at
//     N = 1).  A point-to-point pattern, not a ring collective.
//   * xsknf_gpu_multi_process -- the checksummer on every device's shard, each
//     on its own stream, all in flight together (no data-path collective).
//   * xsknf_gpu_multi_counters -- {frames, bytes, drops, forwards, sum of the
//     written checks, the same weighted by global UMEM offset} per device,
//     summed over devices by ncclAllReduce: the whole batch's result, as one
//     device's pass over all of it would give it.
//   * xsknf_gpu_multi_scatter_packed -- the same distribution moving only the
//     frames' bytes: a gather kernel on the root copies each shard's frames
//     into 16-byte slots (a frame keeps its address mod 16), so a UMEM of 2 KiB
//     chunks holding IMIX frames (mean 352 B) sends ~1/5 of its span bytes.
//   * xsknf_gpu_multi_return -- the results back to the root: each device runs
//     the summing pass in records-only mode over its shard (include/
//     xsknf_gpu.h fused_stores 3: the shard is only read), sends its 4-byte
//     records / verdicts to the root (grouped ncclSend / ncclRecv), and an apply
//     kernel on the root writes every changed check into the root's UMEM and
//     every final verdict: the root ends with the bytes and verdicts of one
//     device's pass over the whole batch, having moved frames out and 4 bytes
//     per frame back.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <new>
#include <vector>

#include "../../include/xsknf_gpu.h"
#include "checksummer_internal.h"

namespace {

constexpr uint64_t kOutOfRange = 1ull << 47;   // an address past any UMEM: verdict -1, no bytes
constexpr uint32_t kFingerprintMod = 65521;
// Bytes per ncclSend / ncclRecv of a scatter.  One ncclSend of a whole span
// past 1 GiB delivered only part of it with this image's RCCL (a send to self
// of the 2 GiB and 16 GiB spans of 1M and 8M IMIX frames: the bytes from 1 GiB
// on -- from 2 GiB on in 4 GiB pieces -- never arrived, while the calls and the
// group returned success); 256 MiB pieces delivered every byte
// (profiles/r06/multi_p2p_pieces.jsonl; the probe, with the piece size as an
// environment knob, is in commit cca61bb's tools/diag_multi_p2p.py).
constexpr uint64_t kP2PPiece = 1ull << 28;

__host__ __device__ inline uint64_t umem_offset(uint64_t addr) {
  return (addr & XSKNF_GPU_UNALIGNED_BUF_ADDR_MASK) + (addr >> XSKNF_GPU_UNALIGNED_BUF_OFFSET_SHIFT);
}

int nccl_fail(ncclResult_t r, const char *where) {
  char buf[256];
  snprintf(buf, sizeof(buf), "%s: %s", where, ncclGetErrorString(r));
  xsknf_gpu::set_error_text(buf);
  return -EIO;
}

int hip_fail(hipError_t e, const char *where) {
  xsknf_gpu::set_error(e, where);
  return e == hipErrorOutOfMemory ? -ENOMEM : -EIO;
}

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// Per frame of one shard: [frames, bytes, drops, forwards, checks, weighted
// checks] -- the bytes over every descriptor's len (xsknf_amd/shard.py
// counters()), the checks over the frames of at least 42 bytes inside the span
// (the UDP check of an ihl-5 frame at +40, as bench.py check_fingerprint reads
// it), weighted by (global offset mod 65521) + 1 so that a check landing in
// another frame shows.  One wave per 64 frames, a block sum, one atomic per
// counter and block (vector atomics to device memory).
__global__ void __launch_bounds__(256) shard_counters(const uint8_t *umem, uint64_t span,
                                                      const xsknf_gpu_desc *descs, const int32_t *verdicts,
                                                      uint64_t n, uint64_t base, unsigned long long *out) {
  unsigned long long c[XSKNF_GPU_MULTI_COUNTERS] = {};
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const xsknf_gpu_desc d = descs[i];
    const int32_t v = verdicts[i];
    c[0] += 1;
    c[1] += d.len;
    c[2] += v == -1;
    c[3] += v >= 0;
    const uint64_t off = umem_offset(d.addr);
    if (d.len >= 42 && off <= span && d.len <= span - off) {
      const unsigned long long ck = umem[off + 40] | static_cast<unsigned>(umem[off + 41]) << 8;
      c[4] += ck;
      c[5] += ck * ((off + base) % kFingerprintMod + 1);
    }
  }
  __shared__ unsigned long long red[XSKNF_GPU_MULTI_COUNTERS][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < XSKNF_GPU_MULTI_COUNTERS; ++k) {
    unsigned long long x = c[k];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) red[k][wv] = x;
  }
  __syncthreads();
  if (threadIdx.x < XSKNF_GPU_MULTI_COUNTERS) {
    const int k = threadIdx.x;
    atomicAdd(&out[k], red[k][0] + red[k][1] + red[k][2] + red[k][3]);
  }
}

// Root: copy frames [0, n) of one shard into its packed buffer.  Frame f's
// bytes lie in the 16-byte aligned chunks [src & ~15, round16(src + len)) of
// memory (src = its address) and go to the slot at dst & ~15 of the packed
// buffer, whose length is exactly those chunks (dst = src mod 16 + the slot's
// start): whole chunks move, and the bytes around the frame in its first and
// last chunk are copied with it into its own slot.  One wave per 64 frames:
// the tile's chunk counts are prefix-summed across the wave and the lanes deal
// the tile's chunks round robin (a 64-B frame is 4-5 chunks, a jumbo one 563).
// A chunk reaching past the UMEM's end is copied byte by byte.
__global__ void __launch_bounds__(256) pack_frames(const uint8_t *umem, uint64_t umem_size,
                                                   const xsknf_gpu_desc *orig, const xsknf_gpu_desc *packed,
                                                   uint64_t n, uint8_t *dst) {
  __shared__ uint32_t pre[4][65];
  __shared__ uint64_t src_of[4][64], dst_of[4][64];   // a frame's first chunk and its slot (read by any lane)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t tiles = (n + 63) / 64;
  for (uint64_t t = blockIdx.x * 4ull + wv; t < tiles; t += gridDim.x * 4ull) {
    const uint64_t f = t * 64 + lane;
    uint64_t s0 = 0, d0 = 0;   // the first chunk's address (absolute) and its slot offset in dst
    uint32_t nch = 0;
    if (f < n) {
      const xsknf_gpu_desc o = orig[f], q = packed[f];
      const uint64_t src = reinterpret_cast<uintptr_t>(umem) + umem_offset(o.addr);
      if (q.addr != kOutOfRange && o.len > 0) {
        s0 = src & ~15ull;
        d0 = q.addr & ~15ull;
        nch = static_cast<uint32_t>(((src & 15) + o.len + 15) >> 4);
      }
    }
    // inclusive scan of the chunk counts over the wave
    uint32_t x = nch;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    pre[wv][lane + 1] = x;
    if (lane == 0) pre[wv][0] = 0;
    src_of[wv][lane] = s0;
    dst_of[wv][lane] = d0;
    __builtin_amdgcn_wave_barrier();   // (one wave's LDS accesses complete in order)
    const uint32_t total = __shfl(x, 63);
    const uint64_t begin = reinterpret_cast<uintptr_t>(umem), end = begin + umem_size;
    for (uint32_t k = lane; k < total; k += 64) {
      // the frame j of the tile whose chunks hold chunk k: pre[j] <= k < pre[j + 1]
      int lo = 0, hi = 63;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pre[wv][mid] <= k) lo = mid; else hi = mid - 1;
      }
      const uint32_t c = k - pre[wv][lo];
      // (from LDS, not by a lane shuffle: the loop's last round leaves lanes
      // inactive, and a shuffle reads nothing from an inactive lane)
      const uint64_t sa = src_of[wv][lo] + 16ull * c, da = dst_of[wv][lo] + 16ull * c;
      if (sa >= begin && sa + 16 <= end) {
        *reinterpret_cast<uint4 *>(dst + da) = *reinterpret_cast<const uint4 *>(sa);
      } else {   // a chunk reaching before the UMEM's first byte or past its last
        for (uint64_t b = sa > begin ? sa : begin; b < sa + 16 && b < end; ++b)
          dst[da + (b - sa)] = *reinterpret_cast<const uint8_t *>(b);
      }
    }
    __builtin_amdgcn_wave_barrier();   // pre[wv] is rewritten by the next tile
  }
}

// Root: the returned records / verdicts of the whole batch, in place: a record
// (XSKNF_GPU_RECORD_TAG | u << 16 | check) writes the check's two bytes, low
// byte first, at the frame's offset u + 6 (checksummer_user.c:108) and becomes
// the forward verdict (:110-111); any other value is already the verdict.
__global__ void __launch_bounds__(256) apply_records(uint8_t *umem, const xsknf_gpu_desc *orig, int32_t *verdicts,
                                                     uint64_t n, int32_t fwd) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint32_t r = static_cast<uint32_t>(verdicts[i]);
    if ((r & XSKNF_GPU_RECORD_TAG_MASK) != XSKNF_GPU_RECORD_TAG) continue;
    uint8_t *p = umem + umem_offset(orig[i].addr) + ((r >> 16) & 0x7f) + 6;
    p[0] = static_cast<uint8_t>(r);
    p[1] = static_cast<uint8_t>(r >> 8);
    verdicts[i] = fwd;
  }
}

struct Shard {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  uint64_t lo = 0, hi = 0;       // frames [lo, hi) of the global batch
  uint64_t b0 = 0, b1 = 0;       // its UMEM byte span on the root (packed: 0 and its packed bytes)
  uint64_t bytes = 0;            // sum of the shard's frame lengths
  uint8_t *umem = nullptr;       // b1 - b0 bytes + 16 spare (the kernels' 16-byte chunk loads), inside umem_alloc
  uint8_t *umem_alloc = nullptr; // at the root's address mod kPlace (span scatter): the same placement as there
  uint64_t umem_cap = 0;
  xsknf_gpu_desc *descs = nullptr;
  int32_t *verdicts = nullptr;
  uint64_t frames_cap = 0;
  unsigned long long *counters = nullptr;   // device: XSKNF_GPU_MULTI_COUNTERS
};

}  // namespace

struct xsknf_gpu_multi {
  int ndev = 0;
  std::vector<int> devices;
  std::vector<ncclComm_t> comms;
  std::vector<Shard> sh;
  xsknf_gpu_desc *root_descs = nullptr;   // the rebased descriptors of every shard, on the root device
  uint64_t root_descs_cap = 0;
  int root_descs_dev = -1;                // the device root_descs lives on
  int root = -1;                          // index of the root of the last scatter
  uint64_t n = 0;                         // frames of the last scatter
  bool packed = false;                    // the last scatter moved packed frames
  bool processed = false;                 // _process wrote checks into the shards since the last scatter
  // on the root device (root_descs_dev): the last scatter's descriptors as the
  // caller gave them (for the results' return) and the packed staging buffer
  xsknf_gpu_desc *root_orig = nullptr;
  uint64_t root_orig_cap = 0;
  uint8_t *root_pack = nullptr;
  uint64_t root_pack_cap = 0;
};

namespace {

// (Re)allocate a root-device buffer to at least `bytes`.
template <typename T>
hipError_t root_buffer(T *&p, uint64_t &cap, uint64_t bytes) {
  if (p && bytes <= cap) return hipSuccess;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  hipError_t e = hipMalloc(reinterpret_cast<void **>(&p), bytes ? bytes : 1);
  if (e == hipSuccess) cap = bytes;
  return e;
}

// The root-side staging of a scatter: the device the root buffers live on
// becomes devices[root] (buffers of an earlier root are freed), the caller's
// descriptors go to root_orig (for the results' return) and `sent` (the
// descriptors each shard receives, in global order) to root_descs.
hipError_t stage_root(xsknf_gpu_multi *m, int root, const xsknf_gpu_desc *descs, const xsknf_gpu_desc *sent,
                      uint64_t n) {
  hipError_t e = hipSuccess;
  if (m->root_descs_dev >= 0 && m->root_descs_dev != m->devices[root]) {
    e = hipSetDevice(m->root_descs_dev);
    for (void *p : {static_cast<void *>(m->root_descs), static_cast<void *>(m->root_orig),
                    static_cast<void *>(m->root_pack)})
      if (e == hipSuccess && p) e = hipFree(p);
    m->root_descs = m->root_orig = nullptr;
    m->root_pack = nullptr;
    m->root_descs_cap = m->root_orig_cap = m->root_pack_cap = 0;
  }
  if (e == hipSuccess) e = hipSetDevice(m->devices[root]);
  m->root_descs_dev = m->devices[root];
  const uint64_t bytes = sizeof(xsknf_gpu_desc) * n;
  uint64_t cap_d = m->root_descs_cap * sizeof(xsknf_gpu_desc), cap_o = m->root_orig_cap * sizeof(xsknf_gpu_desc);
  if (e == hipSuccess) e = root_buffer(m->root_descs, cap_d, bytes);
  if (e == hipSuccess) e = root_buffer(m->root_orig, cap_o, bytes);
  m->root_descs_cap = cap_d / sizeof(xsknf_gpu_desc);
  m->root_orig_cap = cap_o / sizeof(xsknf_gpu_desc);
  if (e == hipSuccess && n) e = hipMemcpy(m->root_descs, sent, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess && n) e = hipMemcpy(m->root_orig, descs, bytes, hipMemcpyHostToDevice);
  return e;
}

// A shard's device buffers for `span` bytes (+ 16 spare: the kernels' 16-byte
// chunk loads) and `frames` descriptors / verdicts; the spare bytes zeroed.
// The span starts at address `place` mod kPlace, so that a shard of a UMEM's
// span keeps the placement its frames had on the root (the channels a frame's
// sectors fall on follow the address: config 4's 64-B frames at 2 KiB strides).
constexpr uint64_t kPlace = 4096;
hipError_t shard_buffers(Shard &s, uint64_t span, uint64_t frames, uint64_t place) {
  hipError_t e = hipSetDevice(s.device);
  const uint64_t need = span + 16 + kPlace;
  if (e == hipSuccess && need > s.umem_cap) {
    if (s.umem_alloc) (void)hipFree(s.umem_alloc);
    s.umem_alloc = s.umem = nullptr;
    s.umem_cap = 0;
    e = hipMalloc(&s.umem_alloc, need);
    if (e == hipSuccess) s.umem_cap = need;
  }
  if (e == hipSuccess) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(s.umem_alloc);
    s.umem = s.umem_alloc + ((place - a) & (kPlace - 1));
  }
  if (e == hipSuccess && frames > s.frames_cap) {
    if (s.descs) (void)hipFree(s.descs);
    if (s.verdicts) (void)hipFree(s.verdicts);
    s.descs = nullptr;
    s.verdicts = nullptr;
    s.frames_cap = 0;
    e = hipMalloc(&s.descs, sizeof(xsknf_gpu_desc) * (frames ? frames : 1));
    if (e == hipSuccess) e = hipMalloc(&s.verdicts, sizeof(int32_t) * (frames ? frames : 1));
    if (e == hipSuccess) s.frames_cap = frames;
  }
  if (e == hipSuccess) e = hipMemsetAsync(s.umem + span, 0, 16, s.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
  return e;
}

// One grouped set of point-to-point moves, in kP2PPiece pieces: each
// (src on devices[from], dst on devices[to], bytes) as ncclSend on `from`'s
// communicator / stream and ncclRecv on `to`'s.
struct Move {
  const uint8_t *src;
  uint8_t *dst;
  uint64_t bytes;
  int from, to;
};

int grouped_moves(xsknf_gpu_multi *m, const std::vector<Move> &moves, const char *what) {
  ncclResult_t r = ncclGroupStart();
  for (const Move &mv : moves)
    for (uint64_t o = 0; o < mv.bytes && r == ncclSuccess; o += kP2PPiece) {
      const size_t len = mv.bytes - o < kP2PPiece ? mv.bytes - o : kP2PPiece;
      r = ncclSend(mv.src + o, len, ncclUint8, mv.to, m->comms[mv.from], m->sh[mv.from].stream);
      if (r == ncclSuccess) r = ncclRecv(mv.dst + o, len, ncclUint8, mv.from, m->comms[mv.to], m->sh[mv.to].stream);
    }
  const ncclResult_t r2 = ncclGroupEnd();
  if (r != ncclSuccess) return nccl_fail(r, what);
  if (r2 != ncclSuccess) return nccl_fail(r2, what);
  for (Shard &s : m->sh) {
    hipError_t e = hipSetDevice(s.device);
    if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
    if (e != hipSuccess) return hip_fail(e, what);
  }
  return 0;
}

}  // namespace

extern "C" {

int xsknf_gpu_multi_create(struct xsknf_gpu_multi **out, const int *devices, int ndev) {
  if (!out || ndev < 1 || ndev > 64) return -EINVAL;
  *out = nullptr;
  int count = 0;
  const int rc = xsknf_gpu_device_count(&count);
  if (rc) return rc;
  std::vector<int> devs(ndev);
  for (int k = 0; k < ndev; ++k) {
    devs[k] = devices ? devices[k] : k;
    if (devs[k] < 0 || devs[k] >= count) return -EINVAL;
    for (int j = 0; j < k; ++j)
      if (devs[j] == devs[k]) return -EINVAL;   // one communicator rank per device
  }
  xsknf_gpu_multi *m = new (std::nothrow) xsknf_gpu_multi;
  if (!m) return -ENOMEM;
  m->ndev = ndev;
  m->devices = devs;
  m->comms.assign(ndev, nullptr);
  m->sh.resize(ndev);
  ncclResult_t r = ncclCommInitAll(m->comms.data(), ndev, devs.data());
  if (r != ncclSuccess) {
    delete m;
    return nccl_fail(r, "ncclCommInitAll");
  }
  for (int k = 0; k < ndev; ++k) {
    Shard &s = m->sh[k];
    s.device = devs[k];
    hipError_t e = hipSetDevice(s.device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&s.e0);
    if (e == hipSuccess) e = hipEventCreate(&s.e1);
    if (e == hipSuccess) e = hipMalloc(&s.counters, sizeof(unsigned long long) * XSKNF_GPU_MULTI_COUNTERS);
    if (e != hipSuccess) {
      xsknf_gpu_multi_destroy(m);
      return hip_fail(e, "multi device setup");
    }
  }
  *out = m;
  return 0;
}

int xsknf_gpu_multi_scatter(struct xsknf_gpu_multi *m, int root, const uint8_t *umem, uint64_t umem_size,
                            const struct xsknf_gpu_desc *descs, uint64_t n, double *seconds) {
  if (!m || root < 0 || root >= m->ndev || (n && (!umem || !descs))) return -EINVAL;
  const int N = m->ndev;
  std::vector<uint64_t> bounds(N + 1), spans(2 * N);
  int rc = xsknf_gpu_shard_plan(descs, n, umem_size, static_cast<uint32_t>(N), bounds.data(), spans.data());
  if (rc) return rc;
  // the rebased descriptors of every shard (each relative to its own span),
  // staged on the root device in global order
  std::vector<xsknf_gpu_desc> rebased(n);
  for (int k = 0; k < N; ++k)
    xsknf_gpu_shard_rebase(descs + bounds[k], bounds[k + 1] - bounds[k], spans[2 * k], umem_size,
                           rebased.data() + bounds[k]);
  hipError_t e = stage_root(m, root, descs, rebased.data(), n);
  if (e != hipSuccess) return hip_fail(e, "multi scatter: root descriptors");
  for (int k = 0; k < N; ++k) {
    Shard &s = m->sh[k];
    s.lo = bounds[k];
    s.hi = bounds[k + 1];
    s.b0 = spans[2 * k];
    s.b1 = spans[2 * k + 1];
    s.bytes = 0;
    for (uint64_t f = s.lo; f < s.hi; ++f) s.bytes += descs[f].len;
    e = shard_buffers(s, s.b1 - s.b0, s.hi - s.lo, reinterpret_cast<uintptr_t>(umem) + s.b0);
    if (e != hipSuccess) return hip_fail(e, "multi scatter: shard buffers");
  }
  // every shard at once: the root sends each its span and descriptors, every
  // device receives its own (the root's to itself), one group
  const double t0 = now_s();
  std::vector<Move> moves;
  for (int k = 0; k < N; ++k) {
    Shard &s = m->sh[k];
    moves.push_back({umem + s.b0, s.umem, s.b1 - s.b0, root, k});
    moves.push_back({reinterpret_cast<const uint8_t *>(m->root_descs + s.lo), reinterpret_cast<uint8_t *>(s.descs),
                     sizeof(xsknf_gpu_desc) * (s.hi - s.lo), root, k});
  }
  rc = grouped_moves(m, moves, "multi scatter: ncclSend / ncclRecv");
  if (rc) return rc;
  if (seconds) *seconds = now_s() - t0;
  m->root = root;
  m->n = n;
  m->processed = false;
  m->packed = false;
  return 0;
}

int xsknf_gpu_multi_scatter_packed(struct xsknf_gpu_multi *m, int root, const uint8_t *umem, uint64_t umem_size,
                                   const struct xsknf_gpu_desc *descs, uint64_t n, double *seconds) {
  if (!m || root < 0 || root >= m->ndev || (n && (!umem || !descs))) return -EINVAL;
  const int N = m->ndev;
  std::vector<uint64_t> bounds(N + 1);
  int rc = xsknf_gpu_shard_plan(descs, n, umem_size, static_cast<uint32_t>(N), bounds.data(), nullptr);
  if (rc) return rc;
  std::vector<xsknf_gpu_desc> packed(n);
  std::vector<uint64_t> pk_lo(N), pk_size(N);
  rc = xsknf_gpu_shard_pack_plan(descs, n, reinterpret_cast<uintptr_t>(umem), umem_size, static_cast<uint32_t>(N),
                                 bounds.data(), packed.data(), pk_size.data());
  if (rc) return rc;
  // the root's own shard is packed straight into its shard buffer; the staging
  // buffer holds the others' (at N = 1 nothing is staged, nothing copied)
  uint64_t total = 0;
  for (int k = 0; k < N; ++k) {
    pk_lo[k] = k == root ? 0 : total;
    total += k == root ? 0 : pk_size[k];
  }
  hipError_t e = stage_root(m, root, descs, packed.data(), n);
  if (e == hipSuccess) e = root_buffer(m->root_pack, m->root_pack_cap, total);
  if (e != hipSuccess) return hip_fail(e, "multi packed scatter: root buffers");
  for (int k = 0; k < N; ++k) {
    Shard &s = m->sh[k];
    s.lo = bounds[k];
    s.hi = bounds[k + 1];
    s.b0 = 0;
    s.b1 = pk_size[k];
    s.bytes = 0;
    for (uint64_t f = s.lo; f < s.hi; ++f) s.bytes += descs[f].len;
    e = shard_buffers(s, pk_size[k], s.hi - s.lo, 0);
    if (e != hipSuccess) return hip_fail(e, "multi packed scatter: shard buffers");
  }
  const double t0 = now_s();
  // gather every shard's frames on the root, on the root's stream (its sends
  // follow on the same stream): the root's own into its shard buffer
  Shard &rs = m->sh[root];
  e = hipSetDevice(rs.device);
  for (int k = 0; k < N && e == hipSuccess; ++k) {
    const uint64_t frames = bounds[k + 1] - bounds[k];
    if (!frames) continue;
    const uint64_t want = (frames + 255) / 256;
    const unsigned grid = static_cast<unsigned>(want < 4096 ? want : 4096);
    hipLaunchKernelGGL(pack_frames, dim3(grid), dim3(256), 0, rs.stream, umem, umem_size, m->root_orig + bounds[k],
                       m->root_descs + bounds[k], frames, k == root ? rs.umem : m->root_pack + pk_lo[k]);
    e = hipGetLastError();
  }
  if (e != hipSuccess) return hip_fail(e, "multi packed scatter: pack_frames");
  std::vector<Move> moves;
  for (int k = 0; k < N; ++k) {
    Shard &s = m->sh[k];
    if (k != root) moves.push_back({m->root_pack + pk_lo[k], s.umem, pk_size[k], root, k});
    // (the root's descriptors too, as a send to itself: the same path at N = 1)
    moves.push_back({reinterpret_cast<const uint8_t *>(m->root_descs + s.lo), reinterpret_cast<uint8_t *>(s.descs),
                     sizeof(xsknf_gpu_desc) * (s.hi - s.lo), root, k});
  }
  rc = grouped_moves(m, moves, "multi packed scatter: ncclSend / ncclRecv");
  if (rc) return rc;
  if (seconds) *seconds = now_s() - t0;
  m->root = root;
  m->n = n;
  m->processed = false;
  m->packed = true;
  return 0;
}

int xsknf_gpu_multi_process(struct xsknf_gpu_multi *m, uint32_t ingress_ifindex, const struct xsknf_csum_opts *opts,
                            uint32_t frame_len_max, uint32_t frame_len_mean, float *ms) {
  if (!m || !opts || m->root < 0) return -EINVAL;
  // every device's launches first (all in flight together), then the waits
  for (Shard &s : m->sh) {
    const uint64_t frames = s.hi - s.lo;
    if (frames > UINT32_MAX) return -EINVAL;
    hipError_t e = hipSetDevice(s.device);
    if (e == hipSuccess) e = hipEventRecord(s.e0, s.stream);
    if (e != hipSuccess) return hip_fail(e, "multi process: start");
    const int rc = xsknf_gpu_checksum_batch_lens(s.umem, s.b1 - s.b0, s.descs, static_cast<uint32_t>(frames),
                                                 ingress_ifindex, opts, s.verdicts, frame_len_max, frame_len_mean,
                                                 s.stream);
    if (rc) return rc;
    e = hipEventRecord(s.e1, s.stream);
    if (e != hipSuccess) return hip_fail(e, "multi process: end");
    m->processed = true;
  }
  for (int k = 0; k < m->ndev; ++k) {
    Shard &s = m->sh[k];
    hipError_t e = hipSetDevice(s.device);
    if (e == hipSuccess) e = hipEventSynchronize(s.e1);
    float t = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, s.e0, s.e1);
    if (e != hipSuccess) return hip_fail(e, "multi process: wait");
    if (ms) ms[k] = t;
  }
  return 0;
}

int xsknf_gpu_multi_counters(struct xsknf_gpu_multi *m, uint64_t *out) {
  if (!m || !out || m->root < 0) return -EINVAL;
  // the weighted check sum needs each frame's place in the root's UMEM, which
  // a packed shard no longer holds: after a packed scatter the results come
  // back whole (xsknf_gpu_multi_return) and are checked there
  if (m->packed) return -EOPNOTSUPP;
  for (Shard &s : m->sh) {
    hipError_t e = hipSetDevice(s.device);
    if (e == hipSuccess)
      e = hipMemsetAsync(s.counters, 0, sizeof(unsigned long long) * XSKNF_GPU_MULTI_COUNTERS, s.stream);
    const uint64_t frames = s.hi - s.lo;
    if (e == hipSuccess && frames) {
      const uint64_t want = (frames + 255) / 256;
      const unsigned grid = static_cast<unsigned>(want < 2048 ? want : 2048);
      hipLaunchKernelGGL(shard_counters, dim3(grid), dim3(256), 0, s.stream, s.umem, s.b1 - s.b0, s.descs,
                         s.verdicts, frames, s.b0, s.counters);
      e = hipGetLastError();
    }
    if (e != hipSuccess) return hip_fail(e, "multi counters: launch");
  }
  ncclResult_t r = ncclGroupStart();
  for (int k = 0; k < m->ndev && r == ncclSuccess; ++k)
    r = ncclAllReduce(m->sh[k].counters, m->sh[k].counters, XSKNF_GPU_MULTI_COUNTERS, ncclUint64, ncclSum,
                      m->comms[k], m->sh[k].stream);
  const ncclResult_t r2 = ncclGroupEnd();
  if (r != ncclSuccess) return nccl_fail(r, "multi counters: ncclAllReduce");
  if (r2 != ncclSuccess) return nccl_fail(r2, "multi counters: ncclGroupEnd");
  for (Shard &s : m->sh) {
    hipError_t e = hipSetDevice(s.device);
    if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
    if (e != hipSuccess) return hip_fail(e, "multi counters: wait");
  }
  // every device holds the sum; the root's copy is the answer
  Shard &rs = m->sh[m->root];
  hipError_t e = hipSetDevice(rs.device);
  if (e == hipSuccess)
    e = hipMemcpy(out, rs.counters, sizeof(unsigned long long) * XSKNF_GPU_MULTI_COUNTERS, hipMemcpyDeviceToHost);
  return e == hipSuccess ? 0 : hip_fail(e, "multi counters: copy");
}

int xsknf_gpu_multi_return(struct xsknf_gpu_multi *m, uint32_t ingress_ifindex, const struct xsknf_csum_opts *opts,
                           uint32_t frame_len_max, uint32_t frame_len_mean, uint8_t *umem, int32_t *verdicts, float *ms,
                           double *seconds) {
  if (!m || !opts || m->root < 0 || (m->n && (!umem || !verdicts))) return -EINVAL;
  // the records describe a pass over the frames as the scatter sent them: once
  // _process has rewritten checks in the shards, a second pass is not the same
  // (a frame whose UDP header overlaps its IP addresses, ihl 2 or 3, sums the
  // check it just wrote), so the caller scatters again
  if (m->processed) {
    xsknf_gpu::set_error_text("xsknf_gpu_multi_return: the shards were checksummed in place since the scatter");
    return -EBUSY;
  }
  xsknf_gpu_launch_cfg cfg;
  int rc = xsknf_gpu_launch_cfg_for_lens(frame_len_max, frame_len_mean, &cfg);
  if (rc) return rc;
  cfg.fused_stores = 3;   // records only: the shard is read, each changed check comes back as a record
  const double t0 = now_s();
  for (Shard &s : m->sh) {
    const uint64_t frames = s.hi - s.lo;
    if (frames > UINT32_MAX) return -EINVAL;
    hipError_t e = hipSetDevice(s.device);
    if (e == hipSuccess) e = hipEventRecord(s.e0, s.stream);
    if (e != hipSuccess) return hip_fail(e, "multi return: start");
    rc = xsknf_gpu_checksum_batch_cfg(s.umem, s.b1 - s.b0, s.descs, static_cast<uint32_t>(frames), ingress_ifindex,
                                      opts, s.verdicts, &cfg, s.stream);
    if (rc) return rc;
    e = hipEventRecord(s.e1, s.stream);
    if (e != hipSuccess) return hip_fail(e, "multi return: end");
  }
  // every device's records to the root, into the caller's verdict array, one group
  std::vector<Move> moves;
  for (int k = 0; k < m->ndev; ++k) {
    Shard &s = m->sh[k];
    moves.push_back({reinterpret_cast<const uint8_t *>(s.verdicts), reinterpret_cast<uint8_t *>(verdicts + s.lo),
                     sizeof(int32_t) * (s.hi - s.lo), k, m->root});
  }
  rc = grouped_moves(m, moves, "multi return: ncclSend / ncclRecv");
  if (rc) return rc;
  for (int k = 0; k < m->ndev && ms; ++k) {
    hipError_t e = hipSetDevice(m->sh[k].device);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms[k], m->sh[k].e0, m->sh[k].e1);
    if (e != hipSuccess) return hip_fail(e, "multi return: events");
  }
  // the root applies them to its UMEM, with the descriptors the caller scattered
  Shard &rs = m->sh[m->root];
  hipError_t e = hipSetDevice(rs.device);
  if (e == hipSuccess && m->n) {
    const int32_t fwd = opts->action == XSKNF_CSUM_ACTION_REDIRECT
                            ? static_cast<int32_t>((ingress_ifindex + 1u) % opts->num_interfaces) : -1;
    const uint64_t want = (m->n + 255) / 256;
    const unsigned grid = static_cast<unsigned>(want < 4096 ? want : 4096);
    hipLaunchKernelGGL(apply_records, dim3(grid), dim3(256), 0, rs.stream, umem, m->root_orig, verdicts, m->n, fwd);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(rs.stream);
  }
  if (e != hipSuccess) return hip_fail(e, "multi return: apply_records");
  if (seconds) *seconds = now_s() - t0;
  return 0;
}

int xsknf_gpu_multi_shard_info(const struct xsknf_gpu_multi *m, int k, struct xsknf_gpu_shard_info *info) {
  if (!m || !info || k < 0 || k >= m->ndev) return -EINVAL;
  const Shard &s = m->sh[k];
  info->device = s.device;
  info->flags = m->packed ? XSKNF_GPU_SHARD_PACKED : 0;
  info->frame_lo = s.lo;
  info->frame_hi = s.hi;
  info->span_lo = s.b0;   // (packed: 0 .. the shard's packed bytes)
  info->span_hi = s.b1;
  info->frame_bytes = s.bytes;
  info->umem = s.umem;
  info->descs = s.descs;
  info->verdicts = s.verdicts;
  return 0;
}

int xsknf_gpu_multi_fetch(const struct xsknf_gpu_multi *m, int k, uint8_t *umem_out, struct xsknf_gpu_desc *descs_out,
                          int32_t *verdicts_out) {
  if (!m || k < 0 || k >= m->ndev || m->root < 0) return -EINVAL;
  const Shard &s = m->sh[k];
  hipError_t e = hipSetDevice(s.device);
  if (e == hipSuccess && umem_out && s.b1 > s.b0)
    e = hipMemcpy(umem_out, s.umem, s.b1 - s.b0, hipMemcpyDeviceToHost);
  if (e == hipSuccess && descs_out && s.hi > s.lo)
    e = hipMemcpy(descs_out, s.descs, sizeof(xsknf_gpu_desc) * (s.hi - s.lo), hipMemcpyDeviceToHost);
  if (e == hipSuccess && verdicts_out && s.hi > s.lo)
    e = hipMemcpy(verdicts_out, s.verdicts, sizeof(int32_t) * (s.hi - s.lo), hipMemcpyDeviceToHost);
  return e == hipSuccess ? 0 : hip_fail(e, "multi fetch");
}

int xsknf_gpu_multi_destroy(struct xsknf_gpu_multi *m) {
  if (!m) return -EINVAL;
  for (Shard &s : m->sh) {
    if (hipSetDevice(s.device) != hipSuccess) continue;
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.umem_alloc) (void)hipFree(s.umem_alloc);
    if (s.descs) (void)hipFree(s.descs);
    if (s.verdicts) (void)hipFree(s.verdicts);
    if (s.counters) (void)hipFree(s.counters);
    if (s.e0) (void)hipEventDestroy(s.e0);
    if (s.e1) (void)hipEventDestroy(s.e1);
    if (s.stream) (void)hipStreamDestroy(s.stream);
  }
  if (m->root_descs_dev >= 0 && hipSetDevice(m->root_descs_dev) == hipSuccess) {
    if (m->root_descs) (void)hipFree(m->root_descs);
    if (m->root_orig) (void)hipFree(m->root_orig);
    if (m->root_pack) (void)hipFree(m->root_pack);
  }
  for (ncclComm_t c : m->comms)
    if (c) (void)ncclCommDestroy(c);
  delete m;
  return 0;
}

}  // extern "C"
