// host_path.hip -- the batch hook with the UMEM in host memory.
//
// In the reference, an AF_XDP worker (src/xsknf.c:716-742) peeks up to
// batch_size rx descriptors and calls xsknf_packet_processor() on each frame,
// in place in the worker's mmap'd UMEM (src/xsknf.c:654-672, :958/:975), batch
// after batch.  This context is what such a worker holds to run that loop on
// the GPU instead: host UMEM registered once, then batches submitted with the
// descriptors and verdicts in host arrays.
//
// Up to kSlots (5) pieces are in flight per context: each SLOT has its own HIP
// stream, pinned descriptor / record arrays and staging buffers, so the copies
// and kernel of one batch overlap another's, and the host's share of a batch
// (copy plan, writing the checks) overlaps the device's share of the others.
// Five = four batches out plus the one being submitted: past four out a
// launched batch's submit is CPU-bound (launch + event, tools/ctx_depth.sh), so
// a deeper two-phase hook (up to XSKNF_MAX_HOOK_DEPTH = 8, include/xsknf.h)
// waits in submit for its oldest piece; the RESIDENT ring's eight entries keep
// eight out.  xsknf_gpu_ctx_submit() /
// _wait() expose the pipeline; the synchronous xsknf_gpu_ctx_process_batch()
// cuts a large batch into pieces of kPiece frames and runs them through the
// same slots.
//
// ZEROCOPY: the UMEM is pinned and mapped into the device address space; the
//   kernel reads the frames and writes the check bytes over PCIe, in place.
//   Checks are written in-line (2-byte stores: host memory has byte enables).
// STAGED: only the bytes of the batch's frames cross PCIe, into a device
//   mirror of the UMEM, by the cheapest of
//     - up to kMaxDmaRuns DMA copies of merged runs (frames closer than
//       kMergeGap share a run): a contiguous or nearly contiguous batch;
//     - one 2-D DMA copy (row = frame, pitch = the constant stride): aligned
//       chunks in rx order, without the gaps between frames;
//   and summed in HBM with every check deferred: only the 4-byte per-frame
//   records come back and the host writes each frame's 2 check bytes.  A
//   scattered batch (the fill ring hands frames back in recycled order, so a
//   64-frame batch can span the whole UMEM) is instead processed exactly as
//   ZEROCOPY does, in the mapped UMEM over PCIe (measured at 1M frames: a CPU
//   gather into a pinned staging buffer moved 8 GB/s, CPU-bound; the mapped
//   reads with host-applied checks 23 GB/s, host-bound; in place 41 GB/s).
//   Copying frames back would overwrite frames outside the batch that the
//   kernel / NIC may be filling concurrently (fill-ring frames), so it never
//   does; the mirror is only read by the kernels, so batches in flight may
//   share it (their frames are distinct, and a run's gap bytes are the host's
//   own bytes).
//
// RESIDENT: ZEROCOPY, but no batch launches a kernel: ONE resident kernel per
//   device (checksummer.hip resident_kernel, host side ResService below) takes
//   the batches of every RESIDENT context on the device from each context's
//   ring, in entries of up to kResFrames frames, a group of one or four 4-wave
//   blocks per entry, so several batches (or the pieces of a larger one) are
//   processed at once.  Each ring's headers and descriptors sit in device
//   memory the host writes through the BAR (large-BAR devices) or in mapped
//   host memory; completion flags and verdicts in host memory.  submit()
//   writes the descriptors and the entry's header and publishes its sequence
//   number; wait() spins on the entry's `done`.  The kernel exits when every
//   ring is idle, when old, or when a ring joins or leaves, and the next
//   submit() / wait() of any context relaunches it from each entry's first
//   batch not done, so a worker pays a launch only after a pause in the
//   device's traffic.  No batch takes the launch path, and the device's
//   RESIDENT contexts share one stream (one hardware queue), however many
//   workers there are (up to kResMaxRings rings per device).
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <immintrin.h>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/xsknf_gpu.h"
#include "checksummer_internal.h"

namespace {

constexpr int kSlots = 5;   // pieces in flight per context: 4 batches out + the one submitted
constexpr uint32_t kPiece = 65536;          // frames per slot submission of process_batch
constexpr uint64_t kMergeGap = 256;         // frames closer than this share one DMA run
constexpr size_t kMaxDmaRuns = 8;           // more runs than this (and no 2-D shape): mapped reads
constexpr size_t kSortMax = 4096;           // a larger batch out of address order is not sorted

struct Run {
  uint64_t off, len;
};

struct Slot {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  xsknf_gpu_desc *descs = nullptr;          // pinned; the kernel reads them mapped
  xsknf_gpu_desc *descs_mapped = nullptr;
  int32_t *rec = nullptr;                   // pinned; the kernel writes them mapped
  int32_t *rec_mapped = nullptr;
  std::vector<uint64_t> offs;               // frame offsets in the host UMEM (STAGED)
  std::vector<uint32_t> order;
  std::vector<Run> runs;
  // the piece in flight
  bool busy = false;
  uint64_t seq = 0;
  uint32_t n = 0;
  int32_t *out = nullptr;
  int32_t fwd = -1;
  bool host_checks = false;                 // records to apply on the host (STAGED, HBM mirror)
};

}  // namespace

struct RingEntry {
  bool busy = false;
  uint64_t ticket = 0;                      // the context's sequence number (xsknf_gpu_ctx_wait)
  uint64_t rseq = 0;                        // the ring's sequence number (ResSlot::seq)
  uint32_t n = 0;
  int32_t *out = nullptr;
};

struct xsknf_gpu_ctx {
  int device = 0;
  int path = XSKNF_GPU_PATH_ZEROCOPY;
  uint32_t max_batch = 0;
  uint32_t slot_frames = 0;                 // min(max_batch, kPiece)
  uint32_t hint = 0;
  uint8_t *umem_host = nullptr;
  uint64_t umem_size = 0;
  uint8_t *umem_dev = nullptr;              // mapped host pointer (ZEROCOPY) or device mirror (STAGED)
  uint8_t *umem_mapped = nullptr;           // the host UMEM mapped into the device (both paths)
  bool registered = false;
  Slot slot[kSlots];
  int next = 0;                             // slot the next piece goes to (round robin)
  uint64_t seq = 0;                         // pieces submitted
  xsknf_gpu_ctx_stats stats = {};
  // RESIDENT: the context's ring; the kernel and its launches belong to the
  // device's ResService
  xsknf_gpu::ResIn *rin = nullptr;          // headers + descriptors: host memory, or device memory (BAR)
  xsknf_gpu_desc *rdescs = nullptr;
  bool rbar = false;                        // rin / rdescs are device memory written through the BAR
  xsknf_gpu::ResOut *rout = nullptr;        // completion flags + verdicts: host memory
  int32_t *rverd = nullptr;
  xsknf_gpu::ResRing rring = {};            // the kernel's view, filled at creation / registration
  int ring_idx = -1;                        // index in the service's ring table (registered)
  std::atomic<uint64_t> pub[xsknf_gpu::kResSlots] = {};   // last ring number published per entry (relaunch)
  uint64_t rseq = 0;                        // ring entries published
  int failed = 0;                           // -ETIMEDOUT once a batch never completed: every later
                                            // call returns it at once
  RingEntry ring[xsknf_gpu::kResSlots];
};

namespace {

int fail(hipError_t e, const char *where) {
  if (e == hipErrorNoDevice) return xsknf_gpu::set_device_error(e, 0, where);
  xsknf_gpu::set_error(e, where);
  return -EIO;
}

uint64_t umem_offset(uint64_t addr) {
  return (addr & XSKNF_GPU_UNALIGNED_BUF_ADDR_MASK) + (addr >> XSKNF_GPU_UNALIGNED_BUF_OFFSET_SHIFT);
}

// ---- RESIDENT: the device's one resident kernel (ResService) --------------------
//
// Every RESIDENT context of a device registers its ring here; one kernel on
// one stream serves them all (checksummer.hip resident_kernel), so the number
// of workers does not multiply hardware queues or kernels.  The table of rings,
// the block map and each entry's first sequence number go to the device
// (ResLaunch) before each launch.  Whoever finds the kernel gone (its last
// block wrote the launch's epoch to ctl->exited) relaunches it under the
// service's mutex; adding or removing a ring stops the kernel (the stop word),
// changes the table and relaunches.  A ring's group (blocks per entry) is fixed
// for its life -- its host side waits for that many done flags per batch --
// while the entries per block are chosen per launch to fit the grid cap.

// Short lives: a launch on another stream that shares the resident kernel's
// hardware queue waits behind it, so the kernel leaves every few ms (a relaunch
// costs one launch, ~0.5 % of a busy ring's time) and after 1 ms without a
// batch on any ring.
constexpr uint64_t kResIdleTicks = 100000;      // 1 ms without a batch (100 MHz wall clock)
constexpr uint64_t kResLifeTicks = 400000;      // 4 ms

struct ResService {
  std::mutex mu;
  bool init = false;
  int device = -1;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;                 // recorded after each launch
  xsknf_gpu::ResLaunch *L = nullptr;         // device memory
  xsknf_gpu::ResLaunch *Lh = nullptr;        // pinned: what the next launch copies to L
  xsknf_gpu::ResCtl *ctl = nullptr;          // host memory, mapped
  xsknf_gpu::ResCtl *ctl_dev = nullptr;
  uint64_t *stop = nullptr;                  // the stop word: ResStop in device memory (BAR), or ctl->stop
  uint64_t *stop_dev = nullptr;
  bool stop_bar = false;
  std::atomic<bool> launched{false};
  std::atomic<uint64_t> epoch{0};            // the latest launch's number
  xsknf_gpu_ctx *rings[xsknf_gpu::kResMaxRings] = {};
  uint32_t cap = 0;                          // blocks the kernel may have
  std::atomic<uint64_t> launches{0};
};
ResService g_svc[64];

// Is the kernel of the latest launch still there (no block has reported its exit)?
bool svc_running(ResService &s) {
  return s.launched.load(std::memory_order_acquire) &&
         __atomic_load_n(&s.ctl->exited, __ATOMIC_ACQUIRE) != s.epoch.load(std::memory_order_acquire);
}

int svc_init_locked(ResService &s, int device) {
  using namespace xsknf_gpu;
  if (s.init) return 0;
  hipError_t e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipMalloc(&s.L, sizeof(ResLaunch));
  if (e == hipSuccess) e = hipHostMalloc(&s.Lh, sizeof(ResLaunch), hipHostMallocDefault);
  if (e == hipSuccess) e = hipHostMalloc(&s.ctl, sizeof(ResCtl), hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&s.ctl_dev), s.ctl, 0);
  if (e != hipSuccess) {
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    if (s.L) (void)hipFree(s.L);
    if (s.Lh) (void)hipHostFree(s.Lh);
    if (s.ctl) (void)hipHostFree(s.ctl);
    s.done = nullptr, s.stream = nullptr, s.L = nullptr, s.Lh = nullptr, s.ctl = nullptr;
    return fail(e, "resident service");
  }
  memset(s.ctl, 0, sizeof(ResCtl));
  memset(s.Lh, 0, sizeof(ResLaunch));
  // the stop word where the blocks' polls stay on the device (large BAR), as the rings' headers
  s.stop = &s.ctl->stop;
  s.stop_dev = &s.ctl_dev->stop;
  int large_bar = 0;
  void *p = nullptr;
  if (hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, device) == hipSuccess && large_bar &&
      hipExtMallocWithFlags(&p, sizeof(ResStop), hipDeviceMallocFinegrained) == hipSuccess) {
    s.stop = s.stop_dev = static_cast<uint64_t *>(p);
    s.stop_bar = true;
    *s.stop = 0;
    _mm_sfence();
  } else {
    (void)hipGetLastError();
  }
  // at most half the blocks the device holds of this kernel: the resident
  // kernel must never fill the CUs other work needs
  const int per_cu = resident_blocks_per_cu();
  const uint32_t cap = static_cast<uint32_t>(std::max(1, per_cu) * device_cu_count() / 2);
  s.cap = std::max<uint32_t>(kResSlots, std::min(cap, kResMaxBlocks));
  s.device = device;
  s.init = true;
  return 0;
}

void svc_set_stop(ResService &s, uint64_t v) {
  __atomic_store_n(s.stop, v, __ATOMIC_RELEASE);
  if (s.stop_bar) _mm_sfence();   // out of the write-combining buffer
}

// Stop the kernel (if there) and wait for it to leave.
int svc_stop_locked(ResService &s) {
  if (!s.launched.load()) return 0;
  svc_set_stop(s, 1);
  const hipError_t e = hipEventSynchronize(s.done);
  s.launched.store(false, std::memory_order_release);
  if (e != hipSuccess) return fail(e, "resident kernel");
  return 0;
}

// The first sequence number block (entry b, g) of ring c takes: the entry's
// latest batch if published and not done by that block, else the entry's next
// number (a block that left has finished every batch it took).
uint64_t ring_start(const xsknf_gpu_ctx *c, uint32_t b, uint32_t g) {
  using namespace xsknf_gpu;
  const uint64_t p = c->pub[b].load(std::memory_order_acquire);
  if (p == 0) return b ? b : kResSlots;   // the entry's first number (they start at 1)
  if (__atomic_load_n(&c->rout[b * kResGroup + g].done, __ATOMIC_ACQUIRE) == p) return p + kResSlots;
  return p;
}

// Launch the kernel over every registered ring (the previous launch, if any,
// is over: its exit was reported, or it was stopped).
int svc_launch_locked(ResService &s) {
  using namespace xsknf_gpu;
  if (s.launched.load()) {
    const hipError_t e = hipEventSynchronize(s.done);   // its last block has reported; the grid ends now
    s.launched.store(false, std::memory_order_release);
    if (e != hipSuccess) return fail(e, "resident kernel");
  }
  uint32_t need = 0, rings = 0;
  for (const xsknf_gpu_ctx *c : s.rings)
    if (c) need += kResSlots * c->rring.group, ++rings;
  if (!rings) return 0;
  uint32_t E = 1;
  while (E < kResSlots && need / E > s.cap) E *= 2;
  const uint32_t stride = kResSlots / E;
  ResLaunch &h = *s.Lh;
  h.act = 0;
  h.exits = 0;
  uint32_t blk = 0;
  for (uint32_t r = 0; r < kResMaxRings; ++r) {
    const xsknf_gpu_ctx *c = s.rings[r];
    if (!c) continue;
    h.ring[r] = c->rring;
    // entry-minor order: blocks are dealt to the XCDs round robin, so a ring's
    // entries' first blocks (the only ones a batch of <= 64 frames uses) land
    // on consecutive XCDs
    for (uint32_t g = 0; g < c->rring.group; ++g)
      for (uint32_t b = 0; b < stride; ++b) h.block[blk++] = r << 16 | g << 8 | b;
    for (uint32_t b = 0; b < kResSlots; ++b)
      for (uint32_t g = 0; g < c->rring.group; ++g) h.start[r][b * kResGroup + g] = ring_start(c, b, g);
  }
  hipError_t e = hipMemcpyAsync(s.L, s.Lh, sizeof(ResLaunch), hipMemcpyHostToDevice, s.stream);
  if (e != hipSuccess) return fail(e, "hipMemcpyAsync(resident table)");
  svc_set_stop(s, 0);
  ResArgs ra = {};
  ra.L = s.L;
  ra.rings = s.L->ring;
  ra.ctl = s.ctl_dev;
  ra.stop = s.stop_dev;
  ra.epoch = s.epoch.load() + 1;
  ra.blocks = blk;
  ra.entries_per_block = E;
  ra.idle_ticks = kResIdleTicks;
  ra.life_ticks = kResLifeTicks;
  int rc = launch_resident(ra, s.stream);
  if (rc) return rc;
  e = hipEventRecord(s.done, s.stream);
  if (e != hipSuccess) return fail(e, "hipEventRecord(resident)");
  s.epoch.store(ra.epoch, std::memory_order_release);
  s.launched.store(true, std::memory_order_release);
  s.launches += 1;
  return 0;
}

// Make sure the kernel is there (cheap when it is: two loads).
int svc_ensure(xsknf_gpu_ctx *c) {
  ResService &s = g_svc[c->device];
  if (svc_running(s)) return 0;
  std::lock_guard<std::mutex> lk(s.mu);
  if (svc_running(s)) return 0;
  return svc_launch_locked(s);
}

// Register a context's ring (at UMEM registration) and relaunch with it.
int svc_add(xsknf_gpu_ctx *c) {
  using namespace xsknf_gpu;
  if (c->device < 0 || c->device >= 64) return -EINVAL;
  ResService &s = g_svc[c->device];
  std::lock_guard<std::mutex> lk(s.mu);
  int rc = svc_init_locked(s, c->device);
  if (rc) return rc;
  int idx = -1;
  uint32_t min_blocks = c->rring.group;     // at 8 entries per block
  for (uint32_t r = 0; r < kResMaxRings; ++r) {
    if (!s.rings[r] && idx < 0) idx = static_cast<int>(r);
    if (s.rings[r]) min_blocks += s.rings[r]->rring.group;
  }
  if (idx < 0 || min_blocks > s.cap) {
    set_error_text("resident service: no room for another ring on this device");
    return -ENOSPC;
  }
  rc = svc_stop_locked(s);
  if (rc) return rc;
  s.rings[idx] = c;
  c->ring_idx = idx;
  return svc_launch_locked(s);
}

// Take a context's ring out (every batch of it complete, or the context
// failed); the other rings go on in a new launch.
void svc_remove(xsknf_gpu_ctx *c) {
  if (c->ring_idx < 0) return;
  ResService &s = g_svc[c->device];
  std::lock_guard<std::mutex> lk(s.mu);
  (void)svc_stop_locked(s);
  s.rings[c->ring_idx] = nullptr;
  c->ring_idx = -1;
  (void)svc_launch_locked(s);
}

// A context whose batch never completed: stop the kernel, give it a bounded
// time to leave (its polls and batches are bounded by the clock), and take the
// ring out of the table, so that no later launch -- made for the other rings --
// reads this ring's entries again and writes into frames the caller may
// recycle after the error.
void svc_fail(xsknf_gpu_ctx *c) {
  ResService &s = g_svc[c->device];
  std::lock_guard<std::mutex> lk(s.mu);
  svc_set_stop(s, 1);
  for (int i = 0; i < 1000 && s.launched.load() && hipEventQuery(s.done) == hipErrorNotReady; ++i)
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  if (c->ring_idx >= 0) s.rings[c->ring_idx] = nullptr;
  c->ring_idx = -1;
  // the other rings: their next submit or wait relaunches the kernel (svc_ensure)
}

void release(xsknf_gpu_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  for (Slot &s : c->slot) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.descs) (void)hipHostFree(s.descs);
    if (s.rec) (void)hipHostFree(s.rec);
    if (s.stream) (void)hipStreamDestroy(s.stream);
  }
  svc_remove(c);   // the kernel no longer reads this ring
  if (c->rin) (void)(c->rbar ? hipFree(c->rin) : hipHostFree(c->rin));   // rdescs lies in the same block
  if (c->rout) (void)hipHostFree(c->rout);
  if (c->rverd) (void)hipHostFree(c->rverd);
  if (c->registered) (void)hipHostUnregister(c->umem_host);
  if (c->path == XSKNF_GPU_PATH_STAGED && c->umem_dev) (void)hipFree(c->umem_dev);
  delete c;
}

// Finish the slot's piece: wait for its stream, then (STAGED) write the checks
// into the host UMEM from the records, and hand out the verdicts.
int complete(xsknf_gpu_ctx *c, Slot &s) {
  using namespace xsknf_gpu;
  if (!s.busy) return 0;
  s.busy = false;
  hipError_t e = hipEventSynchronize(s.done);
  if (e != hipSuccess) return fail(e, "hipEventSynchronize");
  if (s.host_checks) {
    // checksummer_user.c:108 on the host: the 2 check bytes of every summed frame
    for (uint32_t i = 0; i < s.n; ++i) {
      const uint32_t r = static_cast<uint32_t>(s.rec[i]);
      if ((r & kRecTagMask) == kRecTag) {
        uint8_t *p = c->umem_host + s.offs[i] + ((r >> 16) & 0x7f) + 6;
        p[0] = static_cast<uint8_t>(r);
        p[1] = static_cast<uint8_t>(r >> 8);
        s.out[i] = s.fwd;
      } else {
        s.out[i] = static_cast<int32_t>(r);
      }
    }
  } else {
    memcpy(s.out, s.rec, sizeof(int32_t) * s.n);
  }
  c->stats.batches += 1;
  c->stats.frames += s.n;
  c->stats.bytes_d2h += sizeof(int32_t) * s.n;
  return 0;
}

// ---- RESIDENT: the context's ring -------------------------------------------------

// Wait for a ring entry's batch (relaunching the kernel if it left before
// reaching it) and hand out its verdicts.
int ring_complete(xsknf_gpu_ctx *c, RingEntry &r) {
  using namespace xsknf_gpu;
  if (!r.busy) return 0;
  if (c->failed) return c->failed;
  const xsknf_gpu::ResOut *h = c->rout + (r.rseq % kResSlots) * kResGroup;
  const uint32_t used = res_used_blocks(r.n, c->rring.group);   // the blocks with frames publish done
  const auto all_done = [h, &r, used] {
    for (uint32_t g = 0; g < used; ++g)
      if (__atomic_load_n(&h[g].done, __ATOMIC_ACQUIRE) != r.rseq) return false;
    return true;
  };
  ResService &s = g_svc[c->device];
  double t0 = 0;
  for (uint32_t spin = 1; !all_done(); ++spin) {
    __builtin_ia32_pause();
    if ((spin & 1023) == 0) {
      if (!svc_running(s)) {
        if (all_done()) break;
        const int rc = svc_ensure(c);   // the kernel left before this entry
        if (rc) return rc;
      }
      if ((spin & 65535) == 0) {
        timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        const double t = ts.tv_sec + 1e-9 * ts.tv_nsec;
        if (!t0) t0 = t;
        const hipError_t q = s.done ? hipEventQuery(s.done) : hipSuccess;
        if (q != hipSuccess && q != hipErrorNotReady) return fail(q, "resident kernel");
        if (t - t0 > 10.0) {
          // every launch lives at most a few ms and is relaunched on demand:
          // something is wrong.  Stop the kernel and take the ring out of its
          // table (svc_fail), and fail every later call of this context at once.
          svc_fail(c);
          c->failed = -ETIMEDOUT;
          xsknf_gpu::set_error_text("resident kernel: no completion within 10 s");
          return -ETIMEDOUT;
        }
      }
    }
  }
  memcpy(r.out, c->rverd + static_cast<size_t>(r.rseq % kResSlots) * kResFrames, sizeof(int32_t) * r.n);
  r.busy = false;
  c->stats.batches += 1;
  c->stats.frames += r.n;
  c->stats.bytes_d2h += sizeof(int32_t) * r.n;
  c->stats.resident_batches += 1;
  return 0;
}

int ring_submit(xsknf_gpu_ctx *c, const xsknf_gpu_desc *descs, uint32_t n, uint32_t ingress_ifindex,
                const xsknf_csum_opts *opts, int32_t *verdicts) {
  using namespace xsknf_gpu;
  if (c->failed) return c->failed;
  KernelArgs a;
  int rc = prepare(a, c->umem_dev, c->umem_size, c->rring.descs, n, ingress_ifindex, opts, c->rring.verdicts);
  if (rc != 0) return rc < 0 ? rc : 0;
  const uint64_t r = c->rseq + 1;
  const uint32_t k = static_cast<uint32_t>(r % kResSlots);
  RingEntry &e = c->ring[k];
  rc = ring_complete(c, e);   // the entry's previous batch
  if (rc) return rc;
  memcpy(c->rdescs + static_cast<size_t>(k) * kResFrames, descs, sizeof(xsknf_gpu_desc) * n);
  ResIn &h = c->rin[k];
  h.fwd = a.fwd_verdict;
  h.payload_mult = a.payload_mult;
  // a BAR mapping is write-combining: the descriptors and header must be out
  // before the doorbell, and the doorbell out of the buffer
  if (c->rbar) _mm_sfence();
  __atomic_store_n(&h.seqn, r << 16 | n, __ATOMIC_RELEASE);
  if (c->rbar) _mm_sfence();
  c->pub[k].store(r, std::memory_order_release);
  c->rseq = r;
  c->stats.bytes_h2d += sizeof(xsknf_gpu_desc) * n;
  e.busy = true;
  e.ticket = ++c->seq;
  e.rseq = r;
  e.n = n;
  e.out = verdicts;
  return svc_ensure(c);
}

// Complete every piece / ring batch with a sequence number <= upto, oldest first.
int complete_upto(xsknf_gpu_ctx *c, uint64_t upto) {
  for (;;) {
    Slot *old = nullptr;
    RingEntry *rold = nullptr;
    for (Slot &s : c->slot)
      if (s.busy && s.seq <= upto && (!old || s.seq < old->seq)) old = &s;
    for (RingEntry &r : c->ring)
      if (r.busy && r.ticket <= upto && (!rold || r.ticket < rold->ticket)) rold = &r;
    if (!old && !rold) return 0;
    const int rc = (rold && (!old || rold->ticket < old->seq)) ? ring_complete(c, *rold) : complete(c, *old);
    if (rc) return rc;
  }
}

// STAGED: move the piece's frame bytes to the device mirror and point the
// kernel at it, or (scattered frames) at the mapped host UMEM.  Returns 1 when
// the kernel reads host memory (mapped), 0 when it reads the mirror.
int stage_frames(xsknf_gpu_ctx *c, Slot &s, uint32_t n, xsknf_gpu::KernelArgs &a) {
  s.offs.resize(n);
  s.order.clear();
  bool sorted = true;
  uint64_t prev = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t off = umem_offset(s.descs[i].addr);
    const uint32_t len = s.descs[i].len;
    s.offs[i] = off;
    if (off > c->umem_size || len > c->umem_size - off || len == 0) continue;
    if (off < prev) sorted = false;
    prev = off;
    s.order.push_back(i);
  }
  a.umem_size = c->umem_size;
  if (!sorted && s.order.size() > kSortMax) {
    // a large batch out of address order: scattered for every practical purpose
    // (sorting 64K offsets costs more than reading the frames over PCIe)
    uint64_t moved = 0;
    for (uint32_t i : s.order) moved += s.descs[i].len;
    c->stats.bytes_h2d += moved;
    a.umem = c->umem_mapped;
    return 1;
  }
  if (!sorted)
    std::sort(s.order.begin(), s.order.end(), [&](uint32_t x, uint32_t y) { return s.offs[x] < s.offs[y]; });
  // merged runs
  s.runs.clear();
  for (uint32_t i : s.order) {
    const uint64_t off = s.offs[i], end = off + s.descs[i].len;
    if (!s.runs.empty() && off <= s.runs.back().off + s.runs.back().len + kMergeGap) {
      Run &r = s.runs.back();
      if (end > r.off + r.len) r.len = end - r.off;
    } else {
      s.runs.push_back(Run{off, end - off});
    }
  }
  a.umem = c->umem_dev;
  a.umem_size = c->umem_size;
  uint64_t moved = 0;
  hipError_t e = hipSuccess;
  if (s.runs.size() <= kMaxDmaRuns) {
    for (const Run &r : s.runs) {
      e = hipMemcpyAsync(c->umem_dev + r.off, c->umem_host + r.off, r.len, hipMemcpyHostToDevice, s.stream);
      if (e != hipSuccess) return fail(e, "hipMemcpyAsync(run)");
      moved += r.len;
    }
  } else {
    // one 2-D copy when the frames sit at a constant stride (aligned chunks in rx order)
    const size_t k = s.order.size();
    const uint64_t o0 = s.offs[s.order[0]];
    const uint64_t stride = s.offs[s.order[1]] - o0;
    uint32_t width = 0;
    bool uniform = stride > 0;
    for (size_t j = 0; uniform && j < k; ++j) {
      uniform = s.offs[s.order[j]] == o0 + j * stride;
      width = std::max(width, s.descs[s.order[j]].len);
    }
    uniform = uniform && width <= stride && o0 + (k - 1) * stride + width <= c->umem_size;
    if (uniform) {
      e = hipMemcpy2DAsync(c->umem_dev + o0, stride, c->umem_host + o0, stride, width, k, hipMemcpyHostToDevice,
                           s.stream);
      if (e != hipSuccess) return fail(e, "hipMemcpy2DAsync(frames)");
      moved = static_cast<uint64_t>(width) * k;
    } else {
      // scattered: the kernel reads the frames from the mapped UMEM over PCIe
      a.umem = c->umem_mapped;
      for (uint32_t i : s.order) moved += s.descs[i].len;
      c->stats.bytes_h2d += moved;
      return 1;
    }
  }
  c->stats.bytes_h2d += moved;
  return 0;
}

// A small batch read over PCIe is a few 64-frame tiles: the split kernel
// would read it with a few waves.  The group kernel spreads it over many (4 or
// 2 frames per wave), so more reads are in flight (tools/small_batch.py,
// 1500 B: 64 frames 44.8 -> 18.8 us per call, 256: 46.8 -> 24.1, 1024:
// 51.0 -> 45.0; equal from 4096).
void pcie_small_batch_cfg(uint32_t n, xsknf_gpu_launch_cfg &cfg) {
  if (n > 2048) return;
  cfg.kernel = XSKNF_GPU_KERNEL_AUTO;
  cfg.window_chunks = 0;
  cfg.lds_ring = 0;
  cfg.lanes_per_frame = n <= 256 ? 32 : 64;
  cfg.chunks_per_lane = n <= 256 ? 3 : 2;
  cfg.frames_per_group = n <= 256 ? 2 : 4;
}

// Enqueue one piece (n <= slot_frames) into the next slot.
int submit_piece(xsknf_gpu_ctx *c, const xsknf_gpu_desc *descs, uint32_t n, uint32_t ingress_ifindex,
                 const xsknf_csum_opts *opts, int32_t *verdicts) {
  using namespace xsknf_gpu;
  Slot &s = c->slot[c->next];
  int rc = complete(c, s);
  if (rc) return rc;
  KernelArgs a;
  rc = prepare(a, c->umem_dev, c->umem_size, s.descs_mapped, n, ingress_ifindex, opts, s.rec_mapped);
  if (rc != 0) return rc < 0 ? rc : 0;
  memcpy(s.descs, descs, sizeof(xsknf_gpu_desc) * n);
  c->stats.bytes_h2d += sizeof(xsknf_gpu_desc) * n;

  xsknf_gpu_launch_cfg cfg;
  default_cfg(c->hint ? c->hint : 2048u, cfg);
  bool mapped = c->path != XSKNF_GPU_PATH_STAGED;
  if (!mapped) {
    rc = stage_frames(c, s, n, a);
    if (rc < 0) return rc;
    mapped = rc == 1;   // scattered frames: read (and written) in host memory, as ZEROCOPY
  }
  if (mapped) {
    pcie_small_batch_cfg(n, cfg);
    cfg.fused_stores = 1;   // in place over PCIe, ...
    a.sector_stores = 0;    // ... as 2-byte writes (byte enables; no RMW in host memory)
  } else {
    cfg.fused_stores = 3;   // records only: the checks are applied on the host (complete())
  }
  s.host_checks = !mapped;
  rc = run(a, cfg, s.stream, true);
  if (rc != 0) return rc;
  hipError_t e = hipEventRecord(s.done, s.stream);
  if (e != hipSuccess) return fail(e, "hipEventRecord");
  s.busy = true;
  s.seq = ++c->seq;
  s.n = n;
  s.out = verdicts;
  s.fwd = a.fwd_verdict;
  c->next = (c->next + 1) % kSlots;
  return 0;
}

int submit(xsknf_gpu_ctx *c, const xsknf_gpu_desc *descs, uint32_t n, uint32_t ingress_ifindex,
           const xsknf_csum_opts *opts, int32_t *verdicts, uint64_t *ticket) {
  if (!c || !c->registered || n > c->max_batch) return -EINVAL;
  if (n && (!descs || !verdicts)) return -EINVAL;
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) return fail(e, "hipSetDevice");
  if (c->path == XSKNF_GPU_PATH_RESIDENT) {
    // every batch through the ring, in entries of up to kResFrames frames (a
    // larger batch is processed by several blocks at once)
    for (uint32_t p = 0; p < n; p += xsknf_gpu::kResFrames) {
      const uint32_t k = std::min(xsknf_gpu::kResFrames, n - p);
      const int rc = ring_submit(c, descs + p, k, ingress_ifindex, opts, verdicts + p);
      if (rc) {
        if (p) (void)complete_upto(c, c->seq);
        return rc;
      }
    }
    if (ticket) *ticket = c->seq;
    return 0;
  }
  for (uint32_t p = 0; p < n; p += c->slot_frames) {
    const uint32_t k = std::min(c->slot_frames, n - p);
    const int rc = submit_piece(c, descs + p, k, ingress_ifindex, opts, verdicts + p);
    if (rc) {
      // the batch's earlier pieces are in flight and write into `verdicts` and
      // the frames: no ticket goes back, so finish them (and anything older)
      // before the caller recycles those frames
      if (p) (void)complete_upto(c, c->seq);
      return rc;
    }
  }
  if (ticket) *ticket = c->seq;
  return 0;
}

}  // namespace

extern "C" {

int xsknf_gpu_ctx_create(struct xsknf_gpu_ctx **out, int device, int path, uint32_t max_batch,
                         uint32_t frame_len_hint) {
  if (!out || max_batch == 0) return -EINVAL;
  if (path != XSKNF_GPU_PATH_ZEROCOPY && path != XSKNF_GPU_PATH_STAGED && path != XSKNF_GPU_PATH_RESIDENT)
    return -EINVAL;
  *out = nullptr;
  xsknf_gpu_ctx *c = new (std::nothrow) xsknf_gpu_ctx;
  if (!c) return -ENOMEM;
  c->device = device;
  c->path = path;
  c->max_batch = max_batch;
  c->slot_frames = std::min(max_batch, kPiece);
  c->hint = frame_len_hint;
  if (device < 0 || device >= 64) {
    delete c;
    return -EINVAL;
  }
  hipError_t e = hipSetDevice(device);
  for (Slot &s : c->slot) {
    if (path == XSKNF_GPU_PATH_RESIDENT) break;   // the ring takes every batch
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipHostMalloc(&s.descs, sizeof(xsknf_gpu_desc) * c->slot_frames, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc(&s.rec, sizeof(int32_t) * c->slot_frames, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&s.descs_mapped), s.descs, 0);
    if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&s.rec_mapped), s.rec, 0);
  }
  if (e == hipSuccess && path == XSKNF_GPU_PATH_RESIDENT) {
    using namespace xsknf_gpu;
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    // headers and descriptors in one block: ResIn[kResSlots], then the descriptors
    const size_t in_bytes = sizeof(ResIn) * kResSlots + sizeof(xsknf_gpu_desc) * kResSlots * kResFrames;
    int large_bar = 0;
    const char *bar_env = getenv("XSKNF_RESIDENT_BAR");   // 0: keep the ring in host memory (A/B)
    if ((!bar_env || atoi(bar_env) != 0) &&
        hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, device) == hipSuccess && large_bar) {
      void *p = nullptr;
      if (hipExtMallocWithFlags(&p, in_bytes, hipDeviceMallocFinegrained) == hipSuccess) {
        c->rin = static_cast<ResIn *>(p);
        c->rbar = true;
      } else {
        (void)hipGetLastError();
      }
    }
    if (!c->rin) e = hipHostMalloc(&c->rin, in_bytes, fl);
    if (e == hipSuccess) c->rdescs = reinterpret_cast<xsknf_gpu_desc *>(c->rin + kResSlots);
    if (e == hipSuccess) e = hipHostMalloc(&c->rout, sizeof(ResOut) * kResBlocks, fl);
    if (e == hipSuccess) e = hipHostMalloc(&c->rverd, sizeof(int32_t) * kResSlots * kResFrames, fl);
    if (e == hipSuccess) {
      for (uint32_t k = 0; k < kResSlots; ++k)   // (host stores: the BAR mapping is the same address)
        c->rin[k].seqn = 0;
      for (uint32_t k = 0; k < kResBlocks; ++k) c->rout[k].done = 0;
      if (c->rbar) _mm_sfence();
      if (c->rbar) {
        c->rring.in = c->rin;
        c->rring.descs = c->rdescs;
      } else {
        e = hipHostGetDevicePointer(reinterpret_cast<void **>(&c->rring.in), c->rin, 0);
        if (e == hipSuccess) c->rring.descs = reinterpret_cast<xsknf_gpu_desc *>(c->rring.in + kResSlots);
      }
    }
    if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&c->rring.out), c->rout, 0);
    if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&c->rring.verdicts), c->rverd, 0);
    // batches of up to 64 frames: one block per entry (a group's idle blocks
    // would cost them ~1 us); larger ones: the group deals 64-frame rounds
    c->rring.group = max_batch <= kResBlockFrames ? 1 : kResGroup;
  }
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
  if (e == hipSuccess) e = hipHostRegister(umem, size, hipHostRegisterMapped);
  if (e != hipSuccess) return fail(e, "hipHostRegister(umem)");
  c->registered = true;
  c->umem_host = static_cast<uint8_t *>(umem);
  c->umem_size = size;
  void *dp = nullptr;
  e = hipHostGetDevicePointer(&dp, umem, 0);
  c->umem_mapped = static_cast<uint8_t *>(dp);
  if (e == hipSuccess) {
    if (c->path != XSKNF_GPU_PATH_STAGED)
      c->umem_dev = c->umem_mapped;
    else
      e = hipMalloc(&c->umem_dev, size + 16);   // + the last chunk's 16-byte read
  }
  if (e != hipSuccess) {
    (void)hipHostUnregister(umem);
    c->registered = false;
    c->umem_dev = c->umem_mapped = nullptr;
    return fail(e, "xsknf_gpu_ctx_register_umem");
  }
  if (c->path == XSKNF_GPU_PATH_RESIDENT) {
    // the resident kernel's view of the ring: the mapped UMEM (checks in-line as
    // 2-byte stores: host memory has byte enables), per-batch fields from the ring
    c->rring.umem = c->umem_dev;
    c->rring.umem_size = c->umem_size;
    // the device's resident kernel serves this ring from now on
    const int rc = svc_add(c);
    if (rc) {
      (void)hipHostUnregister(umem);
      c->registered = false;
      c->umem_dev = c->umem_mapped = nullptr;
      return rc;
    }
  }
  return 0;
}

int xsknf_gpu_ctx_submit(struct xsknf_gpu_ctx *c, const struct xsknf_gpu_desc *descs, uint32_t n,
                         uint32_t ingress_ifindex, const struct xsknf_csum_opts *opts, int32_t *verdicts,
                         uint64_t *ticket) {
  if (!ticket) return -EINVAL;
  return submit(c, descs, n, ingress_ifindex, opts, verdicts, ticket);
}

int xsknf_gpu_ctx_wait(struct xsknf_gpu_ctx *c, uint64_t ticket) {
  if (!c) return -EINVAL;
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) return fail(e, "hipSetDevice");
  return complete_upto(c, ticket);
}

int xsknf_gpu_ctx_process_batch(struct xsknf_gpu_ctx *c, const struct xsknf_gpu_desc *descs, uint32_t n,
                                uint32_t ingress_ifindex, const struct xsknf_csum_opts *opts,
                                int32_t *verdicts) {
  uint64_t t = 0;
  const int rc = submit(c, descs, n, ingress_ifindex, opts, verdicts, &t);
  if (rc) {
    if (c) (void)complete_upto(c, UINT64_MAX);   // leave nothing in flight
    return rc;
  }
  return complete_upto(c, t);
}

int xsknf_gpu_ctx_get_stats(const struct xsknf_gpu_ctx *c, struct xsknf_gpu_ctx_stats *stats) {
  if (!c || !stats) return -EINVAL;
  *stats = c->stats;
  if (c->path == XSKNF_GPU_PATH_RESIDENT) stats->resident_launches = g_svc[c->device].launches.load();
  return 0;
}

int xsknf_gpu_ctx_destroy(struct xsknf_gpu_ctx *c) {
  if (!c) return -EINVAL;
  (void)hipSetDevice(c->device);
  (void)complete_upto(c, UINT64_MAX);
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
  if (path != XSKNF_GPU_PATH_ZEROCOPY && path != XSKNF_GPU_PATH_STAGED && path != XSKNF_GPU_PATH_RESIDENT)
    return -EINVAL;
  if (opts->action != XSKNF_CSUM_ACTION_REDIRECT && opts->action != XSKNF_CSUM_ACTION_DROP) return -EINVAL;
  *out = nullptr;
  int devices = 0;
  // (no device: -ENODEV, and the error text says what this process saw)
  const int rc = xsknf_gpu_device_count(&devices);
  if (rc) return rc;
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

}  // extern "C"

namespace {

// The worker's context for `umem`, created and registered on first use
// (umem_size == 0: look up only).
int hook_ctx(xsknf_gpu_hook *h, uint32_t worker_idx, void *umem, uint64_t umem_size, xsknf_gpu_ctx **out) {
  if (!h || worker_idx >= h->workers || !umem) return -EINVAL;
  HookWorker &w = h->w[worker_idx];
  for (HookSlot &s : w.slot) {
    if (s.umem == umem) {
      *out = s.ctx;
      return 0;
    }
  }
  if (umem_size == 0) return -ENOENT;
  HookSlot *free_slot = nullptr;
  for (HookSlot &s : w.slot) {
    if (!s.umem) {
      free_slot = &s;
      break;
    }
  }
  if (!free_slot) return -ENOSPC;
  xsknf_gpu_ctx *ctx = nullptr;
  int rc = xsknf_gpu_ctx_create(&ctx, static_cast<int>(worker_idx % static_cast<uint32_t>(h->devices)), h->path,
                                h->max_batch, h->hint);
  if (rc) return rc;
  rc = xsknf_gpu_ctx_register_umem(ctx, umem, umem_size);
  if (rc) {
    xsknf_gpu_ctx_destroy(ctx);
    return rc;
  }
  free_slot->umem = umem;
  free_slot->ctx = ctx;
  *out = ctx;
  return 0;
}

}  // namespace

extern "C" {

int xsknf_gpu_hook_process(void *hook, uint32_t worker_idx, void *umem, uint64_t umem_size,
                           const struct xsknf_gpu_desc *descs, uint32_t n, uint32_t ingress_ifindex,
                           int32_t *verdicts) {
  xsknf_gpu_hook *h = static_cast<xsknf_gpu_hook *>(hook);
  if (!h || umem_size == 0 || n > h->max_batch) return -EINVAL;
  xsknf_gpu_ctx *ctx = nullptr;
  const int rc = hook_ctx(h, worker_idx, umem, umem_size, &ctx);
  if (rc) return rc;
  return xsknf_gpu_ctx_process_batch(ctx, descs, n, ingress_ifindex, &h->opts, verdicts);
}

int xsknf_gpu_hook_submit(void *hook, uint32_t worker_idx, void *umem, uint64_t umem_size,
                          const struct xsknf_gpu_desc *descs, uint32_t n, uint32_t ingress_ifindex,
                          int32_t *verdicts, uint64_t *ticket) {
  xsknf_gpu_hook *h = static_cast<xsknf_gpu_hook *>(hook);
  if (!h || umem_size == 0 || n > h->max_batch || !ticket) return -EINVAL;
  xsknf_gpu_ctx *ctx = nullptr;
  const int rc = hook_ctx(h, worker_idx, umem, umem_size, &ctx);
  if (rc) return rc;
  return xsknf_gpu_ctx_submit(ctx, descs, n, ingress_ifindex, &h->opts, verdicts, ticket);
}

int xsknf_gpu_hook_complete(void *hook, uint32_t worker_idx, void *umem, uint64_t ticket) {
  xsknf_gpu_hook *h = static_cast<xsknf_gpu_hook *>(hook);
  xsknf_gpu_ctx *ctx = nullptr;
  const int rc = hook_ctx(h, worker_idx, umem, 0, &ctx);
  if (rc) return rc;
  return xsknf_gpu_ctx_wait(ctx, ticket);
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
    stats->resident_batches += s.ctx->stats.resident_batches;
    if (s.ctx->path == XSKNF_GPU_PATH_RESIDENT) stats->resident_launches = g_svc[s.ctx->device].launches.load();
  }
  return 0;
}

int xsknf_gpu_hook_destroy(struct xsknf_gpu_hook *h) {
  if (!h) return -EINVAL;
  for (uint32_t i = 0; i < h->workers; ++i)
    for (HookSlot &s : h->w[i].slot)
      if (s.ctx) xsknf_gpu_ctx_destroy(s.ctx);
  delete[] h->w;
  delete h;
  return 0;
}

}  // extern "C"
