// checksummer_internal.h -- declarations shared by the gfx950 checksummer
// kernels (checksummer.hip) and the host-path context (host_path.hip).
// Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/xsknf_gpu.h"

namespace xsknf_gpu {

struct KernelArgs {
  uint8_t *umem;
  uint64_t umem_size;
  const xsknf_gpu_desc *descs;
  int32_t *verdicts;
  uint32_t n;
  uint32_t payload_mult;   // max(csum_iterations, 0)
  int32_t fwd_verdict;     // REDIRECT ? (ingress+1) % n_if : -1
  uint32_t defer_min_len;  // frames at least this long park a check record for the
                           // scatter pass; shorter ones write their check in-line
  const uint4 *dummy;      // readable 16-byte block for frames that need no bytes
  uint32_t no_scatter;     // 1: leave deferred check records in `verdicts` (the host
                           // path applies them itself)
  uint32_t seq;            // launch sequence number: slot of the record counter
  uint32_t count_records;  // 1: the summing kernel counts its records for the scatter pass
  uint32_t sector_stores;  // 1: an in-line check whose 64-byte sector lies inside the
                           // frame is written as that whole sector (device memory:
                           // no read-modify-write); 0: 2-byte stores (host memory)
  uint32_t plain_sector;   // 1: whole-sector stores of the lane kernel are plain (write-back),
                           // 0: non-temporal
  uint32_t tail_scatter;   // 1 (split kernel): each wave patches the deferred checks of its
                           // own tiles after its last tile; no scatter launch
  uint32_t store_unchanged;  // 1: write a check even when the frame already holds it
                             // (A/B); 0: such a frame is left untouched
};

// Check record parked in verdicts[f] by the summing pass (deferred stores):
// tag 01 in bits 31..30 (no verdict, -1 or 0..XSKNF_MAX_INTERFACES-1, has it),
// u in bits 22..16, the new check in bits 15..0.
constexpr uint32_t kRecTag = XSKNF_GPU_RECORD_TAG;
constexpr uint32_t kRecTagMask = XSKNF_GPU_RECORD_TAG_MASK;
constexpr uint32_t kNoDefer = 0xffffffffu;   // defer_min_len: every check in-line

// Validate arguments and fill `a` (returns 1 for an empty batch, <0 on error).
int prepare(KernelArgs &a, uint8_t *umem, uint64_t umem_size, const xsknf_gpu_desc *descs, uint32_t n,
            uint32_t ingress_ifindex, const xsknf_csum_opts *opts, int32_t *verdicts);
// Launch the shape `cfg` (summing kernel + scatter pass unless a.no_scatter).
// product_shape: cfg is default_cfg()'s (or leaves blocks_per_cu to the library),
// so a lane-kernel launch of more than 2M frames may take the per-lane windows
// and 8 blocks per CU; an explicit shape runs exactly as asked.
int run(const KernelArgs &base, const xsknf_gpu_launch_cfg &cfg, void *stream, bool product_shape);
void default_cfg(uint32_t hint, xsknf_gpu_launch_cfg &c, uint32_t mean = 0);
void set_error(hipError_t e, const char *where);
void set_error_text(const char *text);
// hipGetDeviceCount failed or saw no device: -ENODEV, with what the process saw
// (KFD / render node access, *_VISIBLE_DEVICES, KFD processes) as the error text
int set_device_error(hipError_t e, int count, const char *where);

// ---- the resident worker (XSKNF_GPU_PATH_RESIDENT, host_path.hip) ----------
// ONE kernel per device stays resident and serves the rings of every RESIDENT
// context on that device (one per worker and UMEM: up to kResMaxRings).  Each
// ring has kResSlots entries; a group of `group` 4-wave blocks serves each
// entry: the host writes a batch's descriptors and header into entry
// seq % kResSlots and publishes seq; the entry's blocks poll for it, checksum
// the batch over PCIe in the mapped UMEM (the register kernel's tiles, dealt
// over the group: group_tiles) and each publishes its own `done`.  No launch
// per batch, and up to kResSlots batches per ring in flight at once: the ~10 us
// launch and completion round trip of a small batch becomes a doorbell and a
// flag.  When the rings would need more blocks than the kernel may hold
// (ResArgs::entries_per_block), a block serves several entries of its ring.
#ifndef XSKNF_RES_SLOTS   // (A/B: tools/ab_resring.sh)
#define XSKNF_RES_SLOTS 8
#define XSKNF_RES_FRAMES 256
#endif
#ifndef XSKNF_RES_GROUP   // blocks per ring entry (A/B: tools/ab_resgroup.sh)
#define XSKNF_RES_GROUP 4
#endif
constexpr uint32_t kResSlots = XSKNF_RES_SLOTS;     // ring entries
constexpr uint32_t kResFrames = XSKNF_RES_FRAMES;   // frames per entry (a larger batch takes several)
constexpr uint32_t kResGroup = XSKNF_RES_GROUP;     // blocks per entry at most
constexpr uint32_t kResBlocks = kResSlots * kResGroup;   // done flags per ring (entry x kResGroup + g)
constexpr uint32_t kResMaxRings = 64;        // XSKNF_MAX_WORKERS (32) x a zero-copy and a copy-mode UMEM
constexpr uint32_t kResMaxBlocks = 1024;     // grid limit of the resident kernel (and the device's share)
constexpr uint64_t kResQuit = ~0ull;
constexpr uint32_t kResBlockFrames = 64;   // frames one block takes per round (4 waves x 16-frame tiles)
// blocks of an entry (`group` of them) with frames of an n-frame batch: only
// these publish done (a block without frames moves on; the host reuses the
// entry once these have)
inline constexpr uint32_t res_used_blocks(uint32_t n, uint32_t group) {
  return n == 0 ? 1 : ((n + kResBlockFrames - 1) / kResBlockFrames < group
                           ? (n + kResBlockFrames - 1) / kResBlockFrames : group);
}

struct alignas(64) ResIn {     // host -> device: the entry's header.  Coherent mapped host memory,
                               // or (large-BAR devices) fine-grained device memory the host writes
                               // through the BAR, so the polls and header reads stay on the device
  uint64_t seqn;               // the entry's batch (release): ring sequence number (from 1) << 16 | frames,
                               // one word, so a block reads the count that belongs to the number
  int32_t fwd;                 // forward verdict (prepare()), written before seqn; with payload_mult
  uint32_t payload_mult;       // one 8-byte word the kernel reads with one load
  uint32_t pad[12];
};

struct alignas(64) ResOut {    // device -> host, one per (entry, block of its group): host memory
  uint64_t done;               // seq once the block's share of the batch is complete (release)
  uint64_t pad[7];
};

struct alignas(64) ResCtl {    // host memory, coherent and mapped, one per device
  uint64_t stop;               // host -> device: exit now (unless ResStop is in device memory)
  uint64_t pad0[7];
  uint64_t exited;             // device -> host: the epoch of the launch whose last block has left
  uint64_t pad1[7];
};

struct alignas(64) ResStop {   // host -> device: exit now.  Fine-grained device memory the host
  uint64_t stop;               // writes through the BAR (large-BAR devices), so that the blocks'
  uint64_t pad[7];             // polls of it stay on the device and take nothing from the PCIe
};                             // reads of the batches; else ResCtl::stop in host memory

struct ResRing {               // one RESIDENT context's ring, as the kernel sees it
  uint8_t *umem;               // the context's mapped UMEM (checks in-line as 2-byte stores; n / fwd /
  uint64_t umem_size;          // mult per batch from the entry's header)
  ResIn *in;                   // headers (kResSlots) and, beside them, descriptors (kResSlots x kResFrames)
  xsknf_gpu_desc *descs;
  ResOut *out;                 // done flags (kResBlocks) and verdicts (kResSlots x kResFrames): host memory
  int32_t *verdicts;
  uint32_t group;              // blocks per entry: 1, or kResGroup (fixed for the ring's life: the host
  uint32_t pad;                // waits for res_used_blocks(n, group) flags per batch)
};

struct ResLaunch {             // device memory, written by the host before each launch
  uint64_t act;                // device-wide activity: the clock of the last batch any block finished
                               // (atomic max); kResQuit once a block has left (every block then leaves)
  uint32_t exits;              // blocks that have left (the last one reports the epoch in ResCtl)
  uint32_t pad[13];
  ResRing ring[kResMaxRings];
  uint32_t block[kResMaxBlocks];                  // blockIdx -> ring << 16 | g << 8 | first entry
  uint64_t start[kResMaxRings][kResBlocks];       // the first sequence number per (ring, entry x kResGroup + g)
};

struct ResArgs {
  ResLaunch *L;
  const ResRing *rings;        // = L->ring, read only: its pointers are then known to be global
  ResCtl *ctl;                 // device view of the device's ResCtl
  uint64_t *stop;              // device view of the stop word (ResStop, or ResCtl::stop)
  uint64_t epoch;              // this launch's number (ResCtl::exited)
  uint32_t blocks;             // grid size
  uint32_t entries_per_block;  // 1, 2, 4 or 8: a block serves entries b, b + kResSlots / E, ...
  uint64_t idle_ticks;         // exit after this long without a batch on any ring (100 MHz clock) ...
  uint64_t life_ticks;         // ... or after this long in all; the host relaunches on demand
};

int launch_resident(const ResArgs &ra, hipStream_t stream);
// blocks of the resident kernel one CU holds (occupancy), for the grid's cap
int resident_blocks_per_cu();
int device_cu_count();

}  // namespace xsknf_gpu
