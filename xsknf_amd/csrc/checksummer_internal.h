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
int run(const KernelArgs &base, const xsknf_gpu_launch_cfg &cfg, void *stream);
void default_cfg(uint32_t hint, xsknf_gpu_launch_cfg &c, uint32_t mean = 0);
void set_error(hipError_t e, const char *where);
void set_error_text(const char *text);

}  // namespace xsknf_gpu
