// shard_plan.cpp -- the host-side arithmetic of the multi-device path (no GPU):
// byte-balanced shard cuts, span rebasing and the packed layout
// (include/xsknf_gpu.h xsknf_gpu_shard_plan / _rebase / _pack_plan).  Plain C++,
// so that tests/test_sanitizers.py can build it under AddressSanitizer + UBSan;
// linked into libxsknf_gpu.so with the HIP sources (xsknf_amd/csrc/multi.hip
// uses them for xsknf_gpu_multi_scatter and _scatter_packed).
#include <errno.h>
#include <stdint.h>

#include "../../include/xsknf_gpu.h"

namespace {

constexpr uint64_t kOutOfRange = 1ull << 47;   // an address past any UMEM: verdict -1, no bytes

inline uint64_t umem_offset(uint64_t addr) {
  return (addr & XSKNF_GPU_UNALIGNED_BUF_ADDR_MASK) + (addr >> XSKNF_GPU_UNALIGNED_BUF_OFFSET_SHIFT);
}

inline bool in_umem(const xsknf_gpu_desc &d, uint64_t umem_size) {
  const uint64_t off = umem_offset(d.addr);
  return off <= umem_size && d.len <= umem_size - off;
}

}  // namespace

extern "C" {

int xsknf_gpu_shard_plan(const struct xsknf_gpu_desc *descs, uint64_t n, uint64_t umem_size, uint32_t nshards,
                         uint64_t *bounds, uint64_t *spans) {
  if (nshards == 0 || !bounds || (n && !descs)) return -EINVAL;
  // cuts: shard r starts after the first frame whose running byte count
  // reaches total * r / nshards (shard.py: searchsorted(cumsum, target,
  // "left") + 1, then clamped to n and made non-decreasing).  The targets are
  // the correctly rounded doubles of the rationals, as Python's int / int;
  // the running sums are exact in a double below 2^53 bytes.
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i) total += descs[i].len;
  bounds[0] = 0;
  uint64_t i = 0, csum = n ? descs[0].len : 0;
  for (uint32_t r = 1; r < nshards; ++r) {
    const double target = static_cast<double>(total * r) / nshards;
    while (i < n && static_cast<double>(csum) < target) {
      ++i;
      if (i < n) csum += descs[i].len;
    }
    uint64_t cut = n == 0 ? 0 : i + 1;
    if (cut > n) cut = n;
    if (cut < bounds[r - 1]) cut = bounds[r - 1];
    bounds[r] = cut;
  }
  bounds[nshards] = n;
  if (spans) {
    for (uint32_t r = 0; r < nshards; ++r) {
      uint64_t b0 = UINT64_MAX, b1 = 0;
      for (uint64_t f = bounds[r]; f < bounds[r + 1]; ++f) {
        if (!in_umem(descs[f], umem_size)) continue;
        const uint64_t off = umem_offset(descs[f].addr);
        if (off < b0) b0 = off;
        if (off + descs[f].len > b1) b1 = off + descs[f].len;
      }
      spans[2 * r] = b0 == UINT64_MAX ? 0 : b0;
      spans[2 * r + 1] = b0 == UINT64_MAX ? 0 : b1;
    }
  }
  return 0;
}

int xsknf_gpu_shard_rebase(const struct xsknf_gpu_desc *descs, uint64_t n, uint64_t b0, uint64_t umem_size,
                           struct xsknf_gpu_desc *out) {
  if (n && (!descs || !out)) return -EINVAL;
  for (uint64_t i = 0; i < n; ++i) {
    const xsknf_gpu_desc d = descs[i];
    out[i].addr = in_umem(d, umem_size) ? umem_offset(d.addr) - b0 : kOutOfRange;
    out[i].len = d.len;
    out[i].options = d.options;
  }
  return 0;
}

int xsknf_gpu_shard_pack_plan(const struct xsknf_gpu_desc *descs, uint64_t n, uint64_t umem_addr,
                              uint64_t umem_size, uint32_t nshards, const uint64_t *bounds,
                              struct xsknf_gpu_desc *packed, uint64_t *sizes) {
  if (nshards == 0 || !bounds || !sizes || (n && (!descs || !packed))) return -EINVAL;
  if (bounds[0] != 0 || bounds[nshards] != n) return -EINVAL;
  // shard k's frames in global order, each in its own 16-byte aligned slot at
  // the same address mod 16 as in the UMEM (so the kernels read it exactly as
  // there); the descriptors each shard receives address its own packed bytes
  for (uint32_t k = 0; k < nshards; ++k) {
    if (bounds[k + 1] < bounds[k]) return -EINVAL;
    uint64_t pos = 0;
    for (uint64_t f = bounds[k]; f < bounds[k + 1]; ++f) {
      const xsknf_gpu_desc d = descs[f];
      packed[f].len = d.len;
      packed[f].options = d.options;
      if (!in_umem(d, umem_size)) {
        packed[f].addr = kOutOfRange;
        continue;
      }
      const uint64_t rs = (umem_addr + umem_offset(d.addr)) & 15;
      packed[f].addr = pos + rs;
      pos += d.len ? (rs + d.len + 15) & ~15ull : 0;
    }
    sizes[k] = pos;
  }
  return 0;
}

}  // extern "C"
