// checksummer.hip -- gfx950 kernel for the xsknf checksummer per-packet path.
//
// Reference semantics: examples/checksummer/checksummer_user.c:30-112
// (xsknf_packet_processor), applied to every descriptor of an rx batch as the
// per-frame loop of src/xsknf.c:654-672 does.
//
// The reference sums 16-bit words serially from the UDP header to the end of
// the frame.  The sum is a wrapping u32, so it can be taken in any order and
// in closed form:
//     s = pseudo + max(iters,0) * P                         (mod 2^32)
//     P = sum_{k even} f[u+k] + 256 * sum_{k odd} f[u+k],   k in [0, len-u)
// with f[u+6], f[u+7] (the old check) counted as zero.  "k even" is the set of
// bytes whose ABSOLUTE address parity equals that of the UDP header start, so
// the kernel reads the frame as 16-byte aligned chunks wherever the frame
// starts (unaligned-chunk UMEM puts frames at odd addresses) and splits every
// dword into its low-weight and high-weight byte pairs with v_dot4_u32_u8,
// whose u8 weight operand also carries the [udp, end) byte mask.
//
// Mapping (MI355X: 64-lane waves, HBM-bound, no MFMA): a group of LPF lanes
// owns one frame; a wave holds 64/LPF groups; each lane loads NCH 16-byte
// chunks per pass, so a pass covers LPF*NCH*16 contiguous bytes of the frame
// with dwordx4 loads that are contiguous across the group's lanes.  The first
// 7 chunks (bytes [0,112) of the aligned window, i.e. every header byte the
// reference reads, wherever the frame starts) are staged in LDS once so the
// parse reads bytes by address.  Group partial sums are reduced with DPP
// shuffles; one lane per group writes the 2 check bytes and the verdict.
// The grid is persistent (a few blocks per CU) and strides over frames, with
// the next descriptor prefetched while the current frame's loads are in flight.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <errno.h>
#include <string.h>

#include "../../include/xsknf_gpu.h"

namespace xsknf_gpu {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kHdrChunks = 7;   // (15 + 74 + 8 + 15) / 16 rounded up: max rel offset of f[u+7] is 15+81

__device__ __forceinline__ uint64_t umem_offset(uint64_t addr) {
  return (addr & XSKNF_GPU_UNALIGNED_BUF_ADDR_MASK) + (addr >> XSKNF_GPU_UNALIGNED_BUF_OFFSET_SHIFT);
}

// 0x01 in every byte b of the dword at window offset x with lo <= x+b < hi.
__device__ __forceinline__ uint32_t byte_ones(int lo, int hi, int x) {
  const int a = min(max(lo - x, 0), 4);
  const int b = min(max(hi - x, 0), 4);
  const uint64_t m = ((1ull << (8 * b)) - 1ull) & ~((1ull << (8 * a)) - 1ull);
  return static_cast<uint32_t>(m) & 0x01010101u;
}

// Sum of one 16-byte chunk's bytes in [lo, hi) (window offsets), split by the
// weight classes wl (bytes that are low in their 16-bit word) / wh (high).
__device__ __forceinline__ void chunk_sum(const uint4 v, int x, int lo, int hi, uint32_t wl,
                                          uint32_t wh, uint32_t &acc_lo, uint32_t &acc_hi) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t m = byte_ones(lo, hi, x + 4 * j);
    acc_lo = __builtin_amdgcn_udot4(w[j], m & wl, acc_lo, false);
    acc_hi = __builtin_amdgcn_udot4(w[j], m & wh, acc_hi, false);
  }
}

__device__ __forceinline__ void compiler_barrier() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

template <int LPF>
__device__ __forceinline__ uint32_t group_sum(uint32_t v) {
#pragma unroll
  for (int m = LPF / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, kWave);
  return v;
}

struct KernelArgs {
  uint8_t *umem;
  uint64_t umem_size;
  const xsknf_gpu_desc *descs;
  int32_t *verdicts;
  uint32_t n;
  uint32_t payload_mult;   // max(csum_iterations, 0)
  int32_t fwd_verdict;     // REDIRECT ? (ingress+1) % n_if : -1
};

template <int LPF, int NCH>
__global__ __launch_bounds__(kBlock) void checksum_kernel(const KernelArgs args) {
  static_assert(kWave % LPF == 0, "LPF must divide the wave");
  static_assert(LPF * NCH >= kHdrChunks, "pass 0 must cover the header window");
  constexpr int G = kWave / LPF;     // frames in flight per wave
  constexpr int SPAN = LPF * NCH;    // chunks per pass

  __shared__ uint4 hdr[kWavesPerBlock][G][kHdrChunks];

  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x / kWave;
  const int grp = lane / LPF;
  const int gl = lane % LPF;
  const uint32_t stride = gridDim.x * kWavesPerBlock * G;
  uint32_t f = (blockIdx.x * kWavesPerBlock + wv) * G + grp;

  xsknf_gpu_desc d;
  if (f < args.n) d = args.descs[f];

  for (; f < args.n; f += stride) {
    const uint64_t off = umem_offset(d.addr);
    const uint32_t len = d.len;
    // prefetch the next descriptor of this group while this frame is worked on
    const uint32_t fn = f + stride;
    xsknf_gpu_desc dn;
    if (fn < args.n) dn = args.descs[fn];

    if (off > args.umem_size || len > args.umem_size - off) {
      if (gl == 0) args.verdicts[f] = -1;
      d = dn;
      continue;
    }

    uint8_t *fp = args.umem + off;
    // 16-byte aligned window around the frame, kept as an offset from the kernel
    // argument so the compiler keeps global (not flat) addressing
    const int rs = static_cast<int>(reinterpret_cast<uintptr_t>(fp) & 15);
    const uint4 *cp = reinterpret_cast<const uint4 *>(fp - rs);
    const int nch = (rs + static_cast<int>(len) + 15) >> 4;

    uint4 v[NCH];
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = k * LPF + gl;
      v[k] = (c < nch) ? cp[c] : make_uint4(0, 0, 0, 0);
    }

    // stage the header window; one wave's LDS accesses execute in issue order,
    // so only the compiler has to be kept from moving the reads above the writes
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = k * LPF + gl;
      if (k * LPF < kHdrChunks && c < kHdrChunks && c < nch) hdr[wv][grp][c] = v[k];
    }
    compiler_barrier();
    const uint8_t *h = reinterpret_cast<const uint8_t *>(&hdr[wv][grp][0]) + rs;

    int32_t verdict;
    int u = 0;
    bool do_sum = false;
    if (len < 14) {
      verdict = -1;                                   // :34-37
    } else if (h[12] != 0x08 || h[13] != 0x00) {
      verdict = 0;                                    // :39-41
    } else if (len < 34) {
      verdict = -1;                                   // :43-46
    } else if (h[23] != 17) {
      verdict = 0;                                    // :48-50
    } else {
      u = 14 + ((h[14] & 0x0f) << 2);                 // :52, ihl unvalidated
      if (u + 8 > static_cast<int>(len)) {
        verdict = -1;                                 // :53-55
      } else {
        verdict = args.fwd_verdict;                   // :110-111
        do_sum = true;
      }
    }

    if (do_sum) {
      auto le16 = [&](int i) -> uint32_t { return h[i] | (static_cast<uint32_t>(h[i + 1]) << 8); };
      // :57-65 pseudo-header (read before the check is cleared)
      uint32_t s = le16(26) + le16(28) + le16(30) + le16(32) + 0x1100u + le16(u + 4);
      const uint32_t old_check = le16(u + 6);         // counted as 0 (:68)

      const int lo = rs + u;
      const int hi = rs + static_cast<int>(len);
      const uint32_t wl = (lo & 1) ? 0x01000100u : 0x00010001u;
      const uint32_t wh = wl << 8 | wl >> 24;
      uint32_t acc_lo = 0, acc_hi = 0;
#pragma unroll
      for (int k = 0; k < NCH; ++k) chunk_sum(v[k], (k * LPF + gl) * 16, lo, hi, wl, wh, acc_lo, acc_hi);
      for (int p = SPAN; p < nch; p += SPAN) {        // frames longer than one pass
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
          const int c = p + k * LPF + gl;
          v[k] = (c < nch) ? cp[c] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < NCH; ++k) chunk_sum(v[k], (p + k * LPF + gl) * 16, lo, hi, wl, wh, acc_lo, acc_hi);
      }
      uint32_t P = group_sum<LPF>(acc_lo + (acc_hi << 8));
      P -= old_check;
      s += args.payload_mult * P;                     // :92-103, iterations in closed form
      const uint16_t c = static_cast<uint16_t>(~static_cast<uint16_t>((s & 0xffffu) + (s >> 16)));  // :105-106
      if (gl == 0) {                                  // :108
        fp[u + 6] = static_cast<uint8_t>(c & 0xff);
        fp[u + 7] = static_cast<uint8_t>(c >> 8);
      }
    }
    if (gl == 0) args.verdicts[f] = verdict;
    // the next iteration rewrites this group's LDS window
    compiler_barrier();
    d = dn;
  }
}

// ---- host side -------------------------------------------------------------

thread_local char g_last_error[256] = "";

void set_error(hipError_t e, const char *where) {
  snprintf(g_last_error, sizeof(g_last_error), "%s: %s", where, hipGetErrorString(e));
}

struct DeviceInfo {
  int cus = 0;
  bool ok = false;
};

DeviceInfo device_info(int dev) {
  static DeviceInfo cache[64];
  if (dev < 0 || dev >= 64) return DeviceInfo{};
  if (!cache[dev].ok) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0) {
      cache[dev].cus = cus;
      cache[dev].ok = true;
    }
  }
  return cache[dev];
}

template <int LPF, int NCH>
int launch(const KernelArgs &a, hipStream_t stream, int blocks_per_cu) {
  constexpr int G = kWave / LPF;
  constexpr int frames_per_block = kWavesPerBlock * G;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) { set_error(e, "hipGetDevice"); return -EIO; }
  const DeviceInfo di = device_info(dev);
  const uint32_t cap = static_cast<uint32_t>((di.ok ? di.cus : 256) * blocks_per_cu);
  const uint32_t need = (a.n + frames_per_block - 1) / frames_per_block;
  const uint32_t blocks = need < cap ? need : cap;
  hipLaunchKernelGGL((checksum_kernel<LPF, NCH>), dim3(blocks), dim3(kBlock), 0, stream, a);
  e = hipGetLastError();
  if (e != hipSuccess) { set_error(e, "checksum_kernel launch"); return -EIO; }
  return 0;
}

}  // namespace xsknf_gpu

extern "C" {

uint32_t xsknf_gpu_version(void) { return (0u << 16) | 1u; }

int xsknf_gpu_device_count(int *count) {
  if (!count) return -EINVAL;
  hipError_t e = hipGetDeviceCount(count);
  if (e != hipSuccess) { xsknf_gpu::set_error(e, "hipGetDeviceCount"); *count = 0; return -ENODEV; }
  return 0;
}

const char *xsknf_gpu_last_error(void) { return xsknf_gpu::g_last_error; }

int xsknf_gpu_checksum_batch(uint8_t *umem, uint64_t umem_size, const struct xsknf_gpu_desc *descs,
                             uint32_t n, uint32_t ingress_ifindex, const struct xsknf_csum_opts *opts,
                             int32_t *verdicts, uint32_t frame_len_hint, void *stream) {
  using namespace xsknf_gpu;
  if (!opts || opts->reserved != 0) return -EINVAL;
  if (opts->action != XSKNF_CSUM_ACTION_REDIRECT && opts->action != XSKNF_CSUM_ACTION_DROP) return -EINVAL;
  if (opts->action == XSKNF_CSUM_ACTION_REDIRECT && opts->num_interfaces == 0) return -EINVAL;
  if (n == 0) return 0;
  if (!umem || !descs || !verdicts) return -EINVAL;

  KernelArgs a;
  a.umem = umem;
  a.umem_size = umem_size;
  a.descs = descs;
  a.verdicts = verdicts;
  a.n = n;
  a.payload_mult = opts->csum_iterations > 0 ? static_cast<uint32_t>(opts->csum_iterations) : 0u;
  a.fwd_verdict = opts->action == XSKNF_CSUM_ACTION_REDIRECT
                      ? static_cast<int32_t>((ingress_ifindex + 1u) % opts->num_interfaces)
                      : -1;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint32_t hint = frame_len_hint ? frame_len_hint : 2048u;
  // size classes: one pass must cover hint + 15 bytes of 16-byte misalignment
  if (hint + 15 <= 128) return launch<4, 2>(a, s, 8);
  if (hint + 15 <= 512) return launch<16, 2>(a, s, 8);
  if (hint + 15 <= 1536) return launch<32, 3>(a, s, 8);
  if (hint + 15 <= 4096) return launch<64, 4>(a, s, 8);
  return launch<64, 9>(a, s, 8);
}

}  // extern "C"
