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
constexpr int kHdrChunks = 7;   // window chunks 0..6 hold frame bytes [0, 97) at any 16-byte phase
constexpr int kSlotBytes = 128; // per-frame LDS slot: 16 B lead-in (shift by -rs) + 7 chunks

__device__ __forceinline__ uint64_t umem_offset(uint64_t addr) {
  return (addr & XSKNF_GPU_UNALIGNED_BUF_ADDR_MASK) + (addr >> XSKNF_GPU_UNALIGNED_BUF_OFFSET_SHIFT);
}

// 0x01 in every byte b of the dword at window offset x with lo <= x+b < hi.
// (bytes [a, b) of a dword, a/b clamped to 0..4: two 64-bit shifts of 0x01010101)
__device__ __forceinline__ uint32_t byte_ones(int lo, int hi, int x) {
  const int a8 = min(max(8 * (lo - x), 0), 32);
  const int b8 = min(max(8 * (hi - x), 0), 32);
  const uint32_t below_b = static_cast<uint32_t>((0x01010101ull << b8) >> 32);
  const uint32_t from_a = static_cast<uint32_t>(0x01010101ull << a8);
  return below_b & from_a;
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

// write-only sink for the unconditional stores of frames that write nothing
__device__ uint32_t g_sink[4];

struct KernelArgs {
  uint8_t *umem;
  uint64_t umem_size;
  const xsknf_gpu_desc *descs;
  int32_t *verdicts;
  uint32_t n;
  uint32_t payload_mult;   // max(csum_iterations, 0)
  int32_t fwd_verdict;     // REDIRECT ? (ingress+1) % n_if : -1
  const uint4 *dummy;      // readable 16-byte block for frames that need no bytes
  uint32_t defer;          // 1: park check records in `verdicts`, scatter in a 2nd pass
};

// Two-phase stores.  Rewriting 2 bytes in every frame WHILE the frames stream
// in costs ~25 % of the read bandwidth on MI355X (1M scattered writes mixed into
// the read stream; measured with tools/hbm_probe: 270 -> 346 us at 1500 B),
// while the same writes as a separate write-only pass take ~15 us.  So phase 1
// only reads the UMEM and parks, per frame, either its final verdict or a check
// record in verdicts[f]; phase 2 (scatter_checks) writes the check bytes and
// the final verdict.  Records are tagged 01 in bits 31..30, which no verdict
// (-1 or 0..XSKNF_MAX_INTERFACES-1) has.
constexpr uint32_t kRecTag = 0x40000000u;
constexpr uint32_t kRecTagMask = 0xC0000000u;

__device__ __forceinline__ int32_t make_record(int u, uint32_t check) {
  return static_cast<int32_t>(kRecTag | (static_cast<uint32_t>(u) << 16) | (check & 0xffffu));
}

// Where a frame's bytes are and which 16-byte chunks cover them.  Frames that
// need no bytes (len < 14, or a descriptor outside the UMEM) point at a dummy
// 16-byte block so that every chunk load of the pipeline can be unconditional.
struct FrameRef {
  const uint4 *cp;   // 16-byte aligned window start (cp <= fp)
  uint8_t *fp;       // first byte of the frame
  int rs;            // fp - cp, 0..15
  int len;
  int nch;           // chunks in the window, >= 1
  bool exists;       // index < n
  bool live;         // exists, in range and len >= 14
};

__device__ __forceinline__ FrameRef make_ref(const KernelArgs &a, const xsknf_gpu_desc &d, bool exists) {
  FrameRef r;
  const uint64_t off = umem_offset(d.addr);
  const uint32_t len = d.len;
  const bool in_range = off <= a.umem_size && len <= a.umem_size - off;
  r.exists = exists;
  r.live = exists && in_range && len >= 14;
  r.len = static_cast<int>(len);
  if (r.live) {
    r.fp = a.umem + off;
    r.rs = static_cast<int>(reinterpret_cast<uintptr_t>(r.fp) & 15);
    r.cp = reinterpret_cast<const uint4 *>(r.fp - r.rs);
    r.nch = (r.rs + r.len + 15) >> 4;
  } else {
    r.fp = a.umem;
    r.rs = 0;
    r.cp = a.dummy;
    r.nch = 1;
  }
  return r;
}

// Issue this lane's NCH chunk loads of pass `p0` (chunk index clamped into the
// window: lanes past the end re-read the last chunk, which costs no HBM bytes
// and keeps the loads free of branches so the next frame's loads stay in
// flight while the current frame is reduced).
template <int LPF, int NCH>
__device__ __forceinline__ void load_pass(const FrameRef &r, int p0, int gl, uint4 (&v)[NCH]) {
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = min(p0 + k * LPF + gl, r.nch - 1);
    v[k] = r.cp[c];
  }
}

// The two stores a frame produces (check bytes, verdict).  They are issued at
// the start of the NEXT step, before that step's loads, and by every lane
// unconditionally (lanes of a group write identical values to one address;
// frames with nothing to write aim at a sink word).  No store then sits
// between a frame's loads and their use, nor inside a branch, so the compiler
// can wait for exactly the loads it needs instead of draining vmcnt.
struct PendingStores {
  uint16_t *cdst;
  int32_t *vdst;
  uint32_t check;
  int32_t verdict;
};

__device__ __forceinline__ PendingStores sink_stores() {
  return PendingStores{reinterpret_cast<uint16_t *>(g_sink), reinterpret_cast<int32_t *>(g_sink + 1), 0u, 0};
}

__device__ __forceinline__ void issue(const PendingStores &ps, uint32_t defer) {
  if (!defer) *ps.cdst = static_cast<uint16_t>(ps.check);      // :108
  *ps.vdst = ps.verdict;
}

template <int LPF, int NCH>
__device__ __forceinline__ PendingStores process_frame(const KernelArgs &args, const FrameRef &r,
                                                       uint32_t f, const uint4 (&v)[NCH],
                                                       uint8_t *slot, int gl) {
  constexpr int SPAN = LPF * NCH;
  // Stage window chunks 0..6 in LDS shifted by -rs, so frame byte i sits at
  // slot[16 + i] whatever the frame's alignment: the header fields are then at
  // fixed offsets.  One wave's LDS accesses execute in issue order; only the
  // compiler must be kept from moving the reads above the writes.
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = k * LPF + gl;
    if (k * LPF < kHdrChunks && c < kHdrChunks)
      *reinterpret_cast<uint4 *>(slot + 16 + 16 * c - r.rs) = v[k];
  }
  compiler_barrier();
  const uint4 q0 = *reinterpret_cast<const uint4 *>(slot + 16);   // f[0..15]
  const uint4 q1 = *reinterpret_cast<const uint4 *>(slot + 32);   // f[16..31]
  const uint32_t w8 = *reinterpret_cast<const uint32_t *>(slot + 48);  // f[32..35]
  const int ihl = (q0.w >> 16) & 0x0f;                             // f[14] low nibble
  const int u = 14 + 4 * ihl;                                      // :52, ihl unvalidated
  const uint32_t wa = *reinterpret_cast<const uint32_t *>(slot + 16 + u + 2);  // f[u+2..u+5]
  const uint32_t wb = *reinterpret_cast<const uint32_t *>(slot + 16 + u + 6);  // f[u+6..u+9]
  compiler_barrier();

  const bool ipv4 = (q0.w & 0xffffu) == 0x0008u;                  // f[12..13] == 08 00
  const bool udp = (q1.y >> 24) == 17u;                           // f[23]
  int32_t verdict;
  bool do_sum = false;
  if (!r.live) {
    verdict = -1;                                   // :34-37 (and out-of-range descriptors)
  } else if (!ipv4) {
    verdict = 0;                                    // :39-41
  } else if (r.len < 34) {
    verdict = -1;                                   // :43-46
  } else if (!udp) {
    verdict = 0;                                    // :48-50
  } else if (u + 8 > r.len) {
    verdict = -1;                                   // :53-55
  } else {
    verdict = args.fwd_verdict;                     // :110-111
    do_sum = true;
  }

  // Pass-0 partial sums on every path (also for frames that end up unsummed):
  // every loaded register is consumed unconditionally, so no load of this frame
  // can still be in flight at the loop back-edge.
  const int lo = r.rs + u;
  const int hi = r.rs + r.len;
  const uint32_t wl = (lo & 1) ? 0x01000100u : 0x00010001u;
  const uint32_t wh = wl << 8 | wl >> 24;
  uint32_t acc_lo = 0, acc_hi = 0;
#pragma unroll
  for (int k = 0; k < NCH; ++k) chunk_sum(v[k], (k * LPF + gl) * 16, lo, hi, wl, wh, acc_lo, acc_hi);

  uint16_t check = 0;
  if (do_sum) {
    // :57-65 pseudo-header, read before the check is cleared:
    // le16(26) + le16(28) + le16(30) + le16(32) + 17<<8 + le16(u+4)
    uint32_t s = (q1.z >> 16) + (q1.w & 0xffffu) + (q1.w >> 16) + (w8 & 0xffffu) + 0x1100u + (wa >> 16);
    const uint32_t old_check = wb & 0xffffu;        // counted as 0 (:68)
    for (int p = SPAN; p < r.nch; p += SPAN) {      // frames longer than one pass
      uint4 t[NCH];
      load_pass<LPF, NCH>(r, p, gl, t);
#pragma unroll
      for (int k = 0; k < NCH; ++k) chunk_sum(t[k], (p + k * LPF + gl) * 16, lo, hi, wl, wh, acc_lo, acc_hi);
    }
    uint32_t P = group_sum<LPF>(acc_lo + (acc_hi << 8));
    P -= old_check;
    s += args.payload_mult * P;                     // :92-103, iterations in closed form
    check = static_cast<uint16_t>(~static_cast<uint16_t>((s & 0xffffu) + (s >> 16)));  // :105-106
  }
  PendingStores ps;
  ps.cdst = do_sum ? reinterpret_cast<uint16_t *>(r.fp + u + 6) : reinterpret_cast<uint16_t *>(g_sink);
  ps.vdst = r.exists ? args.verdicts + f : reinterpret_cast<int32_t *>(g_sink + 1);
  ps.check = check;
  ps.verdict = (args.defer && do_sum) ? make_record(u, check) : verdict;
  compiler_barrier();   // the next frame rewrites this group's LDS slot
  return ps;
}

// The G descriptors of one wave's frames are contiguous, so they are fetched
// with wave-uniform scalar loads (s_load, counted by lgkmcnt): the descriptor
// prefetch then never forces the compiler to drain the vector-memory counter
// that the chunk loads of the next frame are still running on.
typedef const __attribute__((address_space(4))) xsknf_gpu_desc *const_desc_ptr;

template <int G>
struct DescSet {
  uint64_t addr[G];
  uint32_t len[G];
};

template <int G>
__device__ __forceinline__ DescSet<G> load_descs(const KernelArgs &a, uint32_t wf, uint32_t last) {
  DescSet<G> ds;
  const const_desc_ptr cd = (const_desc_ptr)(reinterpret_cast<uintptr_t>(a.descs));
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint32_t i = min(wf + g, last);
    ds.addr[g] = cd[i].addr;
    ds.len[g] = cd[i].len;
  }
  return ds;
}

template <int G>
__device__ __forceinline__ xsknf_gpu_desc pick(const DescSet<G> &ds, int grp) {
  xsknf_gpu_desc d;
  d.addr = ds.addr[0];
  d.len = ds.len[0];
#pragma unroll
  for (int g = 1; g < G; ++g) {
    d.addr = grp == g ? ds.addr[g] : d.addr;
    d.len = grp == g ? ds.len[g] : d.len;
  }
  d.options = 0;
  return d;
}

template <int LPF, int NCH, int U>
__global__ __launch_bounds__(kBlock) void checksum_kernel(const KernelArgs args) {
  static_assert(kWave % LPF == 0, "LPF must divide the wave");
  static_assert(LPF * NCH >= kHdrChunks, "pass 0 must cover the header window");
  constexpr int G = kWave / LPF;     // frame groups per wave
  constexpr int FW = G * U;          // frames per wave per iteration
  static_assert(FW <= 8, "descriptor prefetch is held in SGPRs");

  __shared__ __attribute__((aligned(16))) uint8_t lds[kWavesPerBlock][G][kSlotBytes];

  const int lane = threadIdx.x & (kWave - 1);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int grp = lane / LPF;
  const int gl = lane % LPF;
  uint8_t *slot = &lds[wv][grp][0];
  const uint32_t wstride = gridDim.x * kWavesPerBlock * FW;   // frames per grid sweep
  const uint32_t last = args.n - 1;
  uint32_t wf = (blockIdx.x * kWavesPerBlock + wv) * FW;      // this wave's first frame

  // Each iteration issues the chunk loads of U frames per group at once, then
  // reduces them one by one (frame u+1's loads stay in flight while frame u is
  // parsed and summed).  Nothing is carried in flight across the back-edge:
  // descriptors for the next iteration are prefetched with scalar loads.
  DescSet<FW> dcur = load_descs<FW>(args, wf, last);
  while (wf < args.n) {          // wave-uniform loop control
    FrameRef ref[U];
    uint4 v[U][NCH];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t f = wf + u * G + grp;
      ref[u] = make_ref(args, pick<FW>(dcur, u * G + grp), f < args.n);
      load_pass<LPF, NCH>(ref[u], 0, gl, v[u]);
    }
    const uint32_t wn = wf + wstride;
    dcur = load_descs<FW>(args, wn, last);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      issue(process_frame<LPF, NCH>(args, ref[u], wf + u * G + grp, v[u], slot, gl), args.defer);
    }
    wf = wn;
  }
}

// ---- LDS-DMA ring variant --------------------------------------------------
//
// Each wave streams its frames through a private ring of R slots in LDS filled
// by global_load_lds_dwordx4 (LDS-DMA: 16 B per lane straight into LDS, no VGPR
// destination).  At step i the wave issues the DMA of step i+R-1 and then waits
// -- with an explicitly counted vmcnt -- only for step i's slot, so R-1 steps of
// loads stay in flight while step i is parsed, summed and reduced, and the
// loads cost no registers (occupancy stays high).  The DMA is issued from
// inline asm because the compiler drains vmcnt to 0 before every LDS read once
// it sees an LDS-DMA in flight; the waits here count only this wave's own DMAs
// that are younger than the slot being read (other vector-memory operations
// can only make the wait stricter, never too weak).
//
// Slot layout: DMA instruction k of a step writes 1 KiB at slot + k*1024, lane l
// at +16*l, so group g's chunk c = k*LPF + gl sits at slot + k*1024 + g*LPF*16 +
// gl*16, and chunks 0..LPF-1 of a frame (bytes [0, 16*LPF - rs) of the frame,
// every header byte for LPF >= 8) are contiguous at slot + g*LPF*16.

__device__ __forceinline__ void dma16(const void *gaddr, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off"
               :: "v"(gaddr), "s"(lds_addr) : "memory", "m0");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits on gfx950");
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

__device__ __forceinline__ uint32_t lds_u32(uint32_t addr) {
  // may be unaligned: gfx950 LDS serves unaligned dword reads
  return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>(static_cast<uintptr_t>(addr));
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 lds_u128(uint32_t addr) {
  const u32x4 x = *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(static_cast<uintptr_t>(addr));
  return make_uint4(x.x, x.y, x.z, x.w);
}

// Group sum via DPP: the total lands in the group's LAST lane (lane LPF-1).
template <int LPF>
__device__ __forceinline__ uint32_t group_sum_last(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true);   // row_shr:4
  if constexpr (LPF >= 16) v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true);  // row_shr:8
  if constexpr (LPF >= 32) v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false); // row_bcast:15
  if constexpr (LPF >= 64) v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false); // row_bcast:31
  return v;
}

// Issue the NCH DMAs of one frame window per group into `slot` (chunk index
// clamped into the window, as in load_pass).
template <int LPF, int NCH>
__device__ __forceinline__ void dma_pass(const FrameRef &r, int gl, uint32_t slot) {
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = min(k * LPF + gl, r.nch - 1);
    dma16(r.cp + c, slot + k * 1024);
  }
}

// Parse + sum + reduce one frame per group from a landed slot; returns the
// frame's stores (issued by the group's last lane).
template <int LPF, int NCH>
__device__ __forceinline__ void process_slot(const KernelArgs &args, const FrameRef &r, uint32_t f,
                                             uint32_t slot, int grp, int gl, int lane) {
  constexpr int SPAN = LPF * NCH;
  const uint32_t hb = slot + grp * LPF * 16 + r.rs;        // frame byte i at hb + i
  const uint32_t w12 = lds_u32(hb + 12);                   // f[12..15]
  const uint32_t w20 = lds_u32(hb + 20);                   // f[20..23]
  const uint32_t w24 = lds_u32(hb + 24);                   // f[24..27]
  const uint32_t w28 = lds_u32(hb + 28);                   // f[28..31]
  const uint32_t w32 = lds_u32(hb + 32);                   // f[32..35]
  const int u = 14 + 4 * ((w12 >> 16) & 0x0f);             // :52, ihl unvalidated
  const uint32_t wu = lds_u32(hb + u + 4);                 // f[u+4..u+7]: udp len, old check
  uint4 v[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) v[k] = lds_u128(slot + k * 1024 + lane * 16);

  const bool ipv4 = (w12 & 0xffffu) == 0x0008u;           // f[12..13] == 08 00
  const bool udp = (w20 >> 24) == 17u;                     // f[23]
  int32_t verdict;
  bool do_sum = false;
  if (!r.live) {
    verdict = -1;                                   // :34-37 (and out-of-range descriptors)
  } else if (!ipv4) {
    verdict = 0;                                    // :39-41
  } else if (r.len < 34) {
    verdict = -1;                                   // :43-46
  } else if (!udp) {
    verdict = 0;                                    // :48-50
  } else if (u + 8 > r.len) {
    verdict = -1;                                   // :53-55
  } else {
    verdict = args.fwd_verdict;                     // :110-111
    do_sum = true;
  }

  const int lo = r.rs + u;
  const int hi = r.rs + r.len;
  const uint32_t wl = (lo & 1) ? 0x01000100u : 0x00010001u;
  const uint32_t wh = wl << 8 | wl >> 24;
  uint32_t acc_lo = 0, acc_hi = 0;
#pragma unroll
  for (int k = 0; k < NCH; ++k) chunk_sum(v[k], (k * LPF + gl) * 16, lo, hi, wl, wh, acc_lo, acc_hi);
  if (do_sum) {
    for (int p = SPAN; p < r.nch; p += SPAN) {      // frames longer than one pass: direct loads
      uint4 t[NCH];
      load_pass<LPF, NCH>(r, p, gl, t);
#pragma unroll
      for (int k = 0; k < NCH; ++k) chunk_sum(t[k], (p + k * LPF + gl) * 16, lo, hi, wl, wh, acc_lo, acc_hi);
    }
  }
  const uint32_t P = group_sum_last<LPF>(acc_lo + (acc_hi << 8)) - (wu >> 16);   // old check counted as 0 (:68)
  if (gl == LPF - 1 && r.exists) {
    if (do_sum) {
      // :57-65 pseudo-header: le16(26) + le16(28) + le16(30) + le16(32) + 17<<8 + le16(u+4)
      uint32_t s = (w24 >> 16) + (w28 & 0xffffu) + (w28 >> 16) + (w32 & 0xffffu) + 0x1100u + (wu & 0xffffu);
      s += args.payload_mult * P;                   // :92-103, iterations in closed form
      const uint16_t c = static_cast<uint16_t>(~static_cast<uint16_t>((s & 0xffffu) + (s >> 16)));  // :105-106
      if (args.defer) {
        verdict = make_record(u, c);
      } else {
        *reinterpret_cast<uint16_t *>(r.fp + u + 6) = c;   // :108
      }
    }
    args.verdicts[f] = verdict;
  }
}

template <int LPF, int NCH, int R>
__global__ __launch_bounds__(kBlock) void checksum_kernel_dma(const KernelArgs args) {
  static_assert(kWave % LPF == 0 && LPF >= 8, "header window must sit in chunk slot k = 0");
  static_assert(R >= 2 && R <= 4, "ring depth");
  static_assert((R - 1) * NCH < 64, "vmcnt range");
  constexpr int G = kWave / LPF;
  constexpr int SLOT = NCH * 1024;
  static_assert(G <= 8, "descriptor prefetch is held in SGPRs");

  __shared__ __attribute__((aligned(1024))) uint8_t ring[kWavesPerBlock][R][SLOT];

  const int lane = threadIdx.x & (kWave - 1);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int grp = lane / LPF;
  const int gl = lane % LPF;
  const uint32_t ring0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(&ring[wv][0][0]));
  const uint32_t wstride = gridDim.x * kWavesPerBlock * G;
  const uint32_t last = args.n - 1;
  const uint32_t w0 = (blockIdx.x * kWavesPerBlock + wv) * G;

  // frames of step j of this wave: w0 + j * wstride + grp
  FrameRef ref[R];
  // prologue: steps 0 .. R-2 in flight
#pragma unroll
  for (int j = 0; j < R - 1; ++j) {
    const uint32_t wf = w0 + j * wstride;
    ref[j] = make_ref(args, pick<G>(load_descs<G>(args, wf, last), grp), wf + grp < args.n);
    dma_pass<LPF, NCH>(ref[j], gl, ring0 + j * SLOT);
  }
  DescSet<G> dpre = load_descs<G>(args, w0 + (R - 1) * wstride, last);

  // Unrolled by R so ring slots and the per-step FrameRefs are static.
  uint32_t wf = w0;
  while (true) {
#pragma unroll
    for (int s = 0; s < R; ++s) {
      if (wf >= args.n) {        // wave-uniform exit; drain this wave's DMAs first
        wait_vmcnt<0>();
        return;
      }
      const int sn = (s + R - 1) % R;                  // slot of step i+R-1 (freed by step i-1)
      const uint32_t wn = wf + (R - 1) * wstride;
      ref[sn] = make_ref(args, pick<G>(dpre, grp), wn + grp < args.n);
      dpre = load_descs<G>(args, wn + wstride, last);
      dma_pass<LPF, NCH>(ref[sn], gl, ring0 + sn * SLOT);
      wait_vmcnt<(R - 1) * NCH>();                     // step i's slot has landed
      process_slot<LPF, NCH>(args, ref[s], wf + grp, ring0 + s * SLOT, grp, gl, lane);
      wf += wstride;
    }
  }
}

// Phase 2 of the two-phase stores: write the parked check bytes into the
// frames (checksummer_user.c:108) and the final verdicts (:110-111).
__global__ __launch_bounds__(kBlock) void scatter_checks(const KernelArgs args) {
  for (uint32_t f = blockIdx.x * kBlock + threadIdx.x; f < args.n; f += gridDim.x * kBlock) {
    const uint32_t rec = static_cast<uint32_t>(args.verdicts[f]);
    if ((rec & kRecTagMask) == kRecTag) {
      const uint64_t off = umem_offset(args.descs[f].addr);
      const uint32_t u = (rec >> 16) & 0x7f;
      *reinterpret_cast<uint16_t *>(args.umem + off + u + 6) = static_cast<uint16_t>(rec & 0xffffu);
      args.verdicts[f] = args.fwd_verdict;
    }
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

hipError_t launch_scatter(const KernelArgs &a, hipStream_t stream, const DeviceInfo &di) {
  const uint32_t cap = static_cast<uint32_t>((di.ok ? di.cus : 256) * 8);
  const uint32_t need = (a.n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(scatter_checks, dim3(need < cap ? need : cap), dim3(kBlock), 0, stream, a);
  return hipGetLastError();
}

template <int LPF, int NCH, int U>
int launch(const KernelArgs &a, hipStream_t stream, int blocks_per_cu) {
  constexpr int G = kWave / LPF;
  constexpr int frames_per_block = kWavesPerBlock * G * U;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) { set_error(e, "hipGetDevice"); return -EIO; }
  const DeviceInfo di = device_info(dev);
  const uint32_t cap = static_cast<uint32_t>((di.ok ? di.cus : 256) * blocks_per_cu);
  const uint32_t need = (a.n + frames_per_block - 1) / frames_per_block;
  const uint32_t blocks = need < cap ? need : cap;
  hipLaunchKernelGGL((checksum_kernel<LPF, NCH, U>), dim3(blocks), dim3(kBlock), 0, stream, a);
  e = hipGetLastError();
  if (e == hipSuccess && a.defer) e = launch_scatter(a, stream, di);
  if (e != hipSuccess) { set_error(e, "checksum_kernel launch"); return -EIO; }
  return 0;
}

template <int LPF, int NCH, int R>
int launch_dma(const KernelArgs &a, hipStream_t stream, int blocks_per_cu) {
  constexpr int G = kWave / LPF;
  constexpr int frames_per_block = kWavesPerBlock * G;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) { set_error(e, "hipGetDevice"); return -EIO; }
  const DeviceInfo di = device_info(dev);
  const uint32_t cap = static_cast<uint32_t>((di.ok ? di.cus : 256) * blocks_per_cu);
  const uint32_t need = (a.n + frames_per_block - 1) / frames_per_block;
  const uint32_t blocks = need < cap ? need : cap;
  hipLaunchKernelGGL((checksum_kernel_dma<LPF, NCH, R>), dim3(blocks), dim3(kBlock), 0, stream, a);
  e = hipGetLastError();
  if (e == hipSuccess && a.defer) e = launch_scatter(a, stream, di);
  if (e != hipSuccess) { set_error(e, "checksum_kernel_dma launch"); return -EIO; }
  return 0;
}

// Instantiated launch shapes: {lanes per frame, 16-B chunks per lane and pass,
// frames per group and iteration}.  The default picks one by frame_len_hint.
struct Variant {
  int lpf, nch, u, ring;
  int (*fn)(const KernelArgs &, hipStream_t, int);
};

#define XSKNF_V(L, N, U) {L, N, U, 0, &launch<L, N, U>}
#define XSKNF_D(L, N, R) {L, N, 1, R, &launch_dma<L, N, R>}
const Variant kVariants[] = {
    XSKNF_V(8, 1, 1),  XSKNF_V(16, 1, 1), XSKNF_V(16, 1, 2), XSKNF_V(16, 2, 1), XSKNF_V(16, 2, 2),
    XSKNF_V(32, 1, 1), XSKNF_V(32, 1, 2), XSKNF_V(32, 2, 1), XSKNF_V(32, 2, 2), XSKNF_V(32, 3, 1),
    XSKNF_V(32, 3, 2), XSKNF_V(64, 1, 1), XSKNF_V(64, 2, 1), XSKNF_V(64, 2, 2), XSKNF_V(64, 3, 1),
    XSKNF_V(64, 4, 1), XSKNF_V(64, 4, 2), XSKNF_V(64, 6, 1), XSKNF_V(64, 9, 1),
    XSKNF_D(8, 1, 3),  XSKNF_D(8, 1, 4),  XSKNF_D(16, 1, 3), XSKNF_D(16, 2, 3), XSKNF_D(32, 2, 3),
    XSKNF_D(32, 3, 2), XSKNF_D(32, 3, 3), XSKNF_D(64, 2, 3), XSKNF_D(64, 2, 4), XSKNF_D(64, 3, 3),
    XSKNF_D(64, 4, 2), XSKNF_D(64, 4, 3),
};
#undef XSKNF_V
#undef XSKNF_D

const Variant *find_variant(int lpf, int nch, int u, int ring) {
  for (const Variant &v : kVariants)
    if (v.lpf == lpf && v.nch == nch && v.ring == ring && (ring || v.u == u)) return &v;
  return nullptr;
}

// default shape for a length hint: one pass covers hint + 15 bytes of misalignment
void default_shape(uint32_t hint, int &lpf, int &nch, int &u) {
  if (hint + 15 <= 128) { lpf = 8; nch = 1; u = 1; }
  else if (hint + 15 <= 512) { lpf = 16; nch = 2; u = 2; }
  else if (hint + 15 <= 1536) { lpf = 32; nch = 3; u = 2; }
  else if (hint + 15 <= 4096) { lpf = 64; nch = 4; u = 2; }
  else { lpf = 64; nch = 9; u = 1; }
}

int prepare(KernelArgs &a, uint8_t *umem, uint64_t umem_size, const xsknf_gpu_desc *descs, uint32_t n,
            uint32_t ingress_ifindex, const xsknf_csum_opts *opts, int32_t *verdicts) {
  if (!opts || opts->reserved != 0) return -EINVAL;
  if (opts->action != XSKNF_CSUM_ACTION_REDIRECT && opts->action != XSKNF_CSUM_ACTION_DROP) return -EINVAL;
  if (opts->action == XSKNF_CSUM_ACTION_REDIRECT && opts->num_interfaces == 0) return -EINVAL;
  if (n == 0) return 1;
  if (!umem || !descs || !verdicts) return -EINVAL;
  a.umem = umem;
  a.umem_size = umem_size;
  a.descs = descs;
  a.verdicts = verdicts;
  a.n = n;
  a.payload_mult = opts->csum_iterations > 0 ? static_cast<uint32_t>(opts->csum_iterations) : 0u;
  // aligned-down descriptor address: inside the descriptor array's own page
  a.dummy = reinterpret_cast<const uint4 *>(reinterpret_cast<uintptr_t>(descs) & ~static_cast<uintptr_t>(15));
  a.fwd_verdict = opts->action == XSKNF_CSUM_ACTION_REDIRECT
                      ? static_cast<int32_t>((ingress_ifindex + 1u) % opts->num_interfaces)
                      : -1;
  a.defer = 1;
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
  KernelArgs a;
  const int rc = prepare(a, umem, umem_size, descs, n, ingress_ifindex, opts, verdicts);
  if (rc != 0) return rc < 0 ? rc : 0;
  int lpf, nch, u;
  default_shape(frame_len_hint ? frame_len_hint : 2048u, lpf, nch, u);
  return find_variant(lpf, nch, u, 0)->fn(a, static_cast<hipStream_t>(stream), 8);
}

int xsknf_gpu_checksum_batch_cfg(uint8_t *umem, uint64_t umem_size, const struct xsknf_gpu_desc *descs,
                                 uint32_t n, uint32_t ingress_ifindex, const struct xsknf_csum_opts *opts,
                                 int32_t *verdicts, const struct xsknf_gpu_launch_cfg *cfg, void *stream) {
  using namespace xsknf_gpu;
  if (!cfg || cfg->blocks_per_cu < 0 || cfg->blocks_per_cu > 64) return -EINVAL;
  const Variant *v = find_variant(cfg->lanes_per_frame, cfg->chunks_per_lane, cfg->frames_per_group,
                                  cfg->lds_ring);
  if (!v) return -EINVAL;
  if (cfg->fused_stores != 0 && cfg->fused_stores != 1) return -EINVAL;
  KernelArgs a;
  const int rc = prepare(a, umem, umem_size, descs, n, ingress_ifindex, opts, verdicts);
  if (rc != 0) return rc < 0 ? rc : 0;
  a.defer = cfg->fused_stores ? 0u : 1u;
  return v->fn(a, static_cast<hipStream_t>(stream), cfg->blocks_per_cu ? cfg->blocks_per_cu : 8);
}

int xsknf_gpu_default_launch_cfg(uint32_t frame_len_hint, struct xsknf_gpu_launch_cfg *cfg) {
  if (!cfg) return -EINVAL;
  int lpf, nch, u;
  xsknf_gpu::default_shape(frame_len_hint ? frame_len_hint : 2048u, lpf, nch, u);
  cfg->lanes_per_frame = lpf;
  cfg->chunks_per_lane = nch;
  cfg->frames_per_group = u;
  cfg->blocks_per_cu = 8;
  cfg->lds_ring = 0;
  cfg->fused_stores = 0;
  return 0;
}

}  // extern "C"
