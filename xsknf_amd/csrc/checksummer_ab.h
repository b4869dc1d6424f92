// checksummer_ab.h -- A/B-only launch shapes and knobs of checksummer.hip.
//
// Included only by A/B builds (`make ab` -> build/ab/libxsknf_gpu.so, -DXSKNF_AB;
// tools/tune.py, tools/ab_*.sh): nothing here is in the product library.  The
// product translation unit sees no-op stand-ins for the knobs and an empty
// XSKNF_AB_VARIANTS.  The records of every shape below are in
// profiles/r0*/ab* and DESIGN_HISTORY.md.
#pragma once
#include <stdio.h>
#include <stdlib.h>

namespace xsknf_gpu {

// XSKNF_AB_OCCUPANCY=1: print each kernel's blocks per CU as the launches size their grids
inline void ab_note_occupancy(const void *kernel, int threads, int blocks) {
  if (getenv("XSKNF_AB_OCCUPANCY")) fprintf(stderr, "occupancy %p x %d threads: %d blocks per CU\n", kernel, threads, blocks);
}

// XSKNF_SCATTER_BPC=N: blocks per CU of the scatter_checks pass
inline int ab_scatter_bpc(int dflt) {
  static const int bpc = getenv("XSKNF_SCATTER_BPC") ? atoi(getenv("XSKNF_SCATTER_BPC")) : dflt;
  return bpc > 0 ? bpc : dflt;
}

// XSKNF_AB_NO_GRID_BOUND=1: launch_split leaves out the grid bound that keeps a
// pool block's units within its waves' patch lists (tests/test_gpu_parity.py
// drives the kernel's own guard for units past the lists with it)
inline bool ab_no_grid_bound() {
  static const bool off = getenv("XSKNF_AB_NO_GRID_BOUND") != nullptr;
  return off;
}

}  // namespace xsknf_gpu

// Variant constructors of the A/B-only kernels (checksummer.hip's Variant table)
// lane kernel, one 16-wave block per CU with the tile pool (window field 32)
#define XSKNF_LP(N, S) {1, N, S, 0, &launch_lane<N, S, 16>, XSKNF_GPU_KERNEL_AUTO, 32}
// lane kernel with the transposed (coalesced) window load (window field 512)
#define XSKNF_LT(N, S) {1, N, S, 0, &launch_lane<N, S, kWavesPerBlock, 1, 1>, XSKNF_GPU_KERNEL_AUTO, 512}
// (A/B) the pooled lane kernel with the per-tile transposed windows (window field 1056)
#define XSKNF_LPA(N, S) {1, N, S, 0, &launch_lane<N, S, 16, 4, 2>, XSKNF_GPU_KERNEL_AUTO, 1056}
// (A/B) lane kernel held to WPE waves per SIMD (window field 64 + 256 * WPE)
#define XSKNF_LW(N, S, WPE) {1, N, S, 0, &launch_lane<N, S, kWavesPerBlock, WPE>, XSKNF_GPU_KERNEL_AUTO, 64 + 256 * WPE}

// A/B material, appended to the product's Variant table
#define XSKNF_AB_VARIANTS \
    /* A/B material (`make ab` -> build/ab/libxsknf_gpu.so; tools/tune.py), not in the product library */ \
    XSKNF_S(4, 16, 2, 2, 0), XSKNF_S(4, 16, 2, 1, 0), XSKNF_S(4, 8, 4, 2, 0), XSKNF_S(4, 32, 1, 2, 0), \
    XSKNF_S(4, 16, 4, 1, 0), XSKNF_S(5, 16, 2, 2, 0), XSKNF_S(4, 64, 2, 1, 0), XSKNF_S(4, 32, 2, 1, 0), \
    XSKNF_S(7, 16, 2, 1, 0), XSKNF_S(4, 16, 3, 1, 0), XSKNF_S(4, 8, 2, 2, 0), \
    XSKNF_S(4, 16, 2, 1, 1), XSKNF_S(4, 16, 3, 1, 1), \
    XSKNF_S(4, 16, 4, 1, 1), XSKNF_S(4, 32, 2, 1, 1), XSKNF_S(4, 32, 3, 1, 1), \
    XSKNF_S(8, 32, 3, 1, 1), XSKNF_S(8, 16, 2, 1, 1), XSKNF_S(8, 16, 4, 1, 1), \
    XSKNF_SC(16, 2, 3),   /* (jumbo in one 12-wave block per CU: 1520 vs 1456 us, r02 ab_pool_jumbo; removed r05) */ \
    XSKNF_LP(5, 2),   /* lane kernel with the tile pool: 64 B 59.65 vs 59.51 us, a tie (r02 ab_pool_lane.jsonl) */ \
    /* ... in 64-frame units (r05 ab_lane_pool / r05c): 64 B 58.8-59.1 vs 58.5-58.7 static (both write-through), */ \
    /* packed 64 B 37.3 vs 38.0-38.3, packed NIC 20.1-20.4 vs 22.4-22.7 */ \
    XSKNF_LP(5, 1), \
    XSKNF_LPA(5, 1), XSKNF_LPA(5, 2), \
    /* transposed window loads (r04 ab_lane_transposed*.jsonl): aligned 64 B NIC -1 us, worst case +0.3, */ \
    /* packed (-u) frames +1 us; per tile by the frames' spread: worst case +2 us (4 waves per SIMD forced); */ \
    /* round 5, with the write-through sectors (ab_matrix_r05l): all transposed 57.1-57.7 vs 58.2-58.8 us, */ \
    /* packed NIC +1 us; per tile (XSKNF_LA(5, 2)) 56.7-57.1: the product's since */ \
    XSKNF_LT(5, 2), XSKNF_LT(4, 2), XSKNF_LT(5, 1), XSKNF_LA(5, 1), \
    XSKNF_LA(5, 4), XSKNF_LA(4, 2),   /* (r05y: 62.8-63.1 and 57.3-57.9 vs 57.0-57.6 us) */ \
    XSKNF_S(8, 16, 3, 2, 1),   /* long-frame batches: 1500 B -1..2 %; out of the product (DESIGN 3, r02 fault) */ \
    XSKNF_L(5, 4),     XSKNF_L(6, 2),     XSKNF_L(7, 2), \
    XSKNF_L(4, 1),     XSKNF_L(4, 2),     XSKNF_L(5, 1),   /* fewer VGPRs, more waves (r03 64 B A/B) */ \
    XSKNF_LW(4, 1, 8), XSKNF_LW(4, 2, 6), XSKNF_LW(5, 2, 6), XSKNF_LW(5, 1, 8), \
    XSKNF_V(4, 2, 2),  XSKNF_V(4, 2, 4), \
    XSKNF_V(8, 1, 2),  XSKNF_V(8, 1, 4),  XSKNF_V(8, 1, 8),  XSKNF_V(16, 1, 4), XSKNF_V(16, 2, 4), \
    XSKNF_V(16, 2, 8), XSKNF_V(32, 2, 4), XSKNF_V(32, 3, 4), XSKNF_V(32, 3, 8), \
    XSKNF_V(64, 2, 8), XSKNF_V(64, 4, 4), XSKNF_V(64, 9, 2), XSKNF_V(64, 9, 4), \

