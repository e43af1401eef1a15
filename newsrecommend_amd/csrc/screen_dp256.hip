// screen_dp256.hip — screen_kernel instantiations for padded dim 256 (screen.h);
// one translation unit per padded dimension so the build compiles them in parallel.
#include "screen16.h"

namespace nrk {
NRK_SCREEN_DP(256)

// 16x16x32 main pass at DP = 256 (8 waves, 64-item tiles, sched_group_barrier
// interleave).  M = 4 (N1): 15.69 ms vs 15.82 for the 32x32x16 kernel (10M x 256,
// k = 5; the compiler's own schedule 15.97).  M = 16 (k = 200): the full next-
// sub-tile prefetch spills 32 VGPRs beside the lists (34.8 vs 16.7 ms) and no
// prefetch exposes the LDS latency (17.40 vs 15.87 ms); a 2-step fragment ring
// over three LDS buffers fits (2 spills, outside the chain): 15.89 vs 16.41 ms
// for the 32x32x16 kernel (4-step ring 16.19), same ids (profiles/r04_k200_ring_ab.log).
screen_fn pick_screen16_dp256_w8(int M) {
  if (M == 16) return screen16_kernel<256, 1, 16, 8, 64, true, 2>;
  return M == 4 ? screen16_kernel<256, 1, 4, 8, 64, true> : nullptr;
}

screen_fn pick_screen_dp256_w8(int M, bool l2, int mode) {
  // IP: epilogue deferred into the next MFMA chain (configs[4] retrieve
  // 21.7 -> 19.8 ms), 64-item tiles (128 would spill); L2 keeps the direct
  // epilogue.  The k = 200 form (M = 16) fetches 9.0-9.2 GB per launch at
  // 10M x 256 under bench.py (its user-profile queries; 5.26 GB with corpus-row
  // queries: profiles/r03_k200_query_distribution.log) against the 5.12 GB
  // corpus (most likely the 16 query tiles sharing a chunk progress unevenly
  // with these queries and re-fetch rows that left L2).  It runs at 560 GB/s, MFMA-bound
  // (16.0 ms with the profile queries, 16.5 ms with corpus rows); its cost over
  // the k = 5 form is the lane-list insertions.
  if (mode == 1)
    return l2 ? screen_kernel<256, 1, 1, 8, true, 1, false> : screen_kernel<256, 1, 1, 8, false, 1, false, true, 64>;
  if (M == 4)
    return l2 ? screen_kernel<256, 1, 4, 8, true, 0, false> : screen_kernel<256, 1, 4, 8, false, 0, false, true, 64>;
  return l2 ? screen_kernel<256, 1, 16, 8, true, 0, false> : screen_kernel<256, 1, 16, 8, false, 0, false, true, 64>;
}
}  // namespace nrk
