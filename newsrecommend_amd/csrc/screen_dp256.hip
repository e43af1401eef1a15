// screen_dp256.hip — screen_kernel instantiations for padded dim 256 (screen.h);
// one translation unit per padded dimension so the build compiles them in parallel.
#include "screen.h"

namespace nrk {
NRK_SCREEN_DP(256)

screen_fn pick_screen_dp256_w8(int M, bool l2, int mode) {
  // IP: epilogue deferred into the next MFMA chain (configs[4] retrieve
  // 21.7 -> 19.8 ms), 64-item tiles (128 would spill); L2 keeps the direct
  // epilogue.  The k = 200 form (M = 16) reads the corpus once (FETCH_SIZE
  // 5.3 GB per launch at 10M x 256, profiles/r02_pmc_screen_k200.json); its
  // cost over the k = 5 form is the lane-list insertions.
  if (mode == 1)
    return l2 ? screen_kernel<256, 1, 1, 8, true, 1, false> : screen_kernel<256, 1, 1, 8, false, 1, false, true, 64>;
  if (M == 4)
    return l2 ? screen_kernel<256, 1, 4, 8, true, 0, false> : screen_kernel<256, 1, 4, 8, false, 0, false, true, 64>;
  return l2 ? screen_kernel<256, 1, 16, 8, true, 0, false> : screen_kernel<256, 1, 16, 8, false, 0, false, true, 64>;
}
}  // namespace nrk
