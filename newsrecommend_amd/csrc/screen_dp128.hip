// screen_dp128.hip — screen_kernel instantiations for padded dim 128 (screen.h);
// one translation unit per padded dimension so the build compiles them in parallel.
#include "screen16.h"

namespace nrk {
NRK_SCREEN_DP(128)

// 16x16x32 main pass (screen16.h), the k <= 8 form only (2 query tiles, M = 4).
// A/B on one box (tools/bench_screen.py, configs[1]): 128-item tiles with the
// compiler's own schedule 0.810 ms vs the 32x32x16 kernel's 0.830 ms (with
// sched_group_barrier interleaving 0.812, 64-item tiles 0.817: not kept).
// M = 8 / 16 keep the 32x32x16 kernel.
screen_fn pick_screen16_dp128(int qt, int M) {
  if (M != 4 || qt != 2) return nullptr;
  return screen16_kernel<128, 2, 4, 4, 128, false>;
}

// IVF collect (MODE 3), two query tiles per wave (256 probing queries per work
// item, as the 32x32x16 form), 64-item tiles (L2 at configs[3]: 3.04 vs 3.10 ms
// for 128-item tiles, profiles/r04_ivf_collect16_tiles_chunks.log; the inner
// product's 128-item form spills), three tile buffers (with the DMA issued from
// inline assembly: 2.70 ms vs 2.80 for two and four, r04_ivf_collect16_nb_ab.log).
screen_fn pick_collect16_dp128(bool l2) {
  return l2 ? screen16_collect_kernel<128, 2, 4, 64, true, 3> : screen16_collect_kernel<128, 2, 4, 64, false, 3>;
}
}  // namespace nrk
