// screen_dp64.hip — screen_kernel instantiations for padded dim 64 (screen.h);
// one translation unit per padded dimension so the build compiles them in parallel.
#include "screen.h"

namespace nrk {
NRK_SCREEN_DP(64)
}  // namespace nrk
