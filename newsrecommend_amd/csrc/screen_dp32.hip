// screen_dp32.hip — screen_kernel instantiations for padded dim 32 (see screen.h).
#include "screen.h"

namespace nrk {
namespace {

static int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}

template <int DP, int QT, int M, bool L2, int MODE>
static screen_fn pick3() {
  if constexpr (DP == 128 && QT == 2 && M == 4 && !L2 && MODE == 0) {
    const int epi = env_int("NRK_SCREEN_EPI", 0);
    if (epi == 1) return screen_kernel<DP, QT, M, 4, L2, MODE, 1>;
    if (epi == 2) return screen_kernel<DP, QT, M, 4, L2, MODE, 2>;
  }
  // flat modes: epilogue deferred into the next MFMA chain (screen.h); not for
  // DP = 256, L2 with two query tiles, and the DP = 128 two-tile pre-pass
  // (the second accumulator set and the fragment prefetch spill there)
  if constexpr ((MODE == 3 || MODE == 4) && QT == 1 && DP < 256) {  // IVF collect / lane maxima
    if (env_int("NRK_IVF_DEFER", 0)) return screen_kernel<DP, QT, M, 4, L2, MODE, 0, false, true>;
  }
  if constexpr (MODE <= 1 && DP < 256 && !(L2 && QT == 2) && !(DP == 128 && QT == 2 && MODE == 1)) {
    if (env_int("NRK_SCREEN_DEFER", 1)) {
      if constexpr (MODE == 0 && !L2) {  // 128-item tiles: half the barriers (measured +9 %)
        if (env_int("NRK_SCREEN_TI", 128) == 128) return screen_kernel<DP, QT, M, 4, L2, MODE, 0, false, true, 128>;
      }
      return screen_kernel<DP, QT, M, 4, L2, MODE, 0, false, true>;
    }
  }
  // grouped A-fragment reads: default on for the IVF modes (measured), env override
  const int grp = env_int("NRK_AFRAG_GROUP", -1);
  const bool g = grp < 0 ? (MODE >= 2) : grp != 0;
  return g ? screen_kernel<DP, QT, M, 4, L2, MODE, 0, true> : screen_kernel<DP, QT, M, 4, L2, MODE, 0, false>;
}

template <int DP, bool L2, int MODE>
static screen_fn pick2(int qt, int M) {
  constexpr int Q2 = DP == 256 ? 1 : 2;  // DP=256 always runs one query tile per wave
  if (M == 4) return qt == 2 ? pick3<DP, Q2, 4, L2, MODE>() : pick3<DP, 1, 4, L2, MODE>();
  if (M == 8) return pick3<DP, 1, 8, L2, MODE>();
  return pick3<DP, 1, 16, L2, MODE>();
}

// mode: 0 main pass, 1 threshold pre-pass, 2 IVF list scan, 3 IVF collect, 4 IVF lane maxima
template <int DP, bool L2>
static screen_fn pick1(int qt, int M, int mode) {
  constexpr int Q2 = DP == 256 ? 1 : 2;
  if (mode == 1) return qt == 2 ? pick3<DP, Q2, 1, L2, 1>() : pick3<DP, 1, 1, L2, 1>();
  if (mode == 2) return pick2<DP, L2, 2>(qt, M);
  if (mode == 3) return qt == 2 ? pick3<DP, Q2, 1, L2, 3>() : pick3<DP, 1, 1, L2, 3>();
  if (mode == 4) return qt == 2 ? pick3<DP, Q2, 1, L2, 4>() : pick3<DP, 1, 1, L2, 4>();
  return pick2<DP, L2, 0>(qt, M);
}

}  // namespace

screen_fn pick_screen_dp32(int qt, int M, bool l2, int mode) {
  return l2 ? pick1<32, true>(qt, M, mode) : pick1<32, false>(qt, M, mode);
}

}  // namespace nrk
