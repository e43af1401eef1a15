// din_rerank.h — what the fused re-rank kernels share (din_rerank.hip: the
// per-chunk block kernel, the row projections; din_rerank_lane.hip: the
// wave-per-32-candidates projected kernel).
#pragma once
#include <hip/hip_runtime.h>

#include "nrk_common.h"

namespace nrk {
namespace rr {

constexpr int LP = 64;  // history rows held (L <= 64)

struct RerankArgs {
  const uint16_t* table;
  int64_t n_table;
  const int32_t* hist;  // [nU][L]
  int L, nU;
  const int32_t* cand;       // candidate rows
  const int64_t* cand_off;   // [nU] user u: cand[cand_off[u] .. + cand_len[u])
  const int32_t* cand_len;   // [nU]
  const int32_t* extra;      // [nU] appended candidate (< 0: a padded slot), or null
  const int64_t* out_off;    // [nU] logits of user u at out[out_off[u] ..]
  float* out;
  const uint16_t *W1q_hi, *W1q_lo, *W1k_hi, *W1k_lo;  // [A][d]
  const float* b1;                                    // [A]
  const float* w2;                                    // [A]
  const uint16_t *H1q_hi, *H1q_lo, *H1p_hi, *H1p_lo;  // [F][d]
  const float* c1;                                    // [F]
  const uint16_t *H2_hi, *H2_lo;                      // [F/2][F]
  const float* c2;                                    // [F/2]
  const float* h3;                                    // [F/2]
  float c3;
  int F;
  int* queue;  // user counter, zero at launch
  // projected candidates (PROJ): [U' (A) | Q1 (F)] f32 per candidate, cproj
  // parallel to cand, xproj [nU] for the extras (nrk_din_rerank_project), and
  // the history projected per slot: hproj [nU][L] x [P' (A) | R (F)] f32
  // (nrk_din_rerank_project_hist).  The PROJ kernel never reads the table, so
  // it serves bf16 and f32 tables alike.
  const float* cproj;
  const float* xproj;
  const float* hproj;
  const void* sgn;  // din_rerank_lane_kernel: sgn(w2) per P' / U' column (slice order) as f16, in the workspace
};

__device__ __forceinline__ void split_bf16(float x, short& hi, short& lo) {
  const __bf16 h = (__bf16)x;
  hi = __builtin_bit_cast(short, h);
  lo = __builtin_bit_cast(short, (__bf16)(x - (float)h));
}

// Geo<D, A>::col with A at run time
__device__ __forceinline__ int slice_col(int n, int A) {
  const int SL = A / 8, sj = n / SL, w = n % SL;
  const int p4 = SL == 16 ? ((w >> 2) + 2 * (sj >> 2)) & 3 : (w >> 2);
  return sj * SL + 4 * p4 + (w & 3);
}

// the projected re-rank for F <= 64, and for every F at histories of 65..128
// slots (din_rerank_lane.hip); a.sgn: 2 A bytes of workspace the launch fills
// with sgn(w2) per projection column
int launch_lane(int A, const RerankArgs& a, hipStream_t st);
// the longest history (L) launch_lane holds for (A, F): 128
int lane_max_l(int A, int F);

}  // namespace rr
}  // namespace nrk
