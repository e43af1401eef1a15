// nrk_common.h — shared device/host helpers for libnrk (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/nrk.h"

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;

namespace nrk {

// ---------------------------------------------------------------- errors --
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);

#define NRK_CHECK_ARG(cond, ...)                                  \
  do {                                                            \
    if (!(cond)) return ::nrk::fail(NRK_EINVAL, __VA_ARGS__);     \
  } while (0)

#define NRK_CHECK_LAUNCH(what)                                                          \
  do {                                                                                  \
    hipError_t e_ = hipGetLastError();                                                  \
    if (e_ != hipSuccess)                                                               \
      return ::nrk::fail(NRK_ELAUNCH, "%s: launch failed: %s", what, hipGetErrorString(e_)); \
  } while (0)

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ------------------------------------------------------------ bf16 bits --
// Round-to-nearest-even f32 -> bf16 bits.  Inputs of this library are finite
// embeddings; NaN handling is not needed (a NaN may come out as +-inf).
__host__ __device__ inline uint16_t f32_to_bf16_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__host__ __device__ inline float bf16_to_f32(uint16_t b) {
  uint32_t u = ((uint32_t)b) << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// Round a non-negative double UP to float (for rigorous error bounds).
__device__ inline float f64_to_f32_up(double x) {
  float f = (float)x;
  if ((double)f < x) f = __uint_as_float(__float_as_uint(f) + 1u);  // x >= 0, finite
  return f;
}

// Non-negative float atomic max via the integer order of IEEE bits.
__device__ inline void atomic_max_nonneg(float* p, float v) {
  atomicMax(reinterpret_cast<unsigned int*>(p), __float_as_uint(v));
}

// ----------------------------------------------------------- wave utils --
__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ inline float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Cross-lane sums on the VALU (DPP row ops and the CDNA4 half-row / half-wave
// swaps) instead of ds_bpermute (an LDS round trip, ~100 cycles, per step):
// every lane of the group receives the group's sum, in a fixed order.
// (bound_ctrl set: every pattern used below is a full permutation, so it changes
// nothing but lets the compiler fold the move into the consuming v_add / v_max)
#define NRK_DPP(v, ctrl) __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), (ctrl), 0xf, 0xf, true))
// sum over each quad (lanes 4k..4k+3)
__device__ __forceinline__ float quad_sum(float v) {
  v += NRK_DPP(v, 0xB1);  // quad_perm [1,0,3,2]
  v += NRK_DPP(v, 0x4E);  // quad_perm [2,3,0,1]
  return v;
}
// sum over each 8-lane group
__device__ __forceinline__ float oct_sum(float v) {
  v = quad_sum(v);
  return v + NRK_DPP(v, 0x141);  // row_half_mirror: quad 0 <-> quad 1 of each 8
}
// sum over each row of 16 lanes
__device__ __forceinline__ float row_sum16(float v) {
  v = oct_sum(v);
  return v + NRK_DPP(v, 0x140);  // row_mirror: the two 8-lane halves of the row
}
__device__ __forceinline__ float wave_sum_fast(float v);
// sum over each group of N consecutive lanes (N in {4, 8, 16, 64})
template <int N>
__device__ __forceinline__ float group_sum(float v) {
  static_assert(N == 4 || N == 8 || N == 16 || N == 64, "group_sum: N");
  if constexpr (N == 4) return quad_sum(v);
  else if constexpr (N == 8) return oct_sum(v);
  else if constexpr (N == 16) return row_sum16(v);
  else return wave_sum_fast(v);
}
// v[i] + v[i ^ 32]
__device__ __forceinline__ float half_swap_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// sum over the wave (every lane)
__device__ __forceinline__ float wave_sum_fast(float v) {
  v = row_sum16(v);
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);  // rows 2k <-> 2k+1
  return half_swap_sum(v);
}
__device__ __forceinline__ float wave_max_fast(float v) {
  v = fmaxf(v, NRK_DPP(v, 0xB1));
  v = fmaxf(v, NRK_DPP(v, 0x4E));
  v = fmaxf(v, NRK_DPP(v, 0x141));
  v = fmaxf(v, NRK_DPP(v, 0x140));
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// Position of the (j+1)-th set bit of m (j < popcount(m)): history slot of
// compacted row j (the DIN kernels score valid rows first, padding once).
__device__ __forceinline__ int nth_set_bit(uint64_t m, int j) {
  int pos = 0;
#pragma unroll
  for (int half = 32; half > 0; half >>= 1) {
    const int c = __popcll((m >> pos) & ((1ull << half) - 1));
    if (j >= c) {
      j -= c;
      pos += half;
    }
  }
  return pos;
}

// ------------------------------------------------------ index guards --
// Indices the IVF search reads back from its own workspace (list positions,
// query slots, probed lists) are range-checked where they address memory: a
// violation sets bit `code` of the search's guard word and the access is
// skipped, so a broken invariant surfaces as nrk_ivf_search_status() != 0
// (NrkError on the host) instead of an illegal-address fault.  One compare on
// paths that are rare or per candidate, not per screened item.
enum GuardCode : int {
  GUARD_SEED_POS = 1,       // ivf_seed_kernel: seed position outside [0, n)
  GUARD_CAND_POS = 2,       // collect_rescore: candidate position outside [0, n)
  GUARD_COLLECT_QUERY = 4,  // collect: a row's query outside [0, nq)
  GUARD_CAND_COUNT = 8,     // collect_rescore: negative candidate count
  GUARD_FB_QUERY = 16,      // fallback / exact scans: slot query outside [0, nq)
  GUARD_PROBE_LIST = 32,    // exact scans: probed list outside [-1, nlist)
  GUARD_GATHER_PAIR = 64,   // ivf_gather: (query, probe) pair outside [0, nq * nprobe)
  GUARD_COLLECT_POS = 128,  // collect: appended position outside [0, n)
};
__device__ __forceinline__ bool guard_ok(bool ok, int* err, int code) {
  if (!ok && err) atomicOr(err, code);
  return ok;
}

// --------------------------------------------------- ordering (k-NN) --
// "goodness" g: larger is better.  IP: g = score; L2: g = -distance.
// Ties on g break toward the lower id.
__device__ inline bool better(double ga, int64_t ia, double gb, int64_t ib) {
  return (ga > gb) | ((ga == gb) & (ia < ib));  // no short circuit: no exec-mask branches
}

// Bitonic sort of n (power of two) (g, id) pairs in LDS, best first.
// All threads of the block must call it.
__device__ inline void block_bitonic_sort(double* g, int64_t* id, int n) {
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        int j = i ^ stride;
        if (j > i) {
          bool desc = (i & size) == 0;  // best-first in this half
          bool ij = better(g[j], id[j], g[i], id[i]);  // j better than i
          if (desc ? ij : !ij) {
            double tg = g[i]; g[i] = g[j]; g[j] = tg;
            int64_t ti = id[i]; id[i] = id[j]; id[j] = ti;
          }
        }
      }
      __syncthreads();
    }
  }
}

}  // namespace nrk
