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

// --------------------------------------------------- ordering (k-NN) --
// "goodness" g: larger is better.  IP: g = score; L2: g = -distance.
// Ties on g break toward the lower id.
__device__ inline bool better(double ga, int64_t ia, double gb, int64_t ib) {
  return ga > gb || (ga == gb && ia < ib);
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
