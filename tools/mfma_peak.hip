// tools/mfma_peak.hip — the bf16 MFMA rate this MI355X sustains on random
// operands (the DVFS-limited ceiling the screen kernels are measured against):
// bare v_mfma_f32_32x32x16_bf16 and v_mfma_f32_16x16x32_bf16 loops, 8 waves
// per SIMD, operands in registers, the same FLOP per launch for both shapes.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_peak.hip -o /tmp/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
#include <cstring>
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k32(const bf16x8* a, const bf16x8* b, float* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  bf16x8 av[4], bv[4];
  for (int i = 0; i < 4; ++i) { av[i] = a[(t * 4 + i) & 65535]; bv[i] = b[(t * 4 + i) & 65535]; }
  f32x16 acc0 = {}, acc1 = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[i], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bv[i], av[i], acc1, 0, 0, 0);
    }
  }
  float s = 0; for (int g = 0; g < 16; ++g) s += acc0[g] + acc1[g];
  out[t] = s;
}
__global__ __launch_bounds__(256) void k16(const bf16x8* a, const bf16x8* b, float* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  bf16x8 av[4], bv[4];
  for (int i = 0; i < 4; ++i) { av[i] = a[(t * 4 + i) & 65535]; bv[i] = b[(t * 4 + i) & 65535]; }
  f32x4 acc[8] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        acc[2 * i + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[(i + j) & 3], acc[2 * i + j], 0, 0, 0);
        acc[(2 * i + j + 4) & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv[i], av[(i + j) & 3], acc[(2 * i + j + 4) & 7], 0, 0, 0);
      }
    }
  }
  float s = 0; for (int g = 0; g < 8; ++g) for (int i = 0; i < 4; ++i) s += acc[g][i];
  out[t] = s;
}
int main() {
  const int n = 65536 * 8;
  std::vector<short> h(n);
  std::mt19937 rng(1);
  for (auto& x : h) { float f = std::normal_distribution<float>(0, 1)(rng); unsigned u; std::memcpy(&u, &f, 4); x = (short)(u >> 16); }
  short *a, *b; float* o;
  hipMalloc(&a, n * 2); hipMalloc(&b, n * 2); hipMalloc(&o, 256 * 2048 * 4);
  hipMemcpy(a, h.data(), n * 2, hipMemcpyHostToDevice);
  hipMemcpy(b, h.data(), n * 2, hipMemcpyHostToDevice);
  const int blocks = 2048, iters = 4000;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    for (int which = 0; which < 2; ++which) {
      for (int w = 0; w < 3; ++w) {  // warm / DVFS settle
        if (which == 0) hipLaunchKernelGGL(k32, dim3(blocks), dim3(256), 0, 0, (bf16x8*)a, (bf16x8*)b, o, iters);
        else hipLaunchKernelGGL(k16, dim3(blocks), dim3(256), 0, 0, (bf16x8*)a, (bf16x8*)b, o, iters);
      }
      hipEventRecord(e0);
      for (int w = 0; w < 5; ++w) {
        if (which == 0) hipLaunchKernelGGL(k32, dim3(blocks), dim3(256), 0, 0, (bf16x8*)a, (bf16x8*)b, o, iters);
        else hipLaunchKernelGGL(k16, dim3(blocks), dim3(256), 0, 0, (bf16x8*)a, (bf16x8*)b, o, iters);
      }
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      // FLOP per 5 launches: per wave and iteration 8 x 32x32x16 (32768 each) or
      // 16 x 16x16x32 (16384 each): the same
      const double fl = 5.0 * blocks * 4.0 * iters * 8 * 32768.0;
      printf("%s: %.3f ms per launch, %.1f TFLOP/s\n", which ? "16x16x32" : "32x32x16", ms / 5, fl / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
