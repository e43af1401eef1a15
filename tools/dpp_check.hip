// Checks the cross-lane sum / max helpers of nrk_common.h against a host
// reference (exact: the inputs are small integers, so every order sums exactly).
// build: hipcc -O3 --offload-arch=gfx950 tools/dpp_check.hip -o tools/dpp_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include "../newsrecommend_amd/csrc/nrk_common.h"
using namespace nrk;

__global__ void k(const float* in, float* out) {
  const float v = in[threadIdx.x];
  out[threadIdx.x] = wave_sum_fast(v);
  out[64 + threadIdx.x] = oct_sum(v);
  out[128 + threadIdx.x] = half_swap_sum(v);
  out[192 + threadIdx.x] = wave_max_fast(v);
  out[256 + threadIdx.x] = quad_sum(v);
}

int main() {
  float h[64], o[320];
  for (int i = 0; i < 64; ++i) h[i] = (float)((i * 37 + 11) % 97) - 40.f;
  float *din, *dout;
  if (hipMalloc(&din, 64 * 4) != hipSuccess || hipMalloc(&dout, 320 * 4) != hipSuccess) return 2;
  if (hipMemcpy(din, h, 64 * 4, hipMemcpyHostToDevice) != hipSuccess) return 2;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout);
  if (hipMemcpy(o, dout, 320 * 4, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  int bad = 0;
  float tot = 0.f, mx = -INFINITY;
  for (int i = 0; i < 64; ++i) { tot += h[i]; mx = fmaxf(mx, h[i]); }
  for (int i = 0; i < 64; ++i) {
    float s8 = 0.f, s4 = 0.f;
    for (int j = 0; j < 8; ++j) s8 += h[(i & ~7) + j];
    for (int j = 0; j < 4; ++j) s4 += h[(i & ~3) + j];
    const float s32 = h[i] + h[i ^ 32];
    if (o[i] != tot) { ++bad; printf("wave_sum lane %d %g vs %g\n", i, o[i], tot); }
    if (o[64 + i] != s8) { ++bad; printf("oct_sum lane %d %g vs %g\n", i, o[64 + i], s8); }
    if (o[128 + i] != s32) { ++bad; printf("half_swap lane %d %g vs %g\n", i, o[128 + i], s32); }
    if (o[192 + i] != mx) { ++bad; printf("wave_max lane %d %g vs %g\n", i, o[192 + i], mx); }
    if (o[256 + i] != s4) { ++bad; printf("quad_sum lane %d %g vs %g\n", i, o[256 + i], s4); }
  }
  printf(bad ? "dpp_check FAIL (%d)\n" : "dpp_check PASS\n", bad);
  return bad ? 1 : 0;
}
