// Microbenchmark (diagnostic, not product): cost of small dependent kernels as the
// DIN head runs them.  Each case is a chain: writer kernel (128 blocks write 4 MB
// of partials + 128 KB) -> reader kernel; timed with hipEvents over 200 replays.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
struct Big { const float* p[80]; int n[40]; };  // ~800 B of kernel arguments, like HeadArgs
__global__ void writer(float* pw, float* sgp, int n) {
  const int b = blockIdx.x, t = threadIdx.x;
  for (int i = t; i < 8192; i += 256) pw[(size_t)b * 8192 + i] = b + i;
  sgp[b * 256 + t] = b - t;
}
__global__ void empty_small(float* out) { if (threadIdx.x == 0) out[blockIdx.x] = 1.f; }
__global__ void empty_big(Big a) { if (threadIdx.x == 0) const_cast<float*>(a.p[blockIdx.x % 80])[blockIdx.x] = (float)a.n[3]; }
// 8 blocks: each sums 128 x 32 columns of sgp (like hf_bn0sum)
__global__ void small_red(const float* sgp, float* out) {
  const int cl = threadIdx.x & 31, ph = threadIdx.x >> 5, c = 32 * blockIdx.x + cl;
  float v[16]; double s = 0;
#pragma unroll
  for (int u = 0; u < 16; ++u) v[u] = sgp[(ph + 8 * u) * 256 + c];
#pragma unroll
  for (int u = 0; u < 16; ++u) s += v[u];
  __shared__ double r[8][32];
  r[ph][cl] = s; __syncthreads();
  if (ph == 0) { double t = 0; for (int q = 0; q < 8; ++q) t += r[q][cl]; out[c] = (float)t; }
}
// 256 WGs x 512 threads each summing 128 x 128 columns of sgp (like the prologue)
__global__ void wide_red(const float* sgp, float* out) {
  const int c = threadIdx.x & 127, p = threadIdx.x >> 7;
  float v[32]; double s = 0;
#pragma unroll
  for (int u = 0; u < 32; ++u) v[u] = sgp[(p + 4 * u) * 256 + 128 + c];
#pragma unroll
  for (int u = 0; u < 32; ++u) s += v[u];
  if (s == -1.0) out[blockIdx.x] = 0;
}
// 128 blocks x 512 threads: G reduction of 2 columns each (like hf_grads_block)
__global__ void g_red(const float* pw, float* out) {
  const int j = threadIdx.x & 31, cl = (threadIdx.x >> 5) & 1, ph = threadIdx.x >> 6, c = 2 * blockIdx.x + cl;
  float v[16]; double s = 0;
#pragma unroll
  for (int u = 0; u < 16; ++u) v[u] = pw[(size_t)(ph + 8 * u) * 8192 + c * 32 + j];
#pragma unroll
  for (int u = 0; u < 16; ++u) s += v[u];
  __shared__ double r[8][64];
  r[ph][threadIdx.x & 63] = s; __syncthreads();
  if (ph == 0) { double t = 0; for (int q = 0; q < 8; ++q) t += r[q][threadIdx.x & 63]; out[c * 32 + j] = (float)t; }
}
int main() {
  float *pw, *sgp, *out;
  hipMalloc(&pw, 128 * 8192 * 4); hipMalloc(&sgp, 128 * 256 * 4); hipMalloc(&out, 1 << 20);
  Big big{}; for (int i = 0; i < 80; ++i) big.p[i] = out; big.n[3] = 7;
  hipStream_t s; hipStreamCreate(&s);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 20; ++i) launch();
    hipStreamSynchronize(s);
    hipGraph_t g; hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < 50; ++i) launch();
    hipStreamEndCapture(s, &g); hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s); hipStreamSynchronize(s);
    hipEventRecord(e0, s);
    for (int i = 0; i < 20; ++i) hipGraphLaunch(ge, s);
    hipEventRecord(e1, s); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-40s %7.2f us per chain\n", name, ms * 1000 / 1000);
  };
  run("writer", [&] { writer<<<128, 256, 0, s>>>(pw, sgp, 0); });
  run("writer + empty_small(128)", [&] { writer<<<128, 256, 0, s>>>(pw, sgp, 0); empty_small<<<128, 256, 0, s>>>(out); });
  run("writer + empty_big(128)", [&] { writer<<<128, 256, 0, s>>>(pw, sgp, 0); empty_big<<<128, 256, 0, s>>>(big); });
  run("writer + small_red(8)", [&] { writer<<<128, 256, 0, s>>>(pw, sgp, 0); small_red<<<8, 256, 0, s>>>(sgp, out); });
  run("writer + wide_red(256x512)", [&] { writer<<<128, 256, 0, s>>>(pw, sgp, 0); wide_red<<<256, 512, 0, s>>>(sgp, out); });
  run("writer + g_red(128x512)", [&] { writer<<<128, 256, 0, s>>>(pw, sgp, 0); g_red<<<128, 512, 0, s>>>(pw, out); });
  run("empty_small x2", [&] { empty_small<<<128, 256, 0, s>>>(out); empty_small<<<128, 256, 0, s>>>(out); });
  run("empty_big x2", [&] { empty_big<<<128, 256, 0, s>>>(big); empty_big<<<128, 256, 0, s>>>(big); });
  return 0;
}
