// din_head.hip — DIN's MLP head in train mode, forward + backward, and the
// fused clip_grad_norm_ + Adam step (DIN.py:117-123,130-133,143-151).
//
// The head is tiny (2d -> F -> F/2 -> 1 per sample) but in torch it is ~150
// latency-bound launches per step (three train-mode BatchNorms, Linear,
// ReLU, Dropout, BCE and their backward).  Here it is 8 kernels over blocks
// of 32 rows:
//   stats0   per-block sums of x = [q | pooled] for BN0
//   fwd1     BN0 -> Linear(2d,F) -> ReLU -> Dropout, BN1 sums
//   fwd2     BN1 -> Linear(F,F/2) -> ReLU -> Dropout, BN2 sums
//   fwd3     BN2 -> Linear(F/2,1) -> BCEWithLogits (mean); dlogit; BN2-bwd sums
//   bwd2     BN2 bwd -> Dropout/ReLU bwd -> Linear(F,F/2) bwd; BN1-bwd sums
//   bwd1     BN1 bwd -> Dropout/ReLU bwd -> Linear(2d,F) bwd; BN0-bwd sums
//   bwd0     BN0 bwd -> dpooled (the attention backward's input)
//   grads    parameter gradients = fixed-order sums of the block partials
// Batch statistics are summed in fp64 per block and over blocks in a fixed
// order (deterministic); every block recomputes the finalised statistics it
// needs, and the first kernel that finalises a BatchNorm updates its running
// statistics (momentum, unbiased variance) and num_batches_tracked.
// Activations are recomputed in the backward kernels from the stored
// pre-activations a1/a2 and the counter-based dropout masks.
#include <math.h>
#include <stdlib.h>

#include <algorithm>

#include "nrk_common.h"

namespace nrk {

constexpr int HR = 32;  // rows per block

struct HeadArgs {
  nrk_din_head_params p;
  const float* q;
  const float* pooled;
  int64_t ld;  // row stride of pooled / dpooled
  const float* y;
  int B, d, D2, F, F2, nblk;
  float momentum, eps, p_drop;
  uint64_t seed;
  const float* step;  // device step counter (dropout stream per step)
  // workspace
  double *part0, *part1, *part2, *part3, *part4, *part5;
  double *sum0, *sum1, *sum2, *sum3, *sum4, *sum5, *sumw1;  // the partials summed over blocks
  float *stat0, *stat1, *stat2;  // finalised {mean, invstd} per feature
  float *a1, *a2, *dh2, *dh1, *dh0, *pw1;
  float* da1;       // fast head: the gradient at fc.1's output [B][32] (hf_bwd1; the dh0 region)
  uint32_t* mask1;  // fast head, dropout > 0: fc.2 dropout keep bits, one word per row (hf_fwd1)
  uint16_t* mask2;  // fc.6 dropout keep bits, 16 per row (hf_fwd2)
  float* logits;
  float* loss;
  float* dpooled;
  int fast;  // F == 32 fast path: statistics reduced in each consumer's prologue
  int nrg0;  // row groups of hf_stats0
};

__device__ __forceinline__ float hx(const HeadArgs& a, int64_t r, int c) {
  return c < a.d ? a.q[r * a.d + c] : a.pooled[r * a.ld + (c - a.d)];
}

// counter-based dropout mask (splitmix64 of (seed, step, layer, row, col));
// keep_scale_s takes the step value read once per thread
__device__ __forceinline__ float keep_scale_s(const HeadArgs& a, float stepv, int layer, int64_t r, int c) {
  if (a.p_drop <= 0.f) return 1.f;
  uint64_t z = a.seed ^ ((uint64_t)(int64_t)stepv * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)layer << 58) ^
               ((uint64_t)r << 20) ^ (uint64_t)c;
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const float u = (float)(z >> 40) * (1.0f / 16777216.0f);
  return u >= a.p_drop ? 1.f / (1.f - a.p_drop) : 0.f;
}
// the keep scale of bit `bit` of a stored mask word (the same value keep_scale_s
// gave when the word was formed)
__device__ __forceinline__ float keep_bit(const HeadArgs& a, uint32_t word, int bit) {
  if (a.p_drop <= 0.f) return 1.f;
  return (word >> bit) & 1u ? 1.f / (1.f - a.p_drop) : 0.f;
}
__device__ __forceinline__ float keep_scale(const HeadArgs& a, int layer, int64_t r, int c) {
  return keep_scale_s(a, *a.step, layer, r, c);
}

// Column sums over the blocks' partials, fixed order (deterministic): a
// block covers 32 columns with 8 row groups; groups combined in LDS.
template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* __restrict__ part, int nblk, int stride, int ncols,
                                                     double* __restrict__ out) {
  __shared__ double red[8][33];
  const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  double s = 0.0;
  if (c < ncols) {
#pragma unroll 4
    for (int b = g; b < nblk; b += 8) s += (double)part[(int64_t)b * stride + c];
  }
  red[g][cl] = s;
  __syncthreads();
  if (g == 0 && c < ncols) {
    double t = 0.0;
    for (int i = 0; i < 8; ++i) t += red[i][cl];
    out[c] = t;
  }
}

// finalise BN batch statistics of C features (sums S[c], S[C + c]) into LDS;
// the designated block also publishes them and updates the running statistics
__device__ void bn_finalize(const HeadArgs& a, const double* sum, int C, float* s_mean, float* s_inv, float* stat,
                            float* rm, float* rv, int64_t* nb, bool publish) {
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const double mean = sum[c] / a.B;
    double var = sum[C + c] / a.B - mean * mean;
    if (var < 0) var = 0;
    const float inv = (float)(1.0 / sqrt(var + (double)a.eps));
    s_mean[c] = (float)mean;
    s_inv[c] = inv;
    if (publish) {
      stat[c] = (float)mean;
      stat[C + c] = inv;
      rm[c] = (1.f - a.momentum) * rm[c] + a.momentum * (float)mean;
      rv[c] = (1.f - a.momentum) * rv[c] + a.momentum * (float)(var * a.B / (a.B - 1));
    }
  }
  if (publish && threadIdx.x == 0 && nb) *nb += 1;
}

// bn_finalize with the designated block's running statistics loaded at kernel
// entry (pre_rm / pre_rv: columns t and t + blockDim.x of thread t, C <= 2 x
// blockDim.x), so the publish adds no memory round trip at the kernel's tail
struct RunStatPre {
  float rm[2], rv[2];
  int64_t nb;
};
__device__ __forceinline__ RunStatPre run_stat_pre(const float* rm, const float* rv, const int64_t* nb, int C,
                                                   bool publish) {
  RunStatPre r{};
  r.nb = publish && threadIdx.x == 0 && nb ? *nb : 0;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = threadIdx.x + u * blockDim.x;
    r.rm[u] = publish && c < C ? rm[c] : 0.f;
    r.rv[u] = publish && c < C ? rv[c] : 0.f;
  }
  return r;
}
__device__ void bn_finalize_pre(const HeadArgs& a, const double* sum, int C, float* s_mean, float* s_inv, float* stat,
                                float* rm, float* rv, int64_t* nb, bool publish, const RunStatPre& pre) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = threadIdx.x + u * blockDim.x;
    if (c >= C) break;
    const double mean = sum[c] / a.B;
    double var = sum[C + c] / a.B - mean * mean;
    if (var < 0) var = 0;
    const float inv = (float)(1.0 / sqrt(var + (double)a.eps));
    s_mean[c] = (float)mean;
    s_inv[c] = inv;
    if (publish) {
      stat[c] = (float)mean;
      stat[C + c] = inv;
      rm[c] = (1.f - a.momentum) * pre.rm[u] + a.momentum * (float)mean;
      rv[c] = (1.f - a.momentum) * pre.rv[u] + a.momentum * (float)(var * a.B / (a.B - 1));
    }
  }
  if (publish && threadIdx.x == 0 && nb) *nb = pre.nb + 1;
}

__device__ __forceinline__ void load_stat(const float* stat, int C, float* s_mean, float* s_inv) {
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    s_mean[c] = stat[c];
    s_inv[c] = stat[C + c];
  }
}

// Fixed-order column sums of nblk partial rows (stride doubles apart) for
// columns [0, ncol) into s_out (LDS), by every block of a consumer kernel
// (the launch-boundary reduce: no separate colsum launch).  256 threads.
__device__ void colsum_prologue(const double* __restrict__ part, int nblk, int stride, int ncol,
                                double* s_tmp /*[256]*/, double* s_out) {
  const int t = threadIdx.x;
  if (ncol > 256 && ncol <= 512 && nblk <= 16) {  // hf_fwd1's BN0 sums: both columns' loads in one round
    double v[2][16];
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int c = t + 256 * k;
        v[k][u] = c < ncol && u < nblk ? part[(int64_t)u * stride + c] : 0.0;
      }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      double acc = 0.0;
#pragma unroll
      for (int u = 0; u < 16; ++u) acc += v[k][u];
      if (t + 256 * k < ncol) s_out[t + 256 * k] = acc;
    }
    __syncthreads();
    return;
  }
  if (ncol > 128) {
    for (int c = t; c < ncol; c += 256) {
      double acc = 0.0;
      for (int b0 = 0; b0 < nblk; b0 += 16) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = b0 + u < nblk ? part[(int64_t)(b0 + u) * stride + c] : 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += v[u];
      }
      s_out[c] = acc;
    }
    __syncthreads();
    return;
  }
  const int nph = 256 / ncol;
  const int c = t % ncol, ph = t / ncol;
  if (ph < nph) {
    double acc = 0.0;
    for (int b0 = ph; b0 < nblk; b0 += 32 * nph) {  // 32 loads in flight, summed in block order
      double v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        const int b = b0 + u * nph;
        v[u] = b < nblk ? part[(int64_t)b * stride + c] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 32; ++u) acc += v[u];
    }
    s_tmp[ph * ncol + c] = acc;
  }
  __syncthreads();
  if (t < ncol) {
    double acc = 0.0;
    for (int q = 0; q < nph; ++q) acc += s_tmp[q * ncol + t];
    s_out[t] = acc;
  }
  __syncthreads();
}

// x = [q | pooled] as float4 (d % 4 == 0): element 4*c4 .. of row r
__device__ __forceinline__ float4 hx4(const HeadArgs& a, int64_t r, int c) {
  return c < a.d ? *reinterpret_cast<const float4*>(a.q + r * a.d + c)
                 : *reinterpret_cast<const float4*>(a.pooled + r * a.ld + (c - a.d));
}

// dot product of n terms x[i*sx] * y[i*sy] with 4 independent chains (the
// LDS loads of 4 terms are in flight together: these kernels run one wave
// per SIMD, so a rolled loop waits out every ds_read latency)
__device__ __forceinline__ float dot4(const float* x, int sx, const float* y, int sy, int n, float init) {
  float c0 = init, c1 = 0.f, c2 = 0.f, c3 = 0.f;
  int i = 0;
  for (; i + 4 <= n; i += 4) {
    c0 = fmaf(x[i * sx], y[i * sy], c0);
    c1 = fmaf(x[(i + 1) * sx], y[(i + 1) * sy], c1);
    c2 = fmaf(x[(i + 2) * sx], y[(i + 2) * sy], c2);
    c3 = fmaf(x[(i + 3) * sx], y[(i + 3) * sy], c3);
  }
  for (; i < n; ++i) c0 = fmaf(x[i * sx], y[i * sy], c0);
  return (c0 + c1) + (c2 + c3);
}

__global__ __launch_bounds__(256) void head_stats0(HeadArgs a) {
  const int64_t r0 = (int64_t)blockIdx.x * HR;
  for (int c = threadIdx.x; c < a.D2; c += 256) {
    double s = 0.0, ss = 0.0;
    for (int r = 0; r < HR; ++r) {
      const double v = hx(a, r0 + r, c);
      s += v;
      ss += v * v;
    }
    a.part0[(int64_t)blockIdx.x * 2 * a.D2 + c] = s;
    a.part0[(int64_t)blockIdx.x * 2 * a.D2 + a.D2 + c] = ss;
  }
}

// LDS: h0 [HR][D2+1], W1 chunk [FC][D2+1], mean/inv [D2] x 2, d1 [HR][F].
// W1 passes through LDS FC = 32 output units at a time (2d = 512 and F = 128
// would need 328 KB at once).
constexpr int FC = 32;
__global__ __launch_bounds__(256) void head_fwd1(HeadArgs a) {
  extern __shared__ float sm[];
  const int D2 = a.D2, F = a.F, ds = D2 + 1;
  const int fc = F < FC ? F : FC;
  float* h0 = sm;
  float* w1 = h0 + HR * ds;
  float* mean = w1 + fc * ds;
  float* inv = mean + D2;
  float* d1 = inv + D2;
  const int64_t r0 = (int64_t)blockIdx.x * HR;
  bn_finalize(a, a.sum0, D2, mean, inv, a.stat0, a.p.bn0_rm, a.p.bn0_rv, a.p.bn0_nb, blockIdx.x == 0);
  __syncthreads();
  for (int e = threadIdx.x; e < HR * D2; e += 256) {
    const int r = e / D2, c = e % D2;
    h0[r * ds + c] = (hx(a, r0 + r, c) - mean[c]) * inv[c] * a.p.bn0_w[c] + a.p.bn0_b[c];
  }
  for (int j0 = 0; j0 < F; j0 += fc) {
    const int nj = F - j0 < fc ? F - j0 : fc;
    __syncthreads();  // (the previous chunk's dot products are done with w1)
    for (int e = threadIdx.x; e < nj * D2; e += 256) w1[(e / D2) * ds + e % D2] = a.p.fc1_w[(int64_t)j0 * D2 + e];
    __syncthreads();
    for (int o = threadIdx.x; o < HR * nj; o += 256) {
      const int r = o / nj, jj = o % nj, j = j0 + jj;
      float acc = a.p.fc1_b[j];
      acc = dot4(h0 + r * ds, 1, w1 + jj * ds, 1, D2, acc);
      a.a1[(r0 + r) * F + j] = acc;
      d1[r * F + j] = fmaxf(acc, 0.f) * keep_scale(a, 1, r0 + r, j);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < F; j += 256) {
    double s = 0.0, ss = 0.0;
    for (int r = 0; r < HR; ++r) {
      const double v = d1[r * F + j];
      s += v;
      ss += v * v;
    }
    a.part1[(int64_t)blockIdx.x * 2 * F + j] = s;
    a.part1[(int64_t)blockIdx.x * 2 * F + F + j] = ss;
  }
}

// LDS: h1 [HR][F], W2 [F2][F], mean1/inv1 [F], d2 [HR][F2]
__global__ __launch_bounds__(256) void head_fwd2(HeadArgs a) {
  extern __shared__ float sm[];
  const int F = a.F, F2 = a.F2;
  float* h1 = sm;
  float* w2 = h1 + HR * F;
  float* mean = w2 + F2 * F;
  float* inv = mean + F;
  float* d2 = inv + F;
  const int64_t r0 = (int64_t)blockIdx.x * HR;
  __shared__ double pro_tmp[256], pro_sum[128];
  const double* S1 = a.sum1;
  if (a.fast) {
    colsum_prologue(a.part1, a.nblk, 2 * F, 2 * F, pro_tmp, pro_sum);
    S1 = pro_sum;
  }
  bn_finalize(a, S1, F, mean, inv, a.stat1, a.p.bn1_rm, a.p.bn1_rv, a.p.bn1_nb, blockIdx.x == 0);
  for (int e = threadIdx.x; e < F2 * F; e += 256) w2[e] = a.p.fc2_w[e];
  __syncthreads();
  for (int e = threadIdx.x; e < HR * F; e += 256) {
    const int r = e / F, j = e % F;
    const float d1 = fmaxf(a.a1[(r0 + r) * F + j], 0.f) * keep_scale(a, 1, r0 + r, j);
    h1[e] = (d1 - mean[j]) * inv[j] * a.p.bn1_w[j] + a.p.bn1_b[j];
  }
  __syncthreads();
  for (int o = threadIdx.x; o < HR * F2; o += 256) {
    const int r = o / F2, k = o % F2;
    float acc = a.p.fc2_b[k];
    acc = dot4(h1 + r * F, 1, w2 + k * F, 1, F, acc);
    a.a2[(r0 + r) * F2 + k] = acc;
    d2[o] = fmaxf(acc, 0.f) * keep_scale(a, 2, r0 + r, k);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < F2; k += 256) {
    double s = 0.0, ss = 0.0;
    for (int r = 0; r < HR; ++r) {
      const double v = d2[r * F2 + k];
      s += v;
      ss += v * v;
    }
    a.part2[(int64_t)blockIdx.x * 2 * F2 + k] = s;
    a.part2[(int64_t)blockIdx.x * 2 * F2 + F2 + k] = ss;
  }
}

// part3 per block: [F2] sum dh2, [F2] sum dh2*xhat2, [F2] dW3, [1] db3, [1] loss
__global__ __launch_bounds__(256) void head_fwd3(HeadArgs a) {
  extern __shared__ float sm[];
  const int F2 = a.F2;
  float* h2 = sm;            // [HR][F2]
  float* xh = h2 + HR * F2;  // [HR][F2] xhat2
  float* mean = xh + HR * F2;
  float* inv = mean + F2;
  float* dl = inv + F2;  // [HR]
  float* lo = dl + HR;   // [HR]
  const int64_t r0 = (int64_t)blockIdx.x * HR;
  __shared__ double pro_tmp[256], pro_sum[64];
  const double* S2 = a.sum2;
  if (a.fast) {
    colsum_prologue(a.part2, a.nblk, 2 * F2, 2 * F2, pro_tmp, pro_sum);
    S2 = pro_sum;
  }
  bn_finalize(a, S2, F2, mean, inv, a.stat2, a.p.bn2_rm, a.p.bn2_rv, a.p.bn2_nb, blockIdx.x == 0);
  __syncthreads();
  for (int e = threadIdx.x; e < HR * F2; e += 256) {
    const int r = e / F2, k = e % F2;
    const float d2 = fmaxf(a.a2[(r0 + r) * F2 + k], 0.f) * keep_scale(a, 2, r0 + r, k);
    const float x = (d2 - mean[k]) * inv[k];
    xh[e] = x;
    h2[e] = x * a.p.bn2_w[k] + a.p.bn2_b[k];
  }
  __syncthreads();
  for (int r = threadIdx.x; r < HR; r += 256) {
    float z = a.p.fc3_b[0];
    for (int k = 0; k < F2; ++k) z = fmaf(h2[r * F2 + k], a.p.fc3_w[k], z);
    const float y = a.y[r0 + r];
    a.logits[r0 + r] = z;
    lo[r] = fmaxf(z, 0.f) - z * y + log1pf(expf(-fabsf(z)));
    dl[r] = (1.f / (1.f + expf(-z)) - y) / (float)a.B;
  }
  __syncthreads();
  double* pp = a.part3 + (int64_t)blockIdx.x * (3 * F2 + 2);
  for (int e = threadIdx.x; e < HR * F2; e += 256) {
    const int r = e / F2, k = e % F2;
    a.dh2[(r0 + r) * F2 + k] = dl[r] * a.p.fc3_w[k];
  }
  for (int k = threadIdx.x; k < F2; k += 256) {
    double sb = 0.0, sg = 0.0, sw = 0.0;
    for (int r = 0; r < HR; ++r) {
      const double g = (double)dl[r] * a.p.fc3_w[k];
      sb += g;
      sg += g * xh[r * F2 + k];
      sw += (double)dl[r] * h2[r * F2 + k];
    }
    pp[k] = sb;
    pp[F2 + k] = sg;
    pp[2 * F2 + k] = sw;
  }
  if (threadIdx.x == 0) {
    double s = 0.0, l = 0.0;
    for (int r = 0; r < HR; ++r) {
      s += dl[r];
      l += lo[r];
    }
    pp[3 * F2] = s;
    pp[3 * F2 + 1] = l;
  }
}

// part4 per block: [F] sum dh1, [F] sum dh1*xhat1, [F2*F] dW2, [F2] db2
__global__ __launch_bounds__(256) void head_bwd2(HeadArgs a) {
  extern __shared__ float sm[];
  const int F = a.F, F2 = a.F2;
  float* h1 = sm;             // [HR][F]
  float* xh1 = h1 + HR * F;   // [HR][F]
  float* da2 = xh1 + HR * F;  // [HR][F2]
  float* dh1 = da2 + HR * F2; // [HR][F]
  float* m1 = dh1 + HR * F;
  float* i1 = m1 + F;
  float* m2 = i1 + F;
  float* i2 = m2 + F2;
  float* sb2 = i2 + F2;  // sum dh2 over the batch
  float* sg2 = sb2 + F2; // sum dh2*xhat2
  float* w2s = sg2 + F2; // fc2 weight [F2][F]
  for (int e = threadIdx.x; e < F2 * F; e += 256) w2s[e] = a.p.fc2_w[e];
  const int64_t r0 = (int64_t)blockIdx.x * HR;
  load_stat(a.stat1, F, m1, i1);
  load_stat(a.stat2, F2, m2, i2);
  __shared__ double pro_tmp[256], pro_sum[64];
  const double* S3 = a.sum3;
  if (a.fast) {
    colsum_prologue(a.part3, a.nblk, 3 * F2 + 2, 2 * F2, pro_tmp, pro_sum);
    S3 = pro_sum;
  }
  for (int k = threadIdx.x; k < F2; k += 256) {
    sb2[k] = (float)S3[k];
    sg2[k] = (float)S3[F2 + k];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < HR * F; e += 256) {
    const int r = e / F, j = e % F;
    const float d1 = fmaxf(a.a1[(r0 + r) * F + j], 0.f) * keep_scale(a, 1, r0 + r, j);
    const float x = (d1 - m1[j]) * i1[j];
    xh1[e] = x;
    h1[e] = x * a.p.bn1_w[j] + a.p.bn1_b[j];
  }
  const float invB = 1.f / (float)a.B;
  for (int e = threadIdx.x; e < HR * F2; e += 256) {
    const int r = e / F2, k = e % F2;
    const float a2 = a.a2[(r0 + r) * F2 + k];
    const float ks = keep_scale(a, 2, r0 + r, k);
    const float xhat = (fmaxf(a2, 0.f) * ks - m2[k]) * i2[k];
    const float g = a.p.bn2_w[k];
    const float dd2 = i2[k] * g * (a.dh2[(r0 + r) * F2 + k] - sb2[k] * invB - xhat * sg2[k] * invB);
    da2[e] = a2 > 0.f ? dd2 * ks : 0.f;
  }
  __syncthreads();
  double* pp = a.part4 + (int64_t)blockIdx.x * (2 * F + F2 * F + F2);
  for (int o = threadIdx.x; o < F2 * F; o += 256) {
    const int k = o / F, j = o % F;
    double s = 0.0;
    for (int r = 0; r < HR; ++r) s += (double)da2[r * F2 + k] * h1[r * F + j];
    pp[2 * F + o] = s;
  }
  for (int k = threadIdx.x; k < F2; k += 256) {
    double s = 0.0;
    for (int r = 0; r < HR; ++r) s += da2[r * F2 + k];
    pp[2 * F + F2 * F + k] = s;
  }
  for (int e = threadIdx.x; e < HR * F; e += 256) {
    const int r = e / F, j = e % F;
    float s = 0.f;
    s = dot4(da2 + r * F2, 1, w2s + j, F, F2, s);
    dh1[e] = s;
    a.dh1[(r0 + r) * F + j] = s;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < F; j += 256) {
    double sb = 0.0, sg = 0.0;
    for (int r = 0; r < HR; ++r) {
      sb += dh1[r * F + j];
      sg += (double)dh1[r * F + j] * xh1[r * F + j];
    }
    pp[j] = sb;
    pp[F + j] = sg;
  }
}

// part5 per block: [D2] sum dh0, [D2] sum dh0*xhat0, [F] db1; pw1 per block [F*D2] (f32).
// W1 passes through LDS FC units at a time (as head_fwd1); dh0 = da1 W1 is
// accumulated over the chunks in registers (2d <= 512: two columns of the
// block's 32 rows per thread).
__global__ __launch_bounds__(256) void head_bwd1(HeadArgs a) {
  extern __shared__ float sm[];
  const int D2 = a.D2, F = a.F, ds = D2 + 1;
  const int fc = F < FC ? F : FC;
  float* h0 = sm;             // [HR][D2+1]
  float* w1 = h0 + HR * ds;   // [FC][D2+1]
  float* da1 = w1 + fc * ds;  // [HR][F]
  float* m0 = da1 + HR * F;
  float* i0 = m0 + D2;
  float* m1 = i0 + D2;
  float* i1 = m1 + F;
  float* sb1 = i1 + F;
  float* sg1 = sb1 + F;
  const int64_t r0 = (int64_t)blockIdx.x * HR;
  load_stat(a.stat0, D2, m0, i0);
  load_stat(a.stat1, F, m1, i1);
  for (int j = threadIdx.x; j < F; j += 256) {
    sb1[j] = (float)a.sum4[j];
    sg1[j] = (float)a.sum4[F + j];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < HR * D2; e += 256) {  // h0 holds xhat0 here (h0 = xhat0 * w + b)
    const int r = e / D2, c = e % D2;
    h0[r * ds + c] = (hx(a, r0 + r, c) - m0[c]) * i0[c];
  }
  const float invB = 1.f / (float)a.B;
  for (int e = threadIdx.x; e < HR * F; e += 256) {
    const int r = e / F, j = e % F;
    const float a1 = a.a1[(r0 + r) * F + j];
    const float ks = keep_scale(a, 1, r0 + r, j);
    const float xhat = (fmaxf(a1, 0.f) * ks - m1[j]) * i1[j];
    const float dd1 = i1[j] * a.p.bn1_w[j] * (a.dh1[(r0 + r) * F + j] - sb1[j] * invB - xhat * sg1[j] * invB);
    da1[e] = a1 > 0.f ? dd1 * ks : 0.f;
  }
  __syncthreads();
  float* pw = a.pw1 + (int64_t)blockIdx.x * F * D2;
  for (int o = threadIdx.x; o < F * D2; o += 256) {
    const int j = o / D2, c = o % D2;
    const float gw = a.p.bn0_w[c], gb = a.p.bn0_b[c];
    float s = 0.f;
    float s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
    for (int r = 0; r < HR; r += 4) {
      s = fmaf(da1[r * F + j], fmaf(h0[r * ds + c], gw, gb), s);
      s1 = fmaf(da1[(r + 1) * F + j], fmaf(h0[(r + 1) * ds + c], gw, gb), s1);
      s2 = fmaf(da1[(r + 2) * F + j], fmaf(h0[(r + 2) * ds + c], gw, gb), s2);
      s3 = fmaf(da1[(r + 3) * F + j], fmaf(h0[(r + 3) * ds + c], gw, gb), s3);
    }
    s = (s + s1) + (s2 + s3);
    pw[o] = s;
  }
  double* pp = a.part5 + (int64_t)blockIdx.x * (2 * D2 + F);
  for (int j = threadIdx.x; j < F; j += 256) {
    double s = 0.0;
    for (int r = 0; r < HR; ++r) s += da1[r * F + j];
    pp[2 * D2 + j] = s;
  }
  // dh0 = da1 W1 (summed over the W1 chunks) and the BN0-backward sums over
  // this block's rows; thread t owns columns t and t + 256
  float dh[2][HR];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int r = 0; r < HR; ++r) dh[u][r] = 0.f;
  for (int j0 = 0; j0 < F; j0 += fc) {
    const int nj = F - j0 < fc ? F - j0 : fc;
    __syncthreads();  // (the previous chunk is done with w1)
    for (int e = threadIdx.x; e < nj * D2; e += 256) w1[(e / D2) * ds + e % D2] = a.p.fc1_w[(int64_t)j0 * D2 + e];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = threadIdx.x + 256 * u;
      if (c < D2) {
        for (int jj = 0; jj < nj; ++jj) {
          const float wv = w1[jj * ds + c];
          const float* dr = da1 + j0 + jj;  // (a broadcast read per row)
#pragma unroll
          for (int r = 0; r < HR; ++r) dh[u][r] = fmaf(dr[r * F], wv, dh[u][r]);
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = threadIdx.x + 256 * u;
    if (c < D2) {
      double sb = 0.0, sg = 0.0;
#pragma unroll
      for (int r = 0; r < HR; ++r) {
        const float s = dh[u][r];
        a.dh0[(r0 + r) * D2 + c] = s;
        const float xhat = h0[r * ds + c];
        sb += s;
        sg += (double)s * xhat;
      }
      pp[c] = sb;
      pp[D2 + c] = sg;
    }
  }
}

// dpooled = the pooled half of BN0's input gradient (padding columns zeroed);
// one thread per (row, column), independent loads
__global__ __launch_bounds__(256) void head_bwd0(HeadArgs a) {
  const int64_t r0 = (int64_t)blockIdx.x * HR;
  const int D2 = a.D2, d = a.d, ld = (int)a.ld;
  const float invB = 1.f / (float)a.B;
  for (int e = threadIdx.x; e < HR * ld; e += 256) {
    const int r = e / ld, cc = e % ld, c = d + cc;
    float v = 0.f;
    if (cc < d) {
      const float m = a.stat0[c], iv = a.stat0[D2 + c];
      const float sb = (float)a.sum5[c], sg = (float)a.sum5[D2 + c];
      const float xhat = (hx(a, r0 + r, c) - m) * iv;
      v = iv * a.p.bn0_w[c] * (a.dh0[(r0 + r) * D2 + c] - sb * invB - xhat * sg * invB);
    }
    a.dpooled[(r0 + r) * a.ld + cc] = v;
  }
}

// parameter gradients from the reduced sums (one thread per element)
__global__ void head_grads(HeadArgs a) {
  const int D2 = a.D2, F = a.F, F2 = a.F2;
  const int n_w1 = F * D2;
  const int total = n_w1 + F + D2 + F2 * F + F2 + F + F2 + 1 + F2;  // BN entries write weight and bias
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    int o = i;
    if (o < n_w1) { a.p.g_fc1_w[o] = (float)a.sumw1[o]; continue; }
    o -= n_w1;
    if (o < F) { a.p.g_fc1_b[o] = (float)a.sum5[2 * D2 + o]; continue; }
    o -= F;
    if (o < D2) {  // BN0 weight: sum dh0 * xhat0; bias: sum dh0
      a.p.g_bn0_w[o] = (float)a.sum5[D2 + o];
      a.p.g_bn0_b[o] = (float)a.sum5[o];
      continue;
    }
    o -= D2;
    if (o < F2 * F) { a.p.g_fc2_w[o] = (float)a.sum4[2 * F + o]; continue; }
    o -= F2 * F;
    if (o < F2) { a.p.g_fc2_b[o] = (float)a.sum4[2 * F + F2 * F + o]; continue; }
    o -= F2;
    if (o < F) {
      a.p.g_bn1_w[o] = (float)a.sum4[F + o];
      a.p.g_bn1_b[o] = (float)a.sum4[o];
      continue;
    }
    o -= F;
    if (o < F2) { a.p.g_fc3_w[o] = (float)a.sum3[2 * F2 + o]; continue; }
    o -= F2;
    if (o < 1) {
      a.p.g_fc3_b[0] = (float)a.sum3[3 * F2];
      *a.loss = (float)(a.sum3[3 * F2 + 1] / a.B);
      continue;
    }
    o -= 1;
    if (o < F2) {
      a.p.g_bn2_w[o] = (float)a.sum3[F2 + o];
      a.p.g_bn2_b[o] = (float)a.sum3[o];
    }
  }
}

// ============================================ fast head (fc_units == 32) ==
// The same train-mode head in 8 launches instead of 15: every BatchNorm's
// batch statistics are summed in the PROLOGUE of the kernel that needs them
// (fixed block order, fp64) instead of by a separate colsum launch, and the
// two 2d-wide layers run on f32 MFMA (v_mfma_f32_32x32x2_f32: exact f32
// products, f32 accumulation):
//   hf_stats0  BN0 partial sums over 16 row groups x 32-column groups
//   hf_fwd1    BN0 -> Linear(2d,32) (MFMA, K split over the 4 waves) -> ReLU -> Dropout
//   head_fwd2 / head_fwd3 / head_bwd2 (a.fast: prologue sums)
//   hf_bwd1    BN1 bwd -> da1;  G = da1^T xhat0 per block (MFMA), sum da1
//   hf_reduce_c1  G, sum da1 and the small layers' partials -> every head gradient;
//              BN0's backward sums follow from G: sum_r dh0 = W1^T sum da1,
//              sum_r dh0 xhat0 = sum_j W1[j] G[j]  (dh0 = da1 W1, never stored)
//   hf_bwd0    dh0 (pooled half) = da1 W1 (MFMA) -> BN0 bwd -> dpooled
constexpr int HF = 32;  // fc_units of the fast path

__device__ __forceinline__ int hacc_row(int g, int h) { return (g & 3) + 8 * (g >> 2) + 4 * h; }

__global__ __launch_bounds__(256) void hf_stats0(HeadArgs a) {
  const int ncg = a.D2 / 32;
  const int cg = blockIdx.x % ncg, rg = blockIdx.x / ncg;
  const int cl = threadIdx.x & 31, ph = threadIdx.x >> 5;
  const int c = 32 * cg + cl;
  const int rows = a.B / a.nrg0;
  const int64_t r0 = (int64_t)rg * rows;
  double sv = 0.0, ssv = 0.0;
#pragma unroll 8
  for (int r = ph; r < rows; r += 8) {
    const double v = hx(a, r0 + r, c);
    sv += v;
    ssv += v * v;
  }
  __shared__ double red[2][8][32];
  red[0][ph][cl] = sv;
  red[1][ph][cl] = ssv;
  __syncthreads();
  if (threadIdx.x < 64) {
    const int wch = threadIdx.x >> 5;
    double t = 0.0;
    for (int q = 0; q < 8; ++q) t += red[wch][q][cl];
    a.part0[(int64_t)rg * 2 * a.D2 + wch * a.D2 + c] = t;
  }
}

// LDS (floats): mean/inv [D2] x 2 | h0 [32][D2+4] | red [4][32][32] | d1 [32][33]
// NX = D2 / 32: float4 of the block's x rows per thread (issued before the
// prologue's partial sums, so the two memory round trips overlap).  W1 (fc.1
// weight, L2-resident: every block reads it) goes to registers for D2 <= 256; for
// D2 > 256 (d = 256, the reference's width) the MFMA reads its rows from global
// memory.  (An LDS tile of W1 cost a dependent round trip before the h0 phase.)
template <int NX>
__global__ __launch_bounds__(256) void hf_fwd1(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ double pro_tmp[256], pro_sum[1024];
  constexpr int D2 = NX * 32, hs = D2 + 4, q4 = D2 / 4;
  // W1 stays in registers (the lane's 32 x D2/8 slice: loaded right after the
  // prologue's partial sums, in flight through the BN0 finalise and the h0 phase)
  // where it fits; the LDS tile costs a dependent round trip before the h0 phase
  constexpr bool W1_REG = NX <= 8;
  const int t = threadIdx.x;
  float* mean = sm;
  float* inv = mean + D2;
  float* h0 = inv + D2;
  float* red = h0 + HR * hs;
  float* d1 = red + 4 * HR * HF;
  const int64_t r0 = (int64_t)blockIdx.x * HR;
  float4 xv[NX];
#pragma unroll
  for (int u = 0; u < NX; ++u) {
    const int e = t + u * 256;
    xv[u] = hx4(a, r0 + e / q4, 4 * (e % q4));
  }
  // the step counter and block 0's running statistics are loaded with the rows,
  // ahead of the prologue's partial sums (W1 after: measured slower ahead of them)
  const float stepv = *a.step;
  const RunStatPre rsp = run_stat_pre(a.p.bn0_rm, a.p.bn0_rv, a.p.bn0_nb, D2, blockIdx.x == 0);
  // this thread's BN0 affine columns (4 (t % q4) .. +3 for every u when 256 % q4 == 0)
  // and fc.1 bias entry (t % 32 for every output it writes), loaded with the rows
  constexpr bool G0_PRE = 256 % q4 == 0;
  const float4 g0 = G0_PRE ? *reinterpret_cast<const float4*>(a.p.bn0_w + 4 * (t % q4)) : float4{};
  const float4 be0 = G0_PRE ? *reinterpret_cast<const float4*>(a.p.bn0_b + 4 * (t % q4)) : float4{};
  const float b1j = a.p.fc1_b[t % HF];
  colsum_prologue(a.part0, a.nrg0, 2 * D2, 2 * D2, pro_tmp, pro_sum);
  float4 w1r[W1_REG ? D2 / 32 : 1];
  if constexpr (W1_REG) {
    const int lane = t & 63, w = t >> 6, i = lane & 31, h = lane >> 5;
    const float* br = a.p.fc1_w + (int64_t)i * D2 + h * (D2 / 2) + w * (D2 / 8);
#pragma unroll
    for (int u = 0; u < D2 / 32; ++u) w1r[u] = *reinterpret_cast<const float4*>(br + 4 * u);
  }
  bn_finalize_pre(a, pro_sum, D2, mean, inv, a.stat0, a.p.bn0_rm, a.p.bn0_rv, a.p.bn0_nb, blockIdx.x == 0, rsp);
  __syncthreads();  // mean / inv published
#pragma unroll
  for (int u = 0; u < NX; ++u) {
    const int e = t + u * 256, row = e / q4, c = 4 * (e % q4);
    float4 x = xv[u];
    const float4 gu = G0_PRE ? g0 : *reinterpret_cast<const float4*>(a.p.bn0_w + c);
    const float4 bu = G0_PRE ? be0 : *reinterpret_cast<const float4*>(a.p.bn0_b + c);
    x.x = (x.x - mean[c]) * inv[c] * gu.x + bu.x;
    x.y = (x.y - mean[c + 1]) * inv[c + 1] * gu.y + bu.y;
    x.z = (x.z - mean[c + 2]) * inv[c + 2] * gu.z + bu.z;
    x.w = (x.w - mean[c + 3]) * inv[c + 3] * gu.w + bu.w;
    *reinterpret_cast<float4*>(h0 + row * hs + c) = x;
  }
  __syncthreads();
  {  // a1 = h0 W1^T: lane half h covers k in [h D2/2, (h+1) D2/2), wave w a quarter of that
    const int lane = t & 63, w = t >> 6, i = lane & 31, h = lane >> 5;
    constexpr int kw = D2 / 8;
    const float* ar = h0 + i * hs + h * (D2 / 2) + w * kw;
    const float* br = a.p.fc1_w + (int64_t)i * D2 + h * (D2 / 2) + w * kw;
    f32x16 acc;
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[g] = 0.f;
#pragma unroll
    for (int kk = 0; kk < kw; kk += 4) {
      const float4 av = *reinterpret_cast<const float4*>(ar + kk);
      float4 bv;
      if constexpr (W1_REG) bv = w1r[kk / 4];
      else bv = *reinterpret_cast<const float4*>(br + kk);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv.w, acc, 0, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) red[w * HR * HF + hacc_row(g, h) * HF + i] = acc[g];
  }
  __syncthreads();
  for (int o = t; o < HR * HF; o += 256) {
    const int r = o / HF, j = o % HF;
    const float v = ((red[o] + red[HR * HF + o]) + (red[2 * HR * HF + o] + red[3 * HR * HF + o])) + b1j;
    a.a1[(r0 + r) * HF + j] = v;
    const float ks = keep_scale_s(a, stepv, 1, r0 + r, j);
    d1[r * (HF + 1) + j] = fmaxf(v, 0.f) * ks;
    if (a.p_drop > 0.f) {  // the keep bits of this wave's two rows, for the later kernels
      const uint64_t bits = __ballot(ks != 0.f);
      if ((t & 63) == 0) *reinterpret_cast<uint64_t*>(a.mask1 + r0 + r) = bits;
    }
  }
  __syncthreads();
  {  // BN1 partial sums: {sum, sum sq} x 32 columns x 4 row groups of 8, combined in a fixed order
    __shared__ double p1[4][2 * HF];
    const int o = t & 63, rq = t >> 6, j = o % HF, sq = o / HF;
    double acc = 0.0;
#pragma unroll
    for (int r = 8 * rq; r < 8 * rq + 8; ++r) {
      const double v = d1[r * (HF + 1) + j];
      acc += sq ? v * v : v;
    }
    p1[rq][o] = acc;
    __syncthreads();
    if (t < 2 * HF) a.part1[(int64_t)blockIdx.x * 2 * HF + t] = (p1[0][t] + p1[1][t]) + (p1[2][t] + p1[3][t]);
  }
}

// LDS (floats): m0/i0 [DC] x 2 | xhat0 [32][DC+4] | da1 [32][33] | m1/i1/sb1/sg1 [32] x 4 | gT [DC][36]
// CS column splits: block b covers rows 32 (b / CS) .. and the DC = D2 / CS columns
// from (b % CS) DC (every split forms the block's da1; split 0 writes it and its sum),
// so the x̂0 loads and the G MFMAs of a row block spread over CS CUs
template <int NX, int CS>
__global__ __launch_bounds__(256) void hf_bwd1(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ double pro_tmp[256], pro_sum[64];
  constexpr int D2 = NX * 32, DC = D2 / CS, hs = DC + 4;
  static_assert(NX % CS == 0, "column split of whole 32-column tiles");
  const int t = threadIdx.x;
  const int rb = (int)blockIdx.x / CS, hh = (int)blockIdx.x % CS, cbase = hh * DC;
  float* m0 = sm;
  float* i0 = m0 + DC;
  float* xh = i0 + DC;
  float* da = xh + HR * hs;
  float* m1 = da + HR * (HF + 1);
  float* i1 = m1 + HF;
  float* sb1 = i1 + HF;
  float* sg1 = sb1 + HF;
  const int64_t r0 = (int64_t)rb * HR;
  const int s4 = 2 * HF + a.F2 * HF + a.F2;
  constexpr int q4 = DC / 4;
  // every load of the block's rows first, then the prologue's partial sums
  float4 xv[NX / CS];
#pragma unroll
  for (int u = 0; u < NX / CS; ++u) {
    const int e = t + u * 256;
    xv[u] = hx4(a, r0 + e / q4, cbase + 4 * (e % q4));
  }
  float a1v[HR * HF / 256], dhv[HR * HF / 256];
#pragma unroll
  for (int u = 0; u < HR * HF / 256; ++u) {
    const int e = t + u * 256;
    a1v[u] = a.a1[r0 * HF + e];
    dhv[u] = a.dh1[r0 * HF + e];
  }
  const float g1j = a.p.bn1_w[t % HF];  // the BN1 weight of every element this thread forms
  uint32_t mw[HR * HF / 256];           // fc.2 keep bits of rows (t >> 5) + 8 u
#pragma unroll
  for (int u = 0; u < HR * HF / 256; ++u) mw[u] = a.p_drop > 0.f ? a.mask1[r0 + (t >> 5) + 8 * u] : 0u;
  for (int c = t; c < DC; c += 256) {
    m0[c] = a.stat0[cbase + c];
    i0[c] = a.stat0[D2 + cbase + c];
  }
  load_stat(a.stat1, HF, m1, i1);
  colsum_prologue(a.part4, a.nblk, s4, 2 * HF, pro_tmp, pro_sum);
  if (t < HF) {
    sb1[t] = (float)pro_sum[t];
    sg1[t] = (float)pro_sum[HF + t];
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < NX / CS; ++u) {
    const int e = t + u * 256, row = e / q4, c = 4 * (e % q4);
    float4 x = xv[u];
    x.x = (x.x - m0[c]) * i0[c];
    x.y = (x.y - m0[c + 1]) * i0[c + 1];
    x.z = (x.z - m0[c + 2]) * i0[c + 2];
    x.w = (x.w - m0[c + 3]) * i0[c + 3];
    *reinterpret_cast<float4*>(xh + row * hs + c) = x;
  }
  const float invB = 1.f / (float)a.B;
  {
#pragma unroll
    for (int u = 0; u < HR * HF / 256; ++u) {
      const int e = t + u * 256, r = e / HF, j = e % HF;
      const float ks = keep_bit(a, mw[u], j);
      const float xhat = (fmaxf(a1v[u], 0.f) * ks - m1[j]) * i1[j];
      const float dd1 = i1[j] * g1j * (dhv[u] - sb1[j] * invB - xhat * sg1[j] * invB);
      const float v = a1v[u] > 0.f ? dd1 * ks : 0.f;
      da[r * (HF + 1) + j] = v;
      if (hh == 0) a.da1[(r0 + r) * HF + j] = v;  // (not in place: the other split still reads dh1)
    }
  }
  __syncthreads();
  {  // G (32 x DC) = da1^T xhat0 over the block's 32 rows; wave w: column tiles w, w+4, ...
     // stored column-major per row block ([D2][32]: a column's 32 entries are one 128-B
     // line, hf_reduce_c1 reads one line per partial block).  The tile goes through
     // LDS (gT [DC][36]) so the global stores are whole lines: scattered 4-B stores
     // of 64 lines per instruction left partially written lines
    const int lane = t & 63, w = t >> 6, i = lane & 31, h = lane >> 5;
    float* gT = sg1 + HF;  // [DC][36] after the BN1 constants
    for (int ct = w; ct < DC / 32; ct += 4) {
      f32x16 acc;
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[g] = 0.f;
#pragma unroll 4
      for (int kk = 0; kk < HR / 2; ++kk) {
        const int row = 2 * kk + h;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(da[row * (HF + 1) + i], xh[row * hs + 32 * ct + i], acc, 0, 0, 0);
      }
#pragma unroll
      for (int g = 0; g < 16; ++g) gT[(32 * ct + i) * 36 + hacc_row(g, h)] = acc[g];
    }
    __syncthreads();
    float4* pg4 = reinterpret_cast<float4*>(a.pw1 + (int64_t)rb * HF * D2 + (int64_t)cbase * HF);
#pragma unroll 4
    for (int e = t; e < DC * HF / 4; e += 256) {
      const int c = e >> 3, qd = e & 7;
      pg4[e] = *reinterpret_cast<const float4*>(gT + c * 36 + 4 * qd);
    }
  }
  if (hh == 0) {  // sum da1 over the block's rows: 32 columns x 8 row groups of 4, fixed-order combine
    __shared__ double p5[8][HF];
    const int j = t & 31, rq = t >> 5;
    double acc = 0.0;
#pragma unroll
    for (int r = 4 * rq; r < 4 * rq + 4; ++r) acc += da[r * (HF + 1) + j];
    p5[rq][j] = acc;
    __syncthreads();
    if (t < HF)
      a.part5[(int64_t)rb * HF + t] = ((p5[0][t] + p5[1][t]) + (p5[2][t] + p5[3][t])) +
                                      ((p5[4][t] + p5[5][t]) + (p5[6][t] + p5[7][t]));
  }
}

// Every head gradient from the block partials (fixed order, fp64), ONE column of
// G per block (256 threads = 8 phases x 32 j, all 16 loads of a thread in flight
// at once): the 4 MB of G partials are read by D2 blocks spread over the chip (a
// 4-column form on D2 / 4 blocks spent 5.8 us in its G phase).  g_fc1_w[j][c] = bn0_w[c] G[j][c] + bn0_b[c] S[j],
// g_bn0_b[c] = sum_j W1[j][c] S[j], g_bn0_w[c] = sum_j W1[j][c] G[j][c] (and sum5).
// Blocks after: 64 columns each of the small layers' partials, 4 phases.
__global__ __launch_bounds__(256) void hf_reduce_c1(HeadArgs a) {
  const int D2 = a.D2, F2 = a.F2, t = threadIdx.x, nblk = a.nblk;
  if ((int)blockIdx.x < D2) {
    const int c = blockIdx.x;
    __shared__ double red[8][32], sred[8][32], Gt[32], St[32];
    const int ph = t >> 5, j = t & 31;
    const float wj = t < 32 ? a.p.fc1_w[(int64_t)j * D2 + c] : 0.f;
    const float bw0 = a.p.bn0_w[c], bb0 = a.p.bn0_b[c];
    double acc = 0.0, s5 = 0.0;
    for (int b0 = ph; b0 < nblk; b0 += 8 * 16) {
      float v[16];
      double w5[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int b = b0 + 8 * u;
        v[u] = b < nblk ? a.pw1[(int64_t)b * HF * D2 + (int64_t)c * HF + j] : 0.f;
        w5[u] = b < nblk ? a.part5[(int64_t)b * HF + j] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        acc += (double)v[u];
        s5 += w5[u];
      }
    }
    red[ph][j] = acc;
    sred[ph][j] = s5;
    __syncthreads();
    if (t < 32) {
      double g = 0.0, s = 0.0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        g += red[q][t];
        s += sred[q][t];
      }
      Gt[t] = g;
      St[t] = s;
      a.p.g_fc1_w[(int64_t)t * D2 + c] = (float)(bw0 * g + bb0 * s);
    }
    __syncthreads();
    if (t < 64) {  // sums over j on wave 0 (lanes 32..63 add zeros)
      double sb = t < 32 ? (double)wj * St[t] : 0.0, sg = t < 32 ? (double)wj * Gt[t] : 0.0;
      sb = wave_sum(sb);
      sg = wave_sum(sg);
      if (t == 0) {
        a.p.g_bn0_b[c] = (float)sb;
        a.p.g_bn0_w[c] = (float)sg;
        a.sum5[c] = sb;
        a.sum5[D2 + c] = sg;
      }
    }
    if (c == 0 && t < HF) a.p.g_fc1_b[t] = (float)St[t];
    return;
  }
  // small layers: column q of the concatenation [part3 (3F2+2) | part4 (2F + F2 F + F2)]
  __shared__ double sr[4][64];
  const int s3 = 3 * F2 + 2, s4 = 2 * HF + F2 * HF + F2;
  const int cl = t & 63, ph = t >> 6;
  const int q = ((int)blockIdx.x - D2) * 64 + cl;
  const bool valid = q < s3 + s4;
  double acc = 0.0;
  if (valid) {
    const double* src = q < s3 ? a.part3 + q : a.part4 + (q - s3);
    const int stride = q < s3 ? s3 : s4;
    for (int b0 = ph; b0 < nblk; b0 += 4 * 32) {
      double v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        const int b = b0 + 4 * u;
        v[u] = b < nblk ? src[(int64_t)b * stride] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 32; ++u) acc += v[u];
    }
  }
  sr[ph][cl] = acc;
  __syncthreads();
  if (t < 64 && valid) {
    const double v = (sr[0][t] + sr[1][t]) + (sr[2][t] + sr[3][t]);
    if (q < s3) {
      if (q < F2) a.p.g_bn2_b[q] = (float)v;
      else if (q < 2 * F2) a.p.g_bn2_w[q - F2] = (float)v;
      else if (q < 3 * F2) a.p.g_fc3_w[q - 2 * F2] = (float)v;
      else if (q == 3 * F2) a.p.g_fc3_b[0] = (float)v;
      else *a.loss = (float)(v / a.B);
    } else {
      const int o = q - s3;
      if (o < HF) a.p.g_bn1_b[o] = (float)v;
      else if (o < 2 * HF) a.p.g_bn1_w[o - HF] = (float)v;
      else if (o < 2 * HF + F2 * HF) a.p.g_fc2_w[o - 2 * HF] = (float)v;
      else a.p.g_fc2_b[o - 2 * HF - F2 * HF] = (float)v;
    }
  }
}

// ---- the small layers of the fast head (F = 32, F/2 = 16, 32 rows per block).
// Every global load of the block's rows and weights is issued before the
// prologue's partial sums (one memory round trip instead of two), and the
// column sums over the block's rows run as row-group partials combined in a
// fixed order (no 32-step dependent LDS chains): the kernels are latency-bound.
constexpr int HF2 = HF / 2;

// BN1 (prologue sums) -> Linear(32, 16) -> ReLU -> Dropout; BN2 partial sums
__global__ __launch_bounds__(256) void hf_fwd2(HeadArgs a) {
  __shared__ __attribute__((aligned(16))) float h1[HR][HF + 4];
  __shared__ __attribute__((aligned(16))) float w2[HF2][HF + 4];
  __shared__ float d2[HR][HF2 + 1];
  __shared__ float mean[HF], inv[HF], b2s[HF2];
  __shared__ double red[2][16][HF2];
  __shared__ double pro_tmp[256], pro_sum[2 * HF];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * HR;
  const float stepv = *a.step;
  const float4 av = reinterpret_cast<const float4*>(a.a1 + r0 * HF)[t];  // row t/8, cols 4(t%8)..
  const uint32_t mw1 = a.p_drop > 0.f ? a.mask1[r0 + (t >> 3)] : 0u;      // its fc.2 keep bits
  float4 wv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (t < HF2 * HF / 4) wv = reinterpret_cast<const float4*>(a.p.fc2_w)[t];
  const float gw = t < HF ? a.p.bn1_w[t] : 0.f, gb = t < HF ? a.p.bn1_b[t] : 0.f;
  if (t < HF2) b2s[t] = a.p.fc2_b[t];
  const RunStatPre rsp = run_stat_pre(a.p.bn1_rm, a.p.bn1_rv, a.p.bn1_nb, HF, blockIdx.x == 0);
  colsum_prologue(a.part1, a.nblk, 2 * HF, 2 * HF, pro_tmp, pro_sum);
  bn_finalize_pre(a, pro_sum, HF, mean, inv, a.stat1, a.p.bn1_rm, a.p.bn1_rv, a.p.bn1_nb, blockIdx.x == 0, rsp);
  __shared__ float gws[HF], gbs[HF];
  if (t < HF) {
    gws[t] = gw;
    gbs[t] = gb;
  }
  __syncthreads();
  {
    const int r = t >> 3, j0 = (t & 7) * 4;
    const float x[4] = {av.x, av.y, av.z, av.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + u;
      const float d1 = fmaxf(x[u], 0.f) * keep_bit(a, mw1, j);
      h1[r][j] = (d1 - mean[j]) * inv[j] * gws[j] + gbs[j];
    }
    if (t < HF2 * HF / 4) *reinterpret_cast<float4*>(&w2[t >> 3][(t & 7) * 4]) = wv;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; ++u) {  // a2 = h1 W2^T + b2: 512 outputs
    const int o = t + 256 * u, r = o >> 4, k = o & 15;
    float4 hv[HF / 4], wq[HF / 4];
#pragma unroll
    for (int i = 0; i < HF / 4; ++i) {
      hv[i] = *reinterpret_cast<const float4*>(&h1[r][4 * i]);
      wq[i] = *reinterpret_cast<const float4*>(&w2[k][4 * i]);
    }
    float c0 = b2s[k], c1 = 0.f, c2 = 0.f, c3 = 0.f;
#pragma unroll
    for (int i = 0; i < HF / 4; ++i) {
      c0 = fmaf(hv[i].x, wq[i].x, c0);
      c1 = fmaf(hv[i].y, wq[i].y, c1);
      c2 = fmaf(hv[i].z, wq[i].z, c2);
      c3 = fmaf(hv[i].w, wq[i].w, c3);
    }
    const float acc = (c0 + c1) + (c2 + c3);
    a.a2[(r0 + r) * HF2 + k] = acc;
    const float ks = keep_scale_s(a, stepv, 2, r0 + r, k);
    d2[r][k] = fmaxf(acc, 0.f) * ks;
    if (a.p_drop > 0.f) {  // the keep bits of this wave's four rows
      const uint64_t bits = __ballot(ks != 0.f);
      if ((t & 63) == 0) *reinterpret_cast<uint64_t*>(a.mask2 + r0 + r) = bits;
    }
  }
  __syncthreads();
  {  // BN2 partial sums: 16 columns x 16 groups of 2 rows
    const int k = t & 15, g = t >> 4;
    const double v0 = d2[2 * g][k], v1 = d2[2 * g + 1][k];
    red[0][g][k] = v0 + v1;
    red[1][g][k] = v0 * v0 + v1 * v1;
  }
  __syncthreads();
  if (t < 2 * HF2) {
    const int which = t >> 4, k = t & 15;
    double s = 0.0;
#pragma unroll
    for (int g = 0; g < 16; ++g) s += red[which][g][k];
    a.part2[(int64_t)blockIdx.x * 2 * HF2 + which * HF2 + k] = s;
  }
}

// BN2 (prologue sums) -> Linear(16, 1) -> BCEWithLogits (mean); dlogit;
// dh2 = dlogit w3; BN2-backward and fc3 partial sums, loss partial
__global__ __launch_bounds__(256) void hf_fwd3(HeadArgs a) {
  __shared__ float h2[HR][HF2 + 1], xh[HR][HF2 + 1];
  __shared__ float mean[HF2], inv[HF2], w3[HF2], gw2[HF2], gb2[HF2], dl[HR], lo[HR];
  __shared__ double red[3][16][HF2];
  __shared__ double pro_tmp[256], pro_sum[2 * HF2];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * HR;
  float4 av = make_float4(0.f, 0.f, 0.f, 0.f);
  if (t < HR * HF2 / 4) av = reinterpret_cast<const float4*>(a.a2 + r0 * HF2)[t];  // row t/4, cols 4(t%4)..
  const float yv = t < HR ? a.y[r0 + t] : 0.f;
  const uint32_t mw2 = a.p_drop > 0.f && t < HR * HF2 / 4 ? a.mask2[r0 + (t >> 2)] : 0u;  // fc.6 keep bits
  const float b3 = a.p.fc3_b[0];
  if (t < HF2) {
    w3[t] = a.p.fc3_w[t];
    gw2[t] = a.p.bn2_w[t];
    gb2[t] = a.p.bn2_b[t];
  }
  const RunStatPre rsp = run_stat_pre(a.p.bn2_rm, a.p.bn2_rv, a.p.bn2_nb, HF2, blockIdx.x == 0);
  colsum_prologue(a.part2, a.nblk, 2 * HF2, 2 * HF2, pro_tmp, pro_sum);
  bn_finalize_pre(a, pro_sum, HF2, mean, inv, a.stat2, a.p.bn2_rm, a.p.bn2_rv, a.p.bn2_nb, blockIdx.x == 0, rsp);
  __syncthreads();
  if (t < HR * HF2 / 4) {
    const int r = t >> 2, k0 = (t & 3) * 4;
    const float x4[4] = {av.x, av.y, av.z, av.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u;
      const float d2 = fmaxf(x4[u], 0.f) * keep_bit(a, mw2, k);
      const float x = (d2 - mean[k]) * inv[k];
      xh[r][k] = x;
      h2[r][k] = x * gw2[k] + gb2[k];
    }
  }
  __syncthreads();
  if (t < HR) {
    float z = b3;
#pragma unroll
    for (int k = 0; k < HF2; ++k) z = fmaf(h2[t][k], w3[k], z);
    a.logits[r0 + t] = z;
    lo[t] = fmaxf(z, 0.f) - z * yv + log1pf(expf(-fabsf(z)));
    dl[t] = (1.f / (1.f + expf(-z)) - yv) / (float)a.B;
  }
  __syncthreads();
  if (t < HR * HF2 / 4) {
    const int r = t >> 2, k0 = (t & 3) * 4;
    reinterpret_cast<float4*>(a.dh2 + r0 * HF2)[t] =
        make_float4(dl[r] * w3[k0], dl[r] * w3[k0 + 1], dl[r] * w3[k0 + 2], dl[r] * w3[k0 + 3]);
  }
  {  // partials: 16 columns x 16 groups of 2 rows
    const int k = t & 15, g = t >> 4;
    double sb = 0.0, sg = 0.0, sw = 0.0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = 2 * g + i;
      const double gg = (double)dl[r] * w3[k];
      sb += gg;
      sg += gg * xh[r][k];
      sw += (double)dl[r] * h2[r][k];
    }
    red[0][g][k] = sb;
    red[1][g][k] = sg;
    red[2][g][k] = sw;
  }
  __syncthreads();
  double* pp = a.part3 + (int64_t)blockIdx.x * (3 * HF2 + 2);
  if (t < 3 * HF2) {
    const int which = t >> 4, k = t & 15;
    double s = 0.0;
#pragma unroll
    for (int g = 0; g < 16; ++g) s += red[which][g][k];
    pp[which * HF2 + k] = s;
  } else if (t >= 64 && t < 128) {  // one wave: sum dlogit and the loss over the rows
    const int l = t - 64;
    const double s = wave_sum(l < HR ? (double)dl[l] : 0.0);
    const double ls = wave_sum(l < HR ? (double)lo[l] : 0.0);
    if (l == 0) {
      pp[3 * HF2] = s;
      pp[3 * HF2 + 1] = ls;
    }
  }
}

// BN2 backward (prologue sums) -> Dropout/ReLU backward -> Linear(32, 16)
// backward (dW2, db2, dh1 = da2 W2); BN1-backward partial sums
__global__ __launch_bounds__(256) void hf_bwd2(HeadArgs a) {
  __shared__ __attribute__((aligned(16))) float h1[HR][HF + 4];
  __shared__ __attribute__((aligned(16))) float xh1[HR][HF + 4];
  __shared__ float da2[HR][HF2 + 1];
  __shared__ float w2[HF2][HF + 1];
  __shared__ float m1[HF], i1[HF], g1[HF], b1[HF], m2[HF2], i2[HF2], g2[HF2], sb2[HF2], sg2[HF2];
  __shared__ double red[2][8][HF];
  __shared__ double pro_tmp[256], pro_sum[2 * HF2];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * HR;
  // every load of the block first
  const float4 a1v = reinterpret_cast<const float4*>(a.a1 + r0 * HF)[t];  // row t/8, cols 4(t%8)..
  const uint32_t mw1 = a.p_drop > 0.f ? a.mask1[r0 + (t >> 3)] : 0u;
  const uint32_t mw2 = a.p_drop > 0.f && t < HR * HF2 / 4 ? a.mask2[r0 + (t >> 2)] : 0u;
  float4 a2v = make_float4(0.f, 0.f, 0.f, 0.f), dhv = a2v, wv = a2v;
  if (t < HR * HF2 / 4) {
    a2v = reinterpret_cast<const float4*>(a.a2 + r0 * HF2)[t];  // row t/4, cols 4(t%4)..
    dhv = reinterpret_cast<const float4*>(a.dh2 + r0 * HF2)[t];
    wv = reinterpret_cast<const float4*>(a.p.fc2_w)[t];  // row t/8 of W2 (16 x 32)
  }
  if (t < HF) {
    m1[t] = a.stat1[t];
    i1[t] = a.stat1[HF + t];
    g1[t] = a.p.bn1_w[t];
    b1[t] = a.p.bn1_b[t];
  } else if (t >= 64 && t < 64 + HF2) {
    const int k = t - 64;
    m2[k] = a.stat2[k];
    i2[k] = a.stat2[HF2 + k];
    g2[k] = a.p.bn2_w[k];
  }
  colsum_prologue(a.part3, a.nblk, 3 * HF2 + 2, 2 * HF2, pro_tmp, pro_sum);
  if (t < HF2) {
    sb2[t] = (float)pro_sum[t];
    sg2[t] = (float)pro_sum[HF2 + t];
  }
  __syncthreads();
  const float invB = 1.f / (float)a.B;
  {
    const int r = t >> 3, j0 = (t & 7) * 4;
    const float x4[4] = {a1v.x, a1v.y, a1v.z, a1v.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + u;
      const float d1 = fmaxf(x4[u], 0.f) * keep_bit(a, mw1, j);
      const float x = (d1 - m1[j]) * i1[j];
      xh1[r][j] = x;
      h1[r][j] = x * g1[j] + b1[j];
    }
  }
  if (t < HR * HF2 / 4) {
    const int r = t >> 2, k0 = (t & 3) * 4;
    const float a4[4] = {a2v.x, a2v.y, a2v.z, a2v.w}, d4[4] = {dhv.x, dhv.y, dhv.z, dhv.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u;
      const float ks = keep_bit(a, mw2, k);
      const float xhat = (fmaxf(a4[u], 0.f) * ks - m2[k]) * i2[k];
      const float dd2 = i2[k] * g2[k] * (d4[u] - sb2[k] * invB - xhat * sg2[k] * invB);
      da2[r][k] = a4[u] > 0.f ? dd2 * ks : 0.f;
    }
    const int wr = t >> 3, wc = (t & 7) * 4;
    w2[wr][wc] = wv.x;
    w2[wr][wc + 1] = wv.y;
    w2[wr][wc + 2] = wv.z;
    w2[wr][wc + 3] = wv.w;
  }
  __syncthreads();
  double* pp = a.part4 + (int64_t)blockIdx.x * (2 * HF + HF2 * HF + HF2);
#pragma unroll
  for (int u = 0; u < 2; ++u) {  // dW2[k][j] = sum_r da2[r][k] h1[r][j] (fp64, rows in order)
    const int o = t + 256 * u, k = o >> 5, j = o & 31;
    double s = 0.0;
#pragma unroll 8
    for (int r = 0; r < HR; ++r) s += (double)da2[r][k] * h1[r][j];
    pp[2 * HF + o] = s;
  }
  if (t < HF2) {
    double s = 0.0;
#pragma unroll 8
    for (int r = 0; r < HR; ++r) s += da2[r][t];
    pp[2 * HF + HF2 * HF + t] = s;
  }
  float dh[4];
  {  // dh1 = da2 W2: row t/8, columns 4(t%8)..
    const int r = t >> 3, j0 = (t & 7) * 4;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
#pragma unroll
      for (int k = 0; k < HF2; k += 4) {
        c0 = fmaf(da2[r][k], w2[k][j0 + u], c0);
        c1 = fmaf(da2[r][k + 1], w2[k + 1][j0 + u], c1);
        c2 = fmaf(da2[r][k + 2], w2[k + 2][j0 + u], c2);
        c3 = fmaf(da2[r][k + 3], w2[k + 3][j0 + u], c3);
      }
      dh[u] = (c0 + c1) + (c2 + c3);
    }
    reinterpret_cast<float4*>(a.dh1 + r0 * HF)[t] = make_float4(dh[0], dh[1], dh[2], dh[3]);
  }
  __syncthreads();  // h1 is re-used below as the dh1 image
  {
    const int r = t >> 3, j0 = (t & 7) * 4;
#pragma unroll
    for (int u = 0; u < 4; ++u) h1[r][j0 + u] = dh[u];
  }
  __syncthreads();
  {  // BN1-backward partials: 32 columns x 8 groups of 4 rows
    const int j = t & 31, g = t >> 5;
    double sb = 0.0, sg = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * g + i;
      sb += h1[r][j];
      sg += (double)h1[r][j] * xh1[r][j];
    }
    red[0][g][j] = sb;
    red[1][g][j] = sg;
  }
  __syncthreads();
  if (t < 2 * HF) {
    const int which = t >> 5, j = t & 31;
    double s = 0.0;
#pragma unroll
    for (int g = 0; g < 8; ++g) s += red[which][g][j];
    pp[which * HF + j] = s;
  }
}

// dpooled = BN0 backward of dh0's pooled half, dh0 = da1 W1 on MFMA
// (wave w: 32-column tiles w, w+4, ... of the pooled half).
__global__ __launch_bounds__(256) void hf_bwd0(HeadArgs a) {
  __shared__ float da[HR][HF + 1];
  const int D2 = a.D2, d = a.d, ld = (int)a.ld, t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * HR;
  for (int e = t; e < HR * HF; e += 256) da[e / HF][e % HF] = a.da1[(r0 + e / HF) * HF + e % HF];
  for (int e = t; e < HR * (ld - d); e += 256) a.dpooled[(r0 + e / (ld - d)) * ld + d + e % (ld - d)] = 0.f;
  __syncthreads();
  const float invB = 1.f / (float)a.B;
  const int lane = t & 63, w = t >> 6, i = lane & 31, h = lane >> 5;
  for (int ct = w; ct < d / 32; ct += 4) {
    const int c = d + 32 * ct + i;  // column of x (pooled half)
    f32x16 acc;
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[g] = 0.f;
    float wv[HF / 2], pv[16];  // every global load before the MFMA chain
#pragma unroll
    for (int kk = 0; kk < HF / 2; ++kk) wv[kk] = a.p.fc1_w[(int64_t)(2 * kk + h) * D2 + c];
#pragma unroll
    for (int g = 0; g < 16; ++g) pv[g] = a.pooled[(r0 + hacc_row(g, h)) * ld + (c - d)];
    const float m = a.stat0[c], iv = a.stat0[D2 + c], gw = a.p.bn0_w[c];
    const float sb = (float)a.sum5[c] * invB, sg = (float)a.sum5[D2 + c] * invB;
#pragma unroll
    for (int kk = 0; kk < HF / 2; ++kk)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(da[i][2 * kk + h], wv[kk], acc, 0, 0, 0);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int64_t r = r0 + hacc_row(g, h);
      const float xhat = (pv[g] - m) * iv;
      a.dpooled[r * ld + (c - d)] = iv * gw * (acc[g] - sb - xhat * sg);
    }
  }
}

// ------------------------------------------------- clip_grad_norm_ + Adam --
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, int64_t n, double* __restrict__ part,
                                                    float* __restrict__ step) {
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += (int64_t)gridDim.x * 256 * 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t i = i0 + (int64_t)u * gridDim.x * 256;
      v[u] = i < n ? g[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += (double)v[u] * v[u];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
  if (blockIdx.x == 0 && threadIdx.x == 0) *step += 1.f;  // Adam's step count, read by the next kernel
}

// torch.optim.Adam (L2 weight decay, capturable formulas) after clip_grad_norm_
__global__ __launch_bounds__(256) void clip_adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                        const double* __restrict__ part, int nparts,
                                                        const float* __restrict__ step, float lr,
                                                        const float* __restrict__ lr_dev, float beta1,
                                                        float beta2, float eps, float wd, float max_norm) {
  __shared__ float s_coef;
  if (threadIdx.x < 64) {  // fixed-order sum of the partials: lane-strided, then a fixed butterfly
    double t = 0.0;
    for (int i = threadIdx.x; i < nparts; i += 64) t += part[i];
    t = wave_sum(t);
    if (threadIdx.x == 0) {
      const float norm = (float)sqrt(t);
      const float c = max_norm / (norm + 1e-6f);
      s_coef = c < 1.f ? c : 1.f;
    }
  }
  __syncthreads();
  const float coef = s_coef;
  const float t = *step;
  if (lr_dev) lr = *lr_dev;  // device-resident lr: a scheduler updates it between graph replays
  const float bc1 = 1.f - powf(beta1, t), bc2 = 1.f - powf(beta2, t);
  const float step_size = lr / bc1, bc2_sqrt = sqrtf(bc2);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float gi = g[i] * coef;
    g[i] = gi;  // clip_grad_norm_ scales the stored gradients
    gi = gi + wd * p[i];
    const float mi = m[i] + (gi - m[i]) * (1.f - beta1);  // torch: exp_avg.lerp_(grad, 1 - beta1)
    const float vi = v[i] * beta2 + (1.f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] - step_size * (mi / denom);
  }
}

// clip_grad_norm_ + Adam in ONE launch: every 1024-thread block sums the
// squares of ALL n gradients itself (fixed order, fp64: identical in every
// block, n is ~42K for the DIN model) and updates its own 1024 parameters;
// the block that finishes last advances Adam's step count (every block read
// it before its ticket).  Two launches (partials, then update) cost ~9 us.
__global__ __launch_bounds__(1024) void clip_adam_fused_kernel(float* __restrict__ p, float* __restrict__ g,
                                                              float* __restrict__ m, float* __restrict__ v,
                                                              int64_t n, float* __restrict__ step,
                                                              unsigned int* __restrict__ ticket, float lr,
                                                              const float* __restrict__ lr_dev, float beta1,
                                                              float beta2, float eps, float wd, float max_norm) {
  __shared__ double red[1024];
  const int t = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * 1024 + t;
  // this thread's element first (its loads overlap the norm's)
  float gi = 0.f, pi = 0.f, mi = 0.f, vi = 0.f;
  if (i < n) {
    gi = g[i];
    pi = p[i];
    mi = m[i];
    vi = v[i];
  }
  const float tstep = *step + 1.f;
  if (lr_dev) lr = *lr_dev;  // device-resident lr: a scheduler updates it between graph replays
  // the norm: float4 loads, 12 in flight per thread (the DIN model's ~42K
  // gradients: one round), four fp64 chains, then a fixed butterfly per wave
  // and the 16 wave sums in order
  const int64_t n4 = n >> 2;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  for (int64_t j0 = t; j0 < n4; j0 += 12 * 1024) {
    float4 x[12];
#pragma unroll
    for (int u = 0; u < 12; ++u) {
      const int64_t j = j0 + (int64_t)u * 1024;
      x[u] = j < n4 ? reinterpret_cast<const float4*>(g)[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 12; ++u) {
      s0 += (double)x[u].x * x[u].x;
      s1 += (double)x[u].y * x[u].y;
      s2 += (double)x[u].z * x[u].z;
      s3 += (double)x[u].w * x[u].w;
    }
  }
  if (t < (int)(n & 3)) {
    const float x = g[4 * n4 + t];
    s0 += (double)x * x;
  }
  const double ws = wave_sum((s0 + s1) + (s2 + s3));
  if ((t & 63) == 0) red[t >> 6] = ws;
  __syncthreads();
  if (t == 0) {
    double tot = 0.0;
    for (int w = 0; w < 16; ++w) tot += red[w];
    red[16] = tot;
  }
  __syncthreads();
  const float norm = (float)sqrt(red[16]);
  const float c = max_norm / (norm + 1e-6f);
  const float coef = c < 1.f ? c : 1.f;
  const float bc1 = 1.f - powf(beta1, tstep), bc2 = 1.f - powf(beta2, tstep);
  const float step_size = lr / bc1, bc2_sqrt = sqrtf(bc2);
  if (i < n) {
    gi *= coef;  // the clipped gradient (stored back by the last block, below)
    gi = gi + wd * pi;
    mi = mi + (gi - mi) * (1.f - beta1);  // torch: exp_avg.lerp_(grad, 1 - beta1)
    vi = vi * beta2 + (1.f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = pi - step_size * (mi / denom);
  }
  // clip_grad_norm_ scales the stored gradients.  No block may do that for its
  // own slice: every block reads ALL of g for the norm, and a block that runs
  // late would read gradients another block had already scaled.  Each block's
  // reads of g are complete here (they fed the norm before the barrier above);
  // the block that draws the last ticket scales g in place, after all of them,
  // and advances Adam's step count (every block read *step before its ticket).
  __shared__ bool s_last;
  if (t == 0) {
    __threadfence();
    s_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  if (coef < 1.f) {
    for (int64_t j = t; j < n4; j += 1024) {
      float4 x = reinterpret_cast<float4*>(g)[j];
      x.x *= coef;
      x.y *= coef;
      x.z *= coef;
      x.w *= coef;
      reinterpret_cast<float4*>(g)[j] = x;
    }
    if (t < (int)(n & 3)) g[4 * n4 + t] *= coef;
  }
  if (t == 0) {
    *step = tstep;
    *ticket = 0u;
  }
}

// clip_grad_norm_ + Adam with the squared norm given as fp64 partials (from
// the kernels that wrote the gradients: din_bwd_reduce_params_kernel): every
// block sums the nparts partials in a fixed order, then clips and updates ONLY
// its own 1024 entries (stores its own slice of g: no cross-block read of g);
// the block that draws the last ticket advances Adam's step count.
__global__ __launch_bounds__(1024) void clip_adam_part_kernel(float* __restrict__ p, float* __restrict__ g,
                                                             float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                             float* __restrict__ step, unsigned int* __restrict__ ticket,
                                                             float lr, const float* __restrict__ lr_dev, float beta1,
                                                             float beta2, float eps, float wd, float max_norm,
                                                             const double* __restrict__ part, int nparts) {
  __shared__ double red[17];
  const int t = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * 1024 + t;
  float gi = 0.f, pi = 0.f, mi = 0.f, vi = 0.f;
  if (i < n) {
    gi = g[i];
    pi = p[i];
    mi = m[i];
    vi = v[i];
  }
  const float tstep = *step + 1.f;
  if (lr_dev) lr = *lr_dev;
  double s = 0.0;
  for (int j = t; j < nparts; j += 1024) s += part[j];
  const double ws = wave_sum(s);
  if ((t & 63) == 0) red[t >> 6] = ws;
  __syncthreads();
  if (t == 0) {
    double tot = 0.0;
    for (int w = 0; w < 16; ++w) tot += red[w];
    red[16] = tot;
  }
  __syncthreads();
  const float norm = (float)sqrt(red[16]);
  const float c = max_norm / (norm + 1e-6f);
  const float coef = c < 1.f ? c : 1.f;
  const float bc1 = 1.f - powf(beta1, tstep), bc2 = 1.f - powf(beta2, tstep);
  const float step_size = lr / bc1, bc2_sqrt = sqrtf(bc2);
  if (i < n) {
    gi *= coef;
    g[i] = gi;  // clip_grad_norm_ scales the stored gradients (this block's own entries)
    gi = gi + wd * pi;
    mi = mi + (gi - mi) * (1.f - beta1);
    vi = vi * beta2 + (1.f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = pi - step_size * (mi / denom);
  }
  if (t == 0) {
    __threadfence();
    if (atomicAdd(ticket, 1u) == gridDim.x - 1) {  // every block read *step before its ticket
      *step = tstep;
      *ticket = 0u;
    }
  }
}

}  // namespace nrk

using namespace nrk;

static void head_sizes(int B, int d, int F, int nblk, size_t* off, size_t* total) {
  const int D2 = 2 * d, F2 = F / 2;
  size_t o = 0;
  auto take = [&](int i, size_t bytes) {
    off[i] = o;
    o = align_up(o + bytes, 256);
  };
  take(0, (size_t)nblk * 2 * D2 * 8);                  // part0
  take(1, (size_t)nblk * 2 * F * 8);                   // part1
  take(2, (size_t)nblk * 2 * F2 * 8);                  // part2
  take(3, (size_t)nblk * (3 * F2 + 2) * 8);            // part3
  take(4, (size_t)nblk * (2 * F + F2 * F + F2) * 8);   // part4
  take(5, (size_t)nblk * (2 * D2 + F) * 8);            // part5
  take(6, (size_t)2 * D2 * 4);                         // stat0
  take(7, (size_t)2 * F * 4);                          // stat1
  take(8, (size_t)2 * F2 * 4);                         // stat2
  take(9, (size_t)B * F * 4);                          // a1
  take(10, (size_t)B * F2 * 4);                        // a2
  take(11, (size_t)B * F2 * 4);                        // dh2
  take(12, (size_t)B * F * 4);                         // dh1
  take(13, (size_t)B * D2 * 4);                        // dh0
  take(14, (size_t)nblk * F * D2 * 4);                 // pw1
  take(15, (size_t)(2 * D2 + 2 * F + 2 * F2 + (3 * F2 + 2) + (2 * F + F2 * F + F2) + (2 * D2 + F) + F * D2) * 8);
  take(16, (size_t)B * 4);                             // mask1
  take(17, (size_t)B * 2);                             // mask2
  *total = o;
}

// The train-mode head's state the attention backward needs when it forms
// dpooled itself (nrk_din_attn_bwd_params_head): BN0's finalised statistics
// {mean [2d], invstd [2d]}, its backward sums {sum dh0 [2d], sum dh0 xhat0 [2d]}
// (fp64) and da1 [B][F] (the gradient at fc.1's output), inside `ws` after
// nrk_din_head_train on the fast path (F = 32).
extern "C" int nrk_din_head_ws_views(int32_t B, int32_t d, int32_t F, const void* ws, size_t ws_bytes,
                                     const float** stat0, const double** sum5, const float** da1) {
  NRK_CHECK_ARG(ws && stat0 && sum5 && da1 && B > 1 && d > 0 && F >= 2, "din_head_ws_views: bad arguments");
  size_t off[18], total = 0;
  head_sizes(B, d, F, (int)cdiv(B, HR), off, &total);
  if (ws_bytes < total) return fail(NRK_EWORKSPACE, "din_head_ws_views: workspace %zu < %zu", ws_bytes, total);
  const char* w = static_cast<const char*>(ws);
  *stat0 = reinterpret_cast<const float*>(w + off[6]);
  const double* sb = reinterpret_cast<const double*>(w + off[15]);
  const int D2_ = 2 * d, F2_ = F / 2;
  *sum5 = sb + 2 * D2_ + 2 * F + 2 * F2_ + (3 * F2_ + 2) + (2 * F + F2_ * F + F2_);
  *da1 = reinterpret_cast<const float*>(w + off[13]);  // hf_bwd1's da1 (the dh0 region, unused by the fast head)
  return NRK_OK;
}

extern "C" int nrk_din_head_workspace(int32_t B, int32_t d, int32_t F, size_t* ws_bytes) {
  NRK_CHECK_ARG(ws_bytes && B > 1 && d > 0 && F >= 2, "din_head_workspace: bad arguments");
  size_t off[18];
  head_sizes(B, d, F, (int)cdiv(B, HR), off, ws_bytes);
  return NRK_OK;
}

extern "C" int nrk_din_head_train(const float* q, const float* pooled, int64_t ld_pooled, const float* labels,
                                  int32_t B, int32_t d, int32_t F, float momentum, float eps, float p_drop,
                                  uint64_t seed, const float* step, const nrk_din_head_params* prm, float* logits,
                                  float* loss, float* dpooled, void* ws, size_t ws_bytes, void* stream) {
  NRK_CHECK_ARG(B > 1 && B % HR == 0, "din_head_train: B=%d must be a positive multiple of %d", B, HR);
  NRK_CHECK_ARG(d > 0 && 2 * d <= 512 && F >= 2 && F <= 128 && F % 2 == 0 && ld_pooled >= d,
                "din_head_train: unsupported d=%d F=%d ld=%lld", d, F, (long long)ld_pooled);
  NRK_CHECK_ARG(p_drop >= 0.f && p_drop < 1.f, "din_head_train: dropout %f", (double)p_drop);
  NRK_CHECK_ARG(q && pooled && labels && step && prm && logits && loss && ws, "din_head_train: null pointer");
  // dpooled == NULL (fast path only): the attention backward forms it from the
  // workspace (nrk_din_attn_bwd_params_head), so the BN0-backward launch is skipped
  NRK_CHECK_ARG(dpooled || (F == 32 && d % 32 == 0), "din_head_train: dpooled may be NULL only with F = 32");
  const int nblk = B / HR;
  size_t off[18], total = 0;
  head_sizes(B, d, F, nblk, off, &total);
  if (ws_bytes < total) return fail(NRK_EWORKSPACE, "din_head_train: workspace %zu < %zu", ws_bytes, total);
  char* w = static_cast<char*>(ws);
  HeadArgs a;
  a.p = *prm;
  a.q = q;
  a.pooled = pooled;
  a.ld = ld_pooled;
  a.y = labels;
  a.B = B;
  a.d = d;
  a.D2 = 2 * d;
  a.F = F;
  a.F2 = F / 2;
  a.nblk = nblk;
  a.momentum = momentum;
  a.eps = eps;
  a.p_drop = p_drop;
  a.seed = seed;
  a.step = step;
  a.part0 = reinterpret_cast<double*>(w + off[0]);
  a.part1 = reinterpret_cast<double*>(w + off[1]);
  a.part2 = reinterpret_cast<double*>(w + off[2]);
  a.part3 = reinterpret_cast<double*>(w + off[3]);
  a.part4 = reinterpret_cast<double*>(w + off[4]);
  a.part5 = reinterpret_cast<double*>(w + off[5]);
  a.stat0 = reinterpret_cast<float*>(w + off[6]);
  a.stat1 = reinterpret_cast<float*>(w + off[7]);
  a.stat2 = reinterpret_cast<float*>(w + off[8]);
  a.a1 = reinterpret_cast<float*>(w + off[9]);
  a.a2 = reinterpret_cast<float*>(w + off[10]);
  a.dh2 = reinterpret_cast<float*>(w + off[11]);
  a.dh1 = reinterpret_cast<float*>(w + off[12]);
  a.dh0 = reinterpret_cast<float*>(w + off[13]);
  a.da1 = a.dh0;
  a.pw1 = reinterpret_cast<float*>(w + off[14]);
  a.mask1 = reinterpret_cast<uint32_t*>(w + off[16]);
  a.mask2 = reinterpret_cast<uint16_t*>(w + off[17]);
  {
    double* sb = reinterpret_cast<double*>(w + off[15]);
    const int D2_ = 2 * d, F2_ = F / 2;
    a.sum0 = sb;
    a.sum1 = a.sum0 + 2 * D2_;
    a.sum2 = a.sum1 + 2 * F;
    a.sum3 = a.sum2 + 2 * F2_;
    a.sum4 = a.sum3 + 3 * F2_ + 2;
    a.sum5 = a.sum4 + 2 * F + F2_ * F + F2_;
    a.sumw1 = a.sum5 + 2 * D2_ + F;
  }
  a.logits = logits;
  a.loss = loss;
  a.dpooled = dpooled;
  hipStream_t st = (hipStream_t)stream;
  const int D2 = 2 * d, F2 = F / 2;
  a.fast = F == HF && d % 32 == 0;
  // row groups of hf_stats0: 16 (measured -0.9 us vs 8, 32 no better)
  a.nrg0 = nblk >= 16 ? 16 : (nblk < 8 ? nblk : 8);
  if (a.fast) {
    const size_t lf1 =
        ((size_t)2 * D2 + (size_t)HR * (D2 + 4) + 4 * HR * HF + HR * (HF + 1)) * 4;
    const size_t lb1 = ((size_t)2 * D2 + (size_t)HR * (D2 + 4) + HR * (HF + 1) + 4 * HF + (size_t)D2 * 36) * 4;
    // + the kernels' static LDS (hf_fwd1: 10 KB of prologue sums): every launch must fit 160 KB
    NRK_CHECK_ARG(lf1 + 10240 <= 160 * 1024 && lb1 + 4096 <= 160 * 1024,
                  "din_head_train: d=%d needs %zu / %zu B of LDS", d, lf1 + 10240, lb1 + 4096);
    const int s3_ = 3 * F2 + 2, s4_ = 2 * F + F2 * F + F2;
    hipLaunchKernelGGL(hf_stats0, dim3((unsigned)(D2 / 32 * a.nrg0)), dim3(256), 0, st, a);
    switch (D2) {  // the fast path needs d % 32 == 0, 2d <= 512
      case 64: hipLaunchKernelGGL(hf_fwd1<2>, dim3(nblk), dim3(256), lf1, st, a); break;
      case 128: hipLaunchKernelGGL(hf_fwd1<4>, dim3(nblk), dim3(256), lf1, st, a); break;
      case 192: hipLaunchKernelGGL(hf_fwd1<6>, dim3(nblk), dim3(256), lf1, st, a); break;
      case 256: hipLaunchKernelGGL(hf_fwd1<8>, dim3(nblk), dim3(256), lf1, st, a); break;
      case 320: hipLaunchKernelGGL(hf_fwd1<10>, dim3(nblk), dim3(256), lf1, st, a); break;
      case 384: hipLaunchKernelGGL(hf_fwd1<12>, dim3(nblk), dim3(256), lf1, st, a); break;
      case 448: hipLaunchKernelGGL(hf_fwd1<14>, dim3(nblk), dim3(256), lf1, st, a); break;
      default: hipLaunchKernelGGL(hf_fwd1<16>, dim3(nblk), dim3(256), lf1, st, a); break;
    }
    hipLaunchKernelGGL(hf_fwd2, dim3(nblk), dim3(256), 0, st, a);
    hipLaunchKernelGGL(hf_fwd3, dim3(nblk), dim3(256), 0, st, a);
    hipLaunchKernelGGL(hf_bwd2, dim3(nblk), dim3(256), 0, st, a);
    // two column halves per 32-row block (one block per row block measured slower)
    const int cs = (D2 / 32) % 2 ? 1 : 2;
    const size_t lb1c = ((size_t)2 * (D2 / cs) + (size_t)HR * (D2 / cs + 4) + HR * (HF + 1) + 4 * HF +
                         (size_t)(D2 / cs) * 36) * 4;
#define NRK_HF_BWD1(NXV)                                                                                    \
  do {                                                                                                      \
    if (cs == 2) hipLaunchKernelGGL((hf_bwd1<NXV, ((NXV) % 2 ? 1 : 2)>), dim3(2 * nblk), dim3(256), lb1c, st, a); \
    else hipLaunchKernelGGL((hf_bwd1<NXV, 1>), dim3(nblk), dim3(256), lb1c, st, a);                        \
  } while (0)
    switch (D2) {
      case 64: NRK_HF_BWD1(2); break;
      case 128: NRK_HF_BWD1(4); break;
      case 192: NRK_HF_BWD1(6); break;
      case 256: NRK_HF_BWD1(8); break;
      case 320: NRK_HF_BWD1(10); break;
      case 384: NRK_HF_BWD1(12); break;
      case 448: NRK_HF_BWD1(14); break;
      default: NRK_HF_BWD1(16); break;
    }
#undef NRK_HF_BWD1
    hipLaunchKernelGGL(hf_reduce_c1, dim3((unsigned)(D2 + cdiv(s3_ + s4_, 64))), dim3(256), 0, st, a);
    if (dpooled) hipLaunchKernelGGL(hf_bwd0, dim3(nblk), dim3(256), 0, st, a);
    NRK_CHECK_LAUNCH("din_head_train (fast)");
    return NRK_OK;
  }
  const int fc = F < FC ? F : FC;  // W1 rows staged at a time (head_fwd1 / head_bwd1)
  const size_t lds1 = ((size_t)(HR + fc) * (D2 + 1) + 2 * D2 + HR * F) * 4;
  const size_t lds2 = ((size_t)HR * F + F2 * F + 2 * F + HR * F2) * 4;
  const size_t lds3 = ((size_t)2 * HR * F2 + 2 * F2 + 2 * HR) * 4;
  const size_t lds4 = ((size_t)3 * HR * F + HR * F2 + 2 * F + 4 * F2 + F2 * F) * 4;
  const size_t lds5 = ((size_t)(HR + fc) * (D2 + 1) + HR * F + 2 * D2 + 4 * F) * 4;
  {
    const size_t mx = std::max(std::max(lds1, lds2), std::max(std::max(lds3, lds4), lds5));
    // (+ head_fwd2 / fwd3 / bwd2's static prologue buffers, 3 KB)
    NRK_CHECK_ARG(mx + 3072 <= 160 * 1024, "din_head_train: d=%d F=%d needs %zu B of LDS", d, F, mx + 3072);
  }
  auto colsum = [&](const double* part, int stride, double* out) {
    hipLaunchKernelGGL(colsum_kernel<double>, dim3((unsigned)cdiv(stride, 32)), dim3(256), 0, st, part, nblk, stride,
                       stride, out);
  };
  const int s3 = 3 * F2 + 2, s4 = 2 * F + F2 * F + F2, s5 = 2 * D2 + F;
  hipLaunchKernelGGL(head_stats0, dim3(nblk), dim3(256), 0, st, a);
  colsum(a.part0, 2 * D2, a.sum0);
  NRK_CHECK_LAUNCH("head_stats0");
  hipLaunchKernelGGL(head_fwd1, dim3(nblk), dim3(256), lds1, st, a);
  colsum(a.part1, 2 * F, a.sum1);
  NRK_CHECK_LAUNCH("head_fwd1");
  hipLaunchKernelGGL(head_fwd2, dim3(nblk), dim3(256), lds2, st, a);
  colsum(a.part2, 2 * F2, a.sum2);
  NRK_CHECK_LAUNCH("head_fwd2");
  hipLaunchKernelGGL(head_fwd3, dim3(nblk), dim3(256), lds3, st, a);
  colsum(a.part3, s3, a.sum3);
  NRK_CHECK_LAUNCH("head_fwd3");
  hipLaunchKernelGGL(head_bwd2, dim3(nblk), dim3(256), lds4, st, a);
  colsum(a.part4, s4, a.sum4);
  NRK_CHECK_LAUNCH("head_bwd2");
  hipLaunchKernelGGL(head_bwd1, dim3(nblk), dim3(256), lds5, st, a);
  colsum(a.part5, s5, a.sum5);
  hipLaunchKernelGGL(colsum_kernel<float>, dim3((unsigned)cdiv(F * D2, 32)), dim3(256), 0, st, a.pw1, nblk, F * D2,
                     F * D2, a.sumw1);
  NRK_CHECK_LAUNCH("head_bwd1");
  hipLaunchKernelGGL(head_bwd0, dim3(nblk), dim3(256), 0, st, a);
  NRK_CHECK_LAUNCH("head_bwd0");
  const int ntot = F * D2 + F + D2 + F2 * F + F2 + F + F2 + 1 + F2;
  hipLaunchKernelGGL(head_grads, dim3((unsigned)cdiv(ntot, 256)), dim3(256), 0, st, a);
  NRK_CHECK_LAUNCH("head_grads");
  return NRK_OK;
}

// workspace: 256 fp64 partials (two-launch form) | the fused form's ticket;
// zero-initialise it once (the kernel leaves it zero)
extern "C" int nrk_clip_adam_workspace(int64_t n, size_t* ws_bytes) {
  NRK_CHECK_ARG(ws_bytes && n >= 0, "clip_adam_workspace: bad arguments");
  *ws_bytes = 256 * 8 + 256;
  return NRK_OK;
}

extern "C" int nrk_clip_adam(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, float* step,
                             float lr, const float* lr_dev, float beta1, float beta2, float eps, float weight_decay, float max_norm,
                             void* ws, size_t ws_bytes, void* stream) {
  NRK_CHECK_ARG(n > 0 && params && grads && exp_avg && exp_avg_sq && step && ws, "clip_adam: bad arguments");
  if (ws_bytes < 256 * 8 + 256) return fail(NRK_EWORKSPACE, "clip_adam: workspace %zu < 2304", ws_bytes);
  hipStream_t st = (hipStream_t)stream;
  if (n <= ((int64_t)1 << 17)) {  // small models (DIN: ~42K): one launch
    unsigned int* ticket = reinterpret_cast<unsigned int*>(static_cast<char*>(ws) + 256 * 8);
    hipLaunchKernelGGL(clip_adam_fused_kernel, dim3((unsigned)cdiv(n, (int64_t)1024)), dim3(1024), 0, st, params,
                       grads, exp_avg, exp_avg_sq, n, step, ticket, lr, lr_dev, beta1, beta2, eps, weight_decay,
                       max_norm);
    NRK_CHECK_LAUNCH("clip_adam_fused_kernel");
    return NRK_OK;
  }
  int nb = (int)cdiv(n, 256);
  if (nb > 256) nb = 256;
  int ns = (int)cdiv(n, 256 * 8);  // sumsq: 8 loads in flight per thread, few partials
  if (ns > 256) ns = 256;
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(sumsq_kernel, dim3(ns), dim3(256), 0, st, grads, n, part, step);
  NRK_CHECK_LAUNCH("sumsq_kernel");
  hipLaunchKernelGGL(clip_adam_kernel, dim3(nb), dim3(256), 0, st, params, grads, exp_avg, exp_avg_sq, n, part, ns,
                     step, lr, lr_dev, beta1, beta2, eps, weight_decay, max_norm);
  NRK_CHECK_LAUNCH("clip_adam_kernel");
  return NRK_OK;
}

extern "C" int nrk_clip_adam_partials(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                                      float* step, float lr, const float* lr_dev, float beta1, float beta2, float eps,
                                      float weight_decay, float max_norm, const double* norm_part, int32_t n_part,
                                      void* ws, size_t ws_bytes, void* stream) {
  NRK_CHECK_ARG(n > 0 && params && grads && exp_avg && exp_avg_sq && step && ws && norm_part && n_part > 0,
                "clip_adam_partials: bad arguments");
  if (ws_bytes < 256 * 8 + 256) return fail(NRK_EWORKSPACE, "clip_adam_partials: workspace %zu < 2304", ws_bytes);
  unsigned int* ticket = reinterpret_cast<unsigned int*>(static_cast<char*>(ws) + 256 * 8);
  hipLaunchKernelGGL(clip_adam_part_kernel, dim3((unsigned)cdiv(n, (int64_t)1024)), dim3(1024), 0, (hipStream_t)stream,
                     params, grads, exp_avg, exp_avg_sq, n, step, ticket, lr, lr_dev, beta1, beta2, eps, weight_decay,
                     max_norm, norm_part, n_part);
  NRK_CHECK_LAUNCH("clip_adam_part_kernel");
  return NRK_OK;
}
