// din_rerank.hip — DIN attention for re-ranking: many candidates per user
// sharing the user's history (DIN.py:166-173, evaluate(): the candidates of
// one user are scored with `his.expand(C, -1, -1)`).
//
// The attention logits of candidate c over history row r are
//   s[c][r] = b2 + sum_n w2[n] relu(U[c][n] + P[r][n]),
//   U[c] = W1q q_c + b1 (caller, one GEMM over all candidates),
//   P[r] = W1k K[r]      (once per USER here, instead of once per candidate),
// so per candidate only the ReLU scoring, the softmax over all L slots
// (padding included, DIN.py:108) and the pool sum_r alpha[c][r] K[r] remain.
// One workgroup (4 waves) per user at a time:
//   1. the user's history rows -> LDS image [64][D] bf16 (XOR-swizzled, zero rows
//      for padding), 2. P = K W1k^T on bf16 MFMA (wave w: units 32w..32w+31),
//   3. per chunk of 64 candidates: U rows -> LDS; lane = history row, each wave
//      scores its candidates against its lane's P row held in registers;
//      softmax across the lanes; alpha split hi + lo bf16 into LDS,
//   4. pooled (64 cand x D) = alpha K on bf16 MFMA (hi and lo passes, f32
//      accumulate), K^T fragments by ds_read_b64_tr_b16.
#include <math.h>

#include "nrk_common.h"

namespace nrk {
namespace rr {

constexpr int LP = 64;   // history rows held (L <= 64)
constexpr int CCH = 64;  // candidates per chunk

template <int CPR>
__device__ __forceinline__ int swz(int row) {
  if constexpr (CPR >= 16) return row & 15;
  else return (row / (16 / CPR)) & (CPR - 1);
}
template <int D>
__device__ __forceinline__ int img_off(int row, int col) {  // byte offset of element (row, col)
  constexpr int CPR = D / 8;
  return row * 2 * D + 16 * ((col >> 3) ^ swz<CPR>(row)) + 2 * (col & 7);
}
__device__ __forceinline__ int arow(int g, int h) { return (g & 3) + 8 * (g >> 2) + 4 * h; }
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

template <int D>
__global__ __launch_bounds__(256, 1) void din_rerank_kernel(const uint16_t* __restrict__ table, int64_t n_table,
                                                            const int32_t* __restrict__ hist, int nU, int L,
                                                            const float* __restrict__ Uc, int C,
                                                            const uint16_t* __restrict__ W1k,
                                                            const float* __restrict__ w2, int A,
                                                            float* __restrict__ pooled) {
  constexpr int CPR = D / 8, KS = D / 16, NDT = D / 32;
  constexpr int PS = 129;  // P row stride (floats): lane = row reads its own row conflict-free
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* img = smem;                                             // [LP][D] bf16
  float* Ps = reinterpret_cast<float*>(smem + LP * D * 2);               // [LP][PS]
  float* Us = Ps + LP * PS;                                              // [CCH][128]
  float* w2s = Us + CCH * 128;                                           // [128]
  uint16_t* ahi = reinterpret_cast<uint16_t*>(w2s + 128);                // [CCH][LP] bf16
  uint16_t* alo = ahi + CCH * LP;                                        // [CCH][LP] bf16
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  const int nsl = A >> 5;

  for (int i = tid; i < 128; i += 256) w2s[i] = i < A ? w2[i] : 0.f;
  bf16x8 wf[KS];
  {
    const int n = 32 * (w < nsl ? w : 0) + r;
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) wf[s2] = *reinterpret_cast<const bf16x8*>(W1k + (int64_t)n * D + 16 * s2 + 8 * h);
  }

  for (int u = blockIdx.x; u < nU; u += gridDim.x) {
    // 1. history image (rows >= L and invalid ids: zeros)
    {  // all of a thread's id loads, then all of its row loads, in flight together
      constexpr int NE = LP * CPR / 256;
      int32_t idv[NE];
#pragma unroll
      for (int k = 0; k < NE; ++k) {
        const int row = (tid + 256 * k) / CPR;
        idv[k] = row < L ? hist[(int64_t)u * L + row] : -1;
      }
      uint4 v[NE];
#pragma unroll
      for (int k = 0; k < NE; ++k) {
        const int cc = (tid + 256 * k) % CPR;
        v[k] = make_uint4(0, 0, 0, 0);
        if (idv[k] >= 0 && idv[k] < n_table) v[k] = *reinterpret_cast<const uint4*>(table + (int64_t)idv[k] * D + cc * 8);
      }
#pragma unroll
      for (int k = 0; k < NE; ++k) {
        const int e = tid + 256 * k, row = e / CPR, cc = e % CPR;
        *reinterpret_cast<uint4*>(img + row * 2 * D + 16 * (cc ^ swz<CPR>(row))) = v[k];
      }
    }
    __syncthreads();
    // 2. P = K W1k^T (columns of units >= A zero)
    for (int e = tid; e < LP * (128 - A); e += 256) Ps[(e / (128 - A)) * PS + A + e % (128 - A)] = 0.f;
    if (w < nsl) {
#pragma unroll
      for (int c = 0; c < LP / 32; ++c) {
        f32x16 acc;
#pragma unroll
        for (int g = 0; g < 16; ++g) acc[g] = 0.f;
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(img + img_off<D>(32 * c + r, 16 * s2 + 8 * h));
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, wf[s2], acc, 0, 0, 0);
        }
#pragma unroll
        for (int g = 0; g < 16; ++g) Ps[(32 * c + arow(g, h)) * PS + 32 * w + r] = acc[g];
      }
    }
    __syncthreads();
    // lane = history row: its P row in registers
    float pr[128];
#pragma unroll
    for (int n = 0; n < 128; ++n) pr[n] = Ps[lane * PS + n];  // units >= A: zeroed below
    const bool rowok = lane < L;

    for (int c0 = 0; c0 < C; c0 += CCH) {
      const int nc = min(CCH, C - c0);
      // 3a. U rows of this chunk
      const float* ub = Uc + ((int64_t)u * C + c0) * A;
      {  // units >= A: zeros (their w2 is 0 too); 8 loads in flight per thread
        float4 v[CCH * 32 / 256];
#pragma unroll
        for (int k = 0; k < CCH * 32 / 256; ++k) {
          const int e = tid + 256 * k, cl = e >> 5, q4 = e & 31;
          v[k] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (cl < nc && 4 * q4 < A) v[k] = *reinterpret_cast<const float4*>(ub + (int64_t)cl * A + 4 * q4);
        }
#pragma unroll
        for (int k = 0; k < CCH * 32 / 256; ++k) {
          const int e = tid + 256 * k, cl = e >> 5, q4 = e & 31;
          *reinterpret_cast<float4*>(Us + cl * 128 + 4 * q4) = v[k];
        }
      }
      __syncthreads();
      // 3b. scores, softmax, alpha: wave w takes candidates 16w .. 16w+15, four at a
      // time (four independent accumulation chains share each w2 / P read)
      for (int g4 = 0; g4 < 4; ++g4) {
        const int cb = 16 * w + 4 * g4;
        float sc[4] = {0.f, 0.f, 0.f, 0.f};
        if (cb < nc) {
          const float* u0 = Us + cb * 128;
#pragma unroll
          for (int n = 0; n < 128; n += 4) {  // units >= A contribute w2 = 0
            const float4 wv = *reinterpret_cast<const float4*>(w2s + n);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float4 uv = *reinterpret_cast<const float4*>(u0 + i * 128 + n);
              sc[i] = fmaf(wv.x, fmaxf(uv.x + pr[n], 0.f), sc[i]);
              sc[i] = fmaf(wv.y, fmaxf(uv.y + pr[n + 1], 0.f), sc[i]);
              sc[i] = fmaf(wv.z, fmaxf(uv.z + pr[n + 2], 0.f), sc[i]);
              sc[i] = fmaf(wv.w, fmaxf(uv.w + pr[n + 3], 0.f), sc[i]);
            }
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int cl = cb + i;
          float al = 0.f;
          if (cl < nc) {
            const float sv = rowok ? sc[i] : -INFINITY;
            const float m = wave_max(sv);
            const float ex = rowok ? expf(sv - m) : 0.f;
            al = ex / wave_sum(ex);
          }
          const bf16x2_t hl = {(__bf16)al, (__bf16)0.f};
          const uint16_t hb = (uint16_t)(__builtin_bit_cast(uint32_t, hl) & 0xFFFF);
          const float rem = al - __uint_as_float((uint32_t)hb << 16);
          const bf16x2_t ll = {(__bf16)rem, (__bf16)0.f};
          ahi[cl * LP + lane] = hb;
          alo[cl * LP + lane] = (uint16_t)(__builtin_bit_cast(uint32_t, ll) & 0xFFFF);
        }
      }
      __syncthreads();
      // 4. pooled = alpha K (hi and lo passes); wave w: dim tiles w, w + 4, ...
      for (int cg = 0; cg < nc; cg += 32) {
        for (int dt = w; dt < NDT; dt += 4) {
          f32x16 acc;
#pragma unroll
          for (int g = 0; g < 16; ++g) acc[g] = 0.f;
#pragma unroll
          for (int c = 0; c < LP / 32; ++c)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
              // k-slot (h, j) <-> row 32c + 16s + 4h + (j & 3) + 8 (j >> 2) (the tr-read order)
              const int rb = 32 * c + 16 * s + 4 * h;
              const int ci = cg + r;
              const uint2 h0 = *reinterpret_cast<const uint2*>(ahi + ci * LP + rb);
              const uint2 h1 = *reinterpret_cast<const uint2*>(ahi + ci * LP + rb + 8);
              const uint2 l0 = *reinterpret_cast<const uint2*>(alo + ci * LP + rb);
              const uint2 l1 = *reinterpret_cast<const uint2*>(alo + ci * LP + rb + 8);
              bf16x8 ah, alw;
              ah[0] = (short)(h0.x & 0xFFFF); ah[1] = (short)(h0.x >> 16); ah[2] = (short)(h0.y & 0xFFFF); ah[3] = (short)(h0.y >> 16);
              ah[4] = (short)(h1.x & 0xFFFF); ah[5] = (short)(h1.x >> 16); ah[6] = (short)(h1.y & 0xFFFF); ah[7] = (short)(h1.y >> 16);
              alw[0] = (short)(l0.x & 0xFFFF); alw[1] = (short)(l0.x >> 16); alw[2] = (short)(l0.y & 0xFFFF); alw[3] = (short)(l0.y >> 16);
              alw[4] = (short)(l1.x & 0xFFFF); alw[5] = (short)(l1.x >> 16); alw[6] = (short)(l1.y & 0xFFFF); alw[7] = (short)(l1.y >> 16);
              const int grp = lane >> 4, i16 = lane & 15;
              const int rowq = 32 * c + 16 * s + 4 * h + (i16 >> 2);
              const int col = 32 * dt + 16 * (grp & 1) + 4 * (i16 & 3);
              typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
              const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + img_off<D>(rowq, col)));
              const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + img_off<D>(rowq + 8, col)));
              const bf16x8 kb = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(alw, kb, acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, kb, acc, 0, 0, 0);
            }
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            const int cand = cg + arow(g, h);
            if (cand < nc) pooled[((int64_t)u * C + c0 + cand) * D + 32 * dt + r] = acc[g];
          }
        }
      }
      __syncthreads();  // Us / alpha are rewritten by the next chunk
    }
  }
}

}  // namespace rr
}  // namespace nrk

using namespace nrk;

extern "C" int nrk_din_rerank_attn(const void* table, int64_t n_table, int32_t dtype, const int32_t* hist, int32_t nU,
                                   int32_t L, const float* Uc, int32_t C, int32_t d, const void* W1k_bf16,
                                   const float* w2, int32_t A, float* pooled, void* stream) {
  NRK_CHECK_ARG(dtype == NRK_DTYPE_BF16, "din_rerank: the table must be bf16");
  NRK_CHECK_ARG(d == 64 || d == 128 || d == 256, "din_rerank: emb_dim %d unsupported (64, 128, 256)", d);
  NRK_CHECK_ARG(A >= 32 && A <= 128 && A % 32 == 0, "din_rerank: attn_units %d unsupported (32..128 step 32)", A);
  NRK_CHECK_ARG(L >= 1 && L <= rr::LP, "din_rerank: history length %d unsupported (1..%d)", L, rr::LP);
  NRK_CHECK_ARG(nU >= 0 && C >= 0, "din_rerank: bad sizes");
  if (nU == 0 || C == 0) return NRK_OK;
  NRK_CHECK_ARG(table && hist && Uc && W1k_bf16 && w2 && pooled, "din_rerank: null pointer");
  const size_t smem = (size_t)rr::LP * d * 2 + ((size_t)rr::LP * 129 + rr::CCH * 128 + 128) * 4 + 2 * (size_t)rr::CCH * rr::LP * 2;
  NRK_CHECK_ARG(smem <= 160 * 1024, "din_rerank: %zu B LDS", smem);
  const int grid = nU < 256 ? nU : 256;
  hipStream_t st = (hipStream_t)stream;
  const uint16_t* tb = static_cast<const uint16_t*>(table);
  const uint16_t* wk = static_cast<const uint16_t*>(W1k_bf16);
  if (d == 256)
    hipLaunchKernelGGL(rr::din_rerank_kernel<256>, dim3(grid), dim3(256), smem, st, tb, n_table, hist, nU, L, Uc, C, wk,
                       w2, A, pooled);
  else if (d == 128)
    hipLaunchKernelGGL(rr::din_rerank_kernel<128>, dim3(grid), dim3(256), smem, st, tb, n_table, hist, nU, L, Uc, C, wk,
                       w2, A, pooled);
  else
    hipLaunchKernelGGL(rr::din_rerank_kernel<64>, dim3(grid), dim3(256), smem, st, tb, n_table, hist, nU, L, Uc, C, wk,
                       w2, A, pooled);
  NRK_CHECK_LAUNCH("din_rerank_kernel");
  return NRK_OK;
}
