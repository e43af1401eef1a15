// din_rerank.hip — DIN attention for re-ranking: many candidates per user
// sharing the user's history (DIN.py:166-173, evaluate(): the candidates of
// one user are scored with `his.expand(C, -1, -1)`).
//
// The attention logits of candidate c over history slot r are
//   s[c][r] = b2 + sum_n w2[n] relu(U[c][n] + P[r][n]),
//   U[c] = W1q q_c + b1 (caller, one GEMM over all candidates),
//   P[r] = W1k K[r]      (once per USER here, instead of once per candidate),
// so per candidate only the ReLU scoring, the softmax over all L slots and
// the pool sum_r alpha[c][r] K[r] remain.  b2 cancels in the softmax.
//
// Padding slots (ids < 0 or >= n_table inside the first L) hold zero keys
// (DIN.py:108 softmaxes over all L slots): their P row is 0, so every padding
// slot of a candidate has the same logit s_pad[c] = sum_n w2[n] relu(U[c][n]),
// and contributes 0 to the pool.  The kernel therefore compacts the nv valid
// rows to the front and scores nv rows plus ONE padding row that enters the
// softmax denominator npad = L - nv times.
//
// One workgroup (8 waves) per user; lane = candidate (64 per wave, 256 per
// chunk), so the softmax is a per-lane loop, not a cross-lane reduction:
//   1. valid mask by ballot, compacted history rows -> LDS image [64][D] bf16
//      (XOR-swizzled, zero rows past nv),
//   2. P = K W1k^T on bf16 MFMA (wave w: units 32w..32w+31) -> LDS, row-major,
//   3. each lane holds its candidate's U slice in registers; per history row
//      the P row is a broadcast LDS read and w2 sits in SGPRs (scalar loads of
//      the pass's 64 units): packed add, max, packed fma —
//      2 VALU per (candidate, row, unit); logits -> the lane's LDS row S[c][.];
//      two waves per 64-candidate group split the rows (8 waves, 2 per SIMD),
//   4. per-lane softmax over S[c][0..nr), alpha split hi + lo bf16, stored as
//      one dword per row in place,
//   5. pooled (64 cand x D) per wave = alpha K on bf16 MFMA (hi and lo passes,
//      f32 accumulate) over ceil(nv/16) row steps, K^T fragments by
//      ds_read_b64_tr_b16.
#include <math.h>

#include "nrk_common.h"

namespace nrk {
namespace rr {

constexpr int LP = 64;    // history rows held (L <= 64)
constexpr int SST = 68;   // S row stride (dwords): 16-B aligned rows, conflict-free b128 fragment reads
constexpr int NH = 2;     // waves per candidate group (they split rows and dim tiles)
constexpr int NT = 256 * NH;  // threads per workgroup
constexpr int CPB = 256;  // candidates per chunk (4 candidate groups x 64 lanes)

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
typedef __attribute__((ext_vector_type(2))) float f2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

template <int D, int A>
constexpr size_t smem_bytes() {
  return (size_t)LP * D * 2 + (size_t)LP * A * 4 + (size_t)CPB * SST * 4;
}

// History of user u: slot ids (lane = slot), the wave-uniform valid mask, and
// this thread's share of the compacted image rows (row (tid + NT k) / CPR,
// 16 B column chunk (tid + NT k) % CPR), loads issued, zeros past nv.
template <int D>
struct HistRows {
  static constexpr int CPR = D / 8, NE = LP * CPR / NT;
  uint64_t vm;
  uint4 v[NE];
  __device__ __forceinline__ void load(const uint16_t* __restrict__ table, int64_t n_table,
                                       const int32_t* __restrict__ hist, int u, int L, int tid) {
    const int lane = tid & 63;
    const int id = lane < L ? hist[(int64_t)u * L + lane] : -1;
    vm = __ballot(lane < L && id >= 0 && id < n_table);
    const int nv = __popcll(vm);
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      const int e = tid + NT * k, row = e / CPR, cc = e % CPR;
      const int src = __shfl(id, row < nv ? nth_set_bit(vm, row) : 0, 64);
      v[k] = make_uint4(0, 0, 0, 0);
      if (row < nv) v[k] = *reinterpret_cast<const uint4*>(table + (int64_t)src * D + cc * 8);
    }
  }
};

template <int D, int A>
__global__ __launch_bounds__(NT, 1) void din_rerank_kernel(const uint16_t* __restrict__ table, int64_t n_table,
                                                           const int32_t* __restrict__ hist, int nU, int L,
                                                           const float* __restrict__ Uc, int ldu, int C,
                                                           const uint16_t* __restrict__ W1k,
                                                           const float* __restrict__ w2,
                                                           float* __restrict__ pooled) {
  constexpr int CPR = D / 8, KS = D / 16, NDT = D / 32, NSL = A / 32;
  constexpr int UH = A % 64 == 0 ? 64 : 32;  // units per scoring pass (the U slice a lane holds)
  constexpr int NP = A / UH;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* img = smem;                                          // [LP][D] bf16
  float* Ps = reinterpret_cast<float*>(smem + LP * D * 2);            // [LP][A]
  float* S = Ps + LP * A;                                             // [CPB][SST]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  const int cw = w & 3, hw = w >> 2;  // candidate group (64 lanes) and its share (row pairs / dim tiles)
  float* Sl = S + (64 * cw + lane) * SST;  // this lane's candidate row; [64 + hw] partial max, [66 + hw] partial sum

  HistRows<D> cur, nxt;
  if (blockIdx.x < nU) cur.load(table, n_table, hist, blockIdx.x, L, tid);

  for (int u = blockIdx.x; u < nU; u += gridDim.x) {
    const int nv = __popcll(cur.vm), npad = L - nv, nr = nv + (npad > 0 ? 1 : 0);
    // 1. history image from the rows loaded during the previous user
#pragma unroll
    for (int k = 0; k < HistRows<D>::NE; ++k) {
      const int e = tid + NT * k, row = e / CPR, cc = e % CPR;
      *reinterpret_cast<uint4*>(img + row * 2 * D + 16 * (cc ^ swz<CPR>(row))) = cur.v[k];
    }
    __syncthreads();
    // 2. P = K W1k^T for the 32-row blocks holding rows 0..nr-1 (rows >= nv: 0);
    // wave w: unit slice w & 3, row block w >> 2
    const int nrb = (nr + 31) >> 5;
    if (cw < NSL && hw < nrb) {
      bf16x8 wf[KS];
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2)
        wf[s2] = *reinterpret_cast<const bf16x8*>(W1k + (int64_t)(32 * cw + r) * D + 16 * s2 + 8 * h);
      for (int c = hw; c < nrb; c += NH) {
      f32x16 acc;
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[g] = 0.f;
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(img + img_off<D>(32 * c + r, 16 * s2 + 8 * h));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, wf[s2], acc, 0, 0, 0);
      }
#pragma unroll
      for (int g = 0; g < 16; ++g) Ps[(32 * c + arow(g, h)) * A + 32 * cw + r] = acc[g];
      }
    }
    // the next user's history rows: loads in flight during steps 3-5
    const int un = u + gridDim.x;
    if (un < nU) nxt.load(table, n_table, hist, un, L, tid);
    __syncthreads();

    const int KR = (nv + 15) >> 4;  // 16-row pool steps
    for (int c0 = 0; c0 < C; c0 += CPB) {
      const int cand = c0 + 64 * cw + lane;
      const float* ub = Uc + ((int64_t)u * C + (cand < C ? cand : 0)) * ldu;
      // 3. logits of row pairs hw, hw + 2, ... in passes of UH units; the last
      // pass keeps the running maximum
      float m = -INFINITY;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int n0 = p * UH;
        f2 ua[UH / 2];
#pragma unroll
        for (int j = 0; j < UH / 4; ++j) {
          const float4 t = *reinterpret_cast<const float4*>(ub + n0 + 4 * j);
          ua[2 * j] = f2{t.x, t.y};
          ua[2 * j + 1] = f2{t.z, t.w};
        }
        for (int rr = 2 * hw; rr < nr; rr += 2 * NH) {  // row rr + 1 <= 63 lies in a computed P block
          const float* p0 = Ps + rr * A + n0;
          f2 a00 = {0.f, 0.f}, a01 = {0.f, 0.f}, a10 = {0.f, 0.f}, a11 = {0.f, 0.f};
#pragma unroll
          for (int j = 0; j < UH / 4; ++j) {
            const float4 q0 = *reinterpret_cast<const float4*>(p0 + 4 * j);
            const float4 q1 = *reinterpret_cast<const float4*>(p0 + A + 4 * j);
            const float4 wv = *reinterpret_cast<const float4*>(w2 + n0 + 4 * j);  // uniform: scalar loads
            const f2 wa = {wv.x, wv.y}, wb = {wv.z, wv.w};
            const f2 z = {0.f, 0.f};
            a00 = __builtin_elementwise_fma(wa, __builtin_elementwise_max(ua[2 * j] + f2{q0.x, q0.y}, z), a00);
            a01 = __builtin_elementwise_fma(wb, __builtin_elementwise_max(ua[2 * j + 1] + f2{q0.z, q0.w}, z), a01);
            a10 = __builtin_elementwise_fma(wa, __builtin_elementwise_max(ua[2 * j] + f2{q1.x, q1.y}, z), a10);
            a11 = __builtin_elementwise_fma(wb, __builtin_elementwise_max(ua[2 * j + 1] + f2{q1.z, q1.w}, z), a11);
            if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // bounds the LDS-read prefetch depth (registers)
          }
          float s0 = (a00.x + a00.y) + (a01.x + a01.y), s1 = (a10.x + a10.y) + (a11.x + a11.y);
          if (p > 0) {
            s0 += Sl[rr];
            s1 += Sl[rr + 1];
          }
          Sl[rr] = s0;
          Sl[rr + 1] = s1;  // row nr (odd nr): a dead slot < SST
          if (p == NP - 1) m = fmaxf(m, rr + 1 < nr ? fmaxf(s0, s1) : s0);
        }
      }
      if (NH > 1) {
        Sl[64 + hw] = m;
        __syncthreads();
        m = fmaxf(Sl[64], Sl[65]);
      }
      // 4. softmax over the L slots (rows < nv once each, row nv = padding npad
      // times): e = exp(s - m) split hi + lo bf16 in place (0 past nv); this
      // wave: rows 32 hw .. 32 hw + 31
      float sum = 0.f;
      const int jend = min(nr > 16 * KR ? nr : 16 * KR, (64 / NH) * (hw + 1));
      for (int j = (64 / NH) * hw; j < jend; ++j) {
        const float e = j < nr ? expf(Sl[j] - m) : 0.f;
        sum += j < nv ? e : (float)npad * e;
        const float al = j < nv ? e : 0.f;
        const bf16x2_t hl = {(__bf16)al, (__bf16)0.f};
        const uint32_t hb = __builtin_bit_cast(uint32_t, hl) & 0xFFFFu;
        const float rem = al - __uint_as_float(hb << 16);
        const bf16x2_t ll = {(__bf16)rem, (__bf16)0.f};
        reinterpret_cast<uint32_t*>(Sl)[j] = hb | (__builtin_bit_cast(uint32_t, ll) << 16);
      }
      Sl[66 + hw] = sum;
      if (NH > 1) __syncthreads();
      // 5. pooled = (e K) / sum for candidate group cw, dim tiles of half hw
      const int grp = lane >> 4, i16 = lane & 15;
      for (int ct = 0; ct < 2; ++ct) {
        const float* sc = S + (64 * cw + 32 * ct) * SST;
        const uint32_t* sa = reinterpret_cast<const uint32_t*>(sc + r * SST);
        bf16x8 ah[4], alw[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          if (ks < KR) {
            // k-slot (h, j) <-> row 16 ks + 4h + (j & 3) + 8 (j >> 2) (the tr-read order)
            const uint4 d0 = *reinterpret_cast<const uint4*>(sa + 16 * ks + 4 * h);
            const uint4 d1 = *reinterpret_cast<const uint4*>(sa + 16 * ks + 4 * h + 8);
            const uint32_t dv[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              ah[ks][j] = (short)(dv[j] & 0xFFFF);
              alw[ks][j] = (short)(dv[j] >> 16);
            }
          }
        }
        float inv[16];
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const float* sg = sc + arow(g, h) * SST;
          inv[g] = 1.f / (NH > 1 ? sg[66] + sg[67] : sg[66]);
        }
        for (int dt = hw * (NDT / NH); dt < (hw + 1) * (NDT / NH); ++dt) {
          f32x16 acc;
#pragma unroll
          for (int g = 0; g < 16; ++g) acc[g] = 0.f;
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            if (ks < KR) {
              const int rowq = 16 * ks + 4 * h + (i16 >> 2);
              const int col = 32 * dt + 16 * (grp & 1) + 4 * (i16 & 3);
              typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
              const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + img_off<D>(rowq, col)));
              const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + img_off<D>(rowq + 8, col)));
              const bf16x8 kb = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(alw[ks], kb, acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[ks], kb, acc, 0, 0, 0);
            }
          }
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            const int cg = c0 + 64 * cw + 32 * ct + arow(g, h);
            if (cg < C) pooled[((int64_t)u * C + cg) * D + 32 * dt + r] = acc[g] * inv[g];
          }
        }
      }
      __syncthreads();  // S is rewritten by the next chunk
    }
    cur = nxt;
  }
}

template <int D, int A>
int launch(const uint16_t* tb, int64_t n_table, const int32_t* hist, int nU, int L, const float* Uc, int ldu, int C,
           const uint16_t* wk, const float* w2, float* pooled, hipStream_t st) {
  constexpr size_t smem = smem_bytes<D, A>();
  static_assert(smem <= 160 * 1024, "din_rerank: LDS");
  const int grid = nU < 65536 ? nU : 65536;
  hipLaunchKernelGGL((din_rerank_kernel<D, A>), dim3(grid), dim3(rr::NT), smem, st, tb, n_table, hist, nU, L, Uc, ldu, C, wk,
                     w2, pooled);
  NRK_CHECK_LAUNCH("din_rerank_kernel");
  return NRK_OK;
}

template <int D>
int launch_a(int A, const uint16_t* tb, int64_t n_table, const int32_t* hist, int nU, int L, const float* Uc, int ldu, int C,
             const uint16_t* wk, const float* w2, float* pooled, hipStream_t st) {
  switch (A) {
    case 32: return launch<D, 32>(tb, n_table, hist, nU, L, Uc, ldu, C, wk, w2, pooled, st);
    case 64: return launch<D, 64>(tb, n_table, hist, nU, L, Uc, ldu, C, wk, w2, pooled, st);
    case 96: return launch<D, 96>(tb, n_table, hist, nU, L, Uc, ldu, C, wk, w2, pooled, st);
    default: return launch<D, 128>(tb, n_table, hist, nU, L, Uc, ldu, C, wk, w2, pooled, st);
  }
}

}  // namespace rr
}  // namespace nrk

using namespace nrk;

extern "C" int nrk_din_rerank_attn(const void* table, int64_t n_table, int32_t dtype, const int32_t* hist, int32_t nU,
                                   int32_t L, const float* Uc, int32_t ldu, int32_t C, int32_t d, const void* W1k_bf16,
                                   const float* w2, int32_t A, float* pooled, void* stream) {
  NRK_CHECK_ARG(dtype == NRK_DTYPE_BF16, "din_rerank: the table must be bf16");
  NRK_CHECK_ARG(d == 64 || d == 128 || d == 256, "din_rerank: emb_dim %d unsupported (64, 128, 256)", d);
  NRK_CHECK_ARG(A >= 32 && A <= 128 && A % 32 == 0, "din_rerank: attn_units %d unsupported (32..128 step 32)", A);
  NRK_CHECK_ARG(L >= 1 && L <= rr::LP, "din_rerank: history length %d unsupported (1..%d)", L, rr::LP);
  NRK_CHECK_ARG(nU >= 0 && C >= 0 && ldu >= A && ldu % 4 == 0, "din_rerank: bad sizes (ldu %d)", ldu);
  if (nU == 0 || C == 0) return NRK_OK;
  NRK_CHECK_ARG(table && hist && Uc && W1k_bf16 && w2 && pooled, "din_rerank: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const uint16_t* tb = static_cast<const uint16_t*>(table);
  const uint16_t* wk = static_cast<const uint16_t*>(W1k_bf16);
  if (d == 256) return rr::launch_a<256>(A, tb, n_table, hist, nU, L, Uc, ldu, C, wk, w2, pooled, st);
  if (d == 128) return rr::launch_a<128>(A, tb, n_table, hist, nU, L, Uc, ldu, C, wk, w2, pooled, st);
  return rr::launch_a<64>(A, tb, n_table, hist, nU, L, Uc, ldu, C, wk, w2, pooled, st);
}

// ------------------------------------------------------------------------
// Candidate projection (the query-side GEMMs of the re-rank, one kernel):
//   out[i][o] = sum_k table[ids[i]][k] W[o][k] + bias[o],  o < NO,
// for the attention layer's U = W1[:, :d] q + b1 (DIN.py:96-104) and the
// head's first-layer query half H1[:, :d] q (DIN.py:200-204, BN folded), with
// W = concat rows, gathered straight from the bf16 item table (no f32 copy of
// the candidate rows).  q is bf16-exact; W (f32) enters as bf16 hi + lo, so
// each product carries W to 16 mantissa bits; f32 accumulate.
// Workgroup: NO/32 waves (4..8), wave w owns output columns 32w..32w+31 and keeps
// their W^T fragments in registers; 32-row tiles of gathered rows are
// double-buffered in LDS (the next tile's loads in flight during this tile's
// MFMAs).  Rows with ids outside [0, n_table) are zero (out = bias).
namespace nrk {
namespace rr {

constexpr int PT = 32;  // rows per projection tile

template <int D>
__global__ __launch_bounds__(512, 1) void item_proj_kernel(const uint16_t* __restrict__ table, int64_t n_table,
                                                           const int32_t* __restrict__ ids, int64_t n,
                                                           const uint16_t* __restrict__ Whi,
                                                           const uint16_t* __restrict__ Wlo,
                                                           const float* __restrict__ bias, int NO,
                                                           float* __restrict__ out) {
  constexpr int CPR = D / 8, KS = D / 16, NCH = PT * CPR, MAXE = NCH / 256;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];  // 2 x [PT][D] bf16 (swizzled)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  const int col = 32 * w + r;
  bf16x8 bh[KS], bl[KS];
#pragma unroll
  for (int s2 = 0; s2 < KS; ++s2) {
    bh[s2] = *reinterpret_cast<const bf16x8*>(Whi + (int64_t)col * D + 16 * s2 + 8 * h);
    bl[s2] = *reinterpret_cast<const bf16x8*>(Wlo + (int64_t)col * D + 16 * s2 + 8 * h);
  }
  const float bv = bias[col];
  const int64_t ntile = (n + PT - 1) / PT;
  // waves 0-3 gather the tiles (16-B chunk e = tid + 256 k: row e / CPR, column chunk e % CPR)
  uint4 v[MAXE];
#define NRK_PROJ_FETCH(T)                                                                                   \
  if (tid < 256) {                                                                                          \
    _Pragma("unroll") for (int k = 0; k < MAXE; ++k) {                                                      \
      const int e = tid + 256 * k;                                                                          \
      const int64_t row = (T) * PT + e / CPR;                                                               \
      const int id = ids[row < n ? row : n - 1];                                                            \
      const bool ok = row < n && id >= 0 && id < n_table;                                                   \
      const uint4 x = *reinterpret_cast<const uint4*>(table + (int64_t)(ok ? id : 0) * D + (e % CPR) * 8); \
      v[k] = ok ? x : make_uint4(0, 0, 0, 0);                                                               \
    }                                                                                                       \
  }
#define NRK_PROJ_STAGE(BUF)                                                                                 \
  if (tid < 256) {                                                                                          \
    _Pragma("unroll") for (int k = 0; k < MAXE; ++k) {                                                      \
      const int e = tid + 256 * k, row = e / CPR, cc = e % CPR;                                             \
      *reinterpret_cast<uint4*>((BUF) + row * 2 * D + 16 * (cc ^ swz<CPR>(row))) = v[k];                    \
    }                                                                                                       \
  }
  int64_t t = blockIdx.x;
  if (t < ntile) {
    NRK_PROJ_FETCH(t)
    NRK_PROJ_STAGE(smem)
  }
  __syncthreads();
  for (int it = 0; t < ntile; t += gridDim.x, ++it) {
    unsigned char* cur = smem + (it & 1) * PT * D * 2;
    const int64_t tn = t + gridDim.x;
    if (tn < ntile) NRK_PROJ_FETCH(tn)
    f32x16 acc;
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[g] = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(cur + img_off<D>(r, 16 * s2 + 8 * h));
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bl[s2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bh[s2], acc, 0, 0, 0);
      if ((s2 & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // bounds the A-fragment prefetch (registers)
    }
    float* ob = out + t * PT * NO + col;
    const int nrow = (int)(n - t * PT < PT ? n - t * PT : PT);
    if (nrow == PT) {
#pragma unroll
      for (int g = 0; g < 16; ++g) ob[arow(g, h) * NO] = acc[g] + bv;
    } else {
#pragma unroll
      for (int g = 0; g < 16; ++g)
        if (arow(g, h) < nrow) ob[arow(g, h) * NO] = acc[g] + bv;
    }
    if (tn < ntile) NRK_PROJ_STAGE(smem + ((it + 1) & 1) * PT * D * 2)
    __syncthreads();
  }
#undef NRK_PROJ_FETCH
#undef NRK_PROJ_STAGE
}

// ------------------------------------------------------------------------
// Re-rank head (DIN.py:200-204 in eval mode, BatchNorms folded into the
// Linears by the caller):
//   h1 = relu(Q1[i] + pooled[i] H1p^T + c1)   (F = 32 units; Q1 = the
//        candidate's query half from item_proj_kernel),
//   h2 = relu(h1 H2^T + c2)                   (F/2 units),
//   logit[i] = h2 . h3 + c3, -inf where cand[i] < 0.
// One wave per 32 candidates: pooled rows are read straight into MFMA A
// fragments and split hi + lo bf16, H1p^T (hi, lo) is read from LDS;
// h1 -> LDS, then lane = candidate finishes the two small layers.
template <int D>
__global__ __launch_bounds__(256, 2) void rerank_head_kernel(const float* __restrict__ pooled, int64_t n,
                                                             const float* __restrict__ Q1, int ldq,
                                                             const int32_t* __restrict__ cand,
                                                             const uint16_t* __restrict__ Hhi,
                                                             const uint16_t* __restrict__ Hlo,
                                                             const float* __restrict__ c1,
                                                             const float* __restrict__ H2,
                                                             const float* __restrict__ c2,
                                                             const float* __restrict__ h3, float c3,
                                                             float* __restrict__ logit) {
  constexpr int KS = D / 16, F = 32, F2 = 16, HS = 33;
  constexpr int HR = D + 8;  // H1p row stride (bf16): rows 16 B apart in bank space, conflict-free fragment reads
  __shared__ float hs[4][32 * HS];
  __shared__ float w2s[F2 * F + F2];
  __shared__ __attribute__((aligned(16))) uint16_t hb_s[2][F * HR];  // H1p hi, lo
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  for (int i = tid; i < F2 * F; i += 256) w2s[i] = H2[i];
  if (tid < F2) w2s[F2 * F + tid] = c2[tid];
  for (int i = tid; i < F * D / 8; i += 256) {
    const int f = i / (D / 8), c8 = i % (D / 8);
    *reinterpret_cast<uint4*>(&hb_s[0][f * HR + 8 * c8]) = *reinterpret_cast<const uint4*>(Hhi + (int64_t)f * D + 8 * c8);
    *reinterpret_cast<uint4*>(&hb_s[1][f * HR + 8 * c8]) = *reinterpret_cast<const uint4*>(Hlo + (int64_t)f * D + 8 * c8);
  }
  const float cb = c1[r];
  float h3r[F2];
#pragma unroll
  for (int j = 0; j < F2; ++j) h3r[j] = h3[j];
  __syncthreads();
  float* hw = hs[w];
  const int64_t ntile = (n + 31) / 32;
  for (int64_t t = (int64_t)blockIdx.x * 4 + w; t < ntile; t += (int64_t)gridDim.x * 4) {
    const int64_t row = t * 32 + r;
    const float* pr = pooled + (row < n ? row : 0) * D + 8 * h;
    f32x16 acc;
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[g] = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) {
      const float4 x0 = *reinterpret_cast<const float4*>(pr + 16 * s2);
      const float4 x1 = *reinterpret_cast<const float4*>(pr + 16 * s2 + 4);
      const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      bf16x8 ah, al;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const __bf16 hb = (__bf16)xv[j];
        ah[j] = __builtin_bit_cast(short, hb);
        al[j] = __builtin_bit_cast(short, (__bf16)(xv[j] - (float)hb));
      }
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(&hb_s[0][r * HR + 16 * s2 + 8 * h]);
      const bf16x8 bl = *reinterpret_cast<const bf16x8*>(&hb_s[1][r * HR + 16 * s2 + 8 * h]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
    }
    // h1 (candidate arow(g, h), unit r) -> LDS
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int64_t rg = t * 32 + arow(g, h);
      const float q1 = rg < n ? Q1[rg * ldq + r] : 0.f;
      hw[arow(g, h) * HS + r] = fmaxf(acc[g] + q1 + cb, 0.f);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's h1 stores
    __builtin_amdgcn_wave_barrier();
    if (h == 0) {  // lane r = candidate t * 32 + r
      float hv[F];
#pragma unroll
      for (int f = 0; f < F; ++f) hv[f] = hw[r * HS + f];
      float lg = c3;
#pragma unroll
      for (int j = 0; j < F2; ++j) {
        float a2 = w2s[F2 * F + j];
#pragma unroll
        for (int f = 0; f < F; ++f) a2 = fmaf(w2s[j * F + f], hv[f], a2);
        lg = fmaf(h3r[j], fmaxf(a2, 0.f), lg);
      }
      if (row < n) logit[row] = cand[row] >= 0 ? lg : -INFINITY;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

template <int D>
int launch_proj(const uint16_t* tb, int64_t n_table, const int32_t* ids, int64_t n, const uint16_t* whi,
                const uint16_t* wlo, const float* bias, int NO, float* out, hipStream_t st) {
  const int64_t ntile = (n + PT - 1) / PT;
  const int grid = (int)(ntile < 512 ? ntile : 512);
  hipLaunchKernelGGL(item_proj_kernel<D>, dim3(grid), dim3(64 * (NO / 32)), (size_t)2 * PT * D * 2, st, tb, n_table,
                     ids, n, whi, wlo, bias, NO, out);
  NRK_CHECK_LAUNCH("item_proj_kernel");
  return NRK_OK;
}

template <int D>
int launch_head(const float* pooled, int64_t n, const float* Q1, int ldq, const int32_t* cand, const uint16_t* hhi,
                const uint16_t* hlo, const float* c1, const float* H2, const float* c2, const float* h3, float c3,
                float* logit, hipStream_t st) {
  const int64_t nw = (n + 31) / 32;
  const int grid = (int)((nw + 3) / 4 < 2048 ? (nw + 3) / 4 : 2048);
  hipLaunchKernelGGL(rerank_head_kernel<D>, dim3(grid), dim3(256), 0, st, pooled, n, Q1, ldq, cand, hhi, hlo, c1, H2,
                     c2, h3, c3, logit);
  NRK_CHECK_LAUNCH("rerank_head_kernel");
  return NRK_OK;
}

}  // namespace rr
}  // namespace nrk

extern "C" int nrk_din_item_proj(const void* table, int64_t n_table, int32_t dtype, const int32_t* ids, int64_t n,
                                 int32_t d, const void* W_hi, const void* W_lo, const float* bias, int32_t NO,
                                 float* out, void* stream) {
  NRK_CHECK_ARG(dtype == NRK_DTYPE_BF16, "din_item_proj: the table must be bf16");
  NRK_CHECK_ARG(d == 64 || d == 128 || d == 256, "din_item_proj: emb_dim %d unsupported (64, 128, 256)", d);
  NRK_CHECK_ARG(NO >= 128 && NO <= 256 && NO % 32 == 0, "din_item_proj: %d outputs unsupported (128..256 step 32)", NO);
  NRK_CHECK_ARG(n >= 0, "din_item_proj: bad sizes");
  if (n == 0) return NRK_OK;
  NRK_CHECK_ARG(table && ids && W_hi && W_lo && bias && out, "din_item_proj: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const uint16_t* tb = static_cast<const uint16_t*>(table);
  const uint16_t* hi = static_cast<const uint16_t*>(W_hi);
  const uint16_t* lo = static_cast<const uint16_t*>(W_lo);
  if (d == 256) return rr::launch_proj<256>(tb, n_table, ids, n, hi, lo, bias, NO, out, st);
  if (d == 128) return rr::launch_proj<128>(tb, n_table, ids, n, hi, lo, bias, NO, out, st);
  return rr::launch_proj<64>(tb, n_table, ids, n, hi, lo, bias, NO, out, st);
}

extern "C" int nrk_din_rerank_head(const float* pooled, int64_t n, int32_t d, const float* Q1, int32_t ldq,
                                   const int32_t* cand, const void* H1p_hi, const void* H1p_lo, const float* c1,
                                   int32_t F, const float* H2, const float* c2, const float* h3, float c3,
                                   float* logit, void* stream) {
  NRK_CHECK_ARG(d == 64 || d == 128 || d == 256, "din_rerank_head: emb_dim %d unsupported (64, 128, 256)", d);
  NRK_CHECK_ARG(F == 32, "din_rerank_head: fc_units %d unsupported (32)", F);
  NRK_CHECK_ARG(n >= 0 && ldq >= F, "din_rerank_head: bad sizes");
  if (n == 0) return NRK_OK;
  NRK_CHECK_ARG(pooled && Q1 && cand && H1p_hi && H1p_lo && c1 && H2 && c2 && h3 && logit,
                "din_rerank_head: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const uint16_t* hi = static_cast<const uint16_t*>(H1p_hi);
  const uint16_t* lo = static_cast<const uint16_t*>(H1p_lo);
  if (d == 256) return rr::launch_head<256>(pooled, n, Q1, ldq, cand, hi, lo, c1, H2, c2, h3, c3, logit, st);
  if (d == 128) return rr::launch_head<128>(pooled, n, Q1, ldq, cand, hi, lo, c1, H2, c2, h3, c3, logit, st);
  return rr::launch_head<64>(pooled, n, Q1, ldq, cand, hi, lo, c1, H2, c2, h3, c3, logit, st);
}
