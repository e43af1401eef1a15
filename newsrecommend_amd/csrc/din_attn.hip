// din_attn.hip — DIN local-activation unit + weighted-sum pool for gfx950.
//
// Replaces AttentionLayer.forward (DIN.py:103-111) and its autograd backward,
// fused with the history gather of TrainDataset.__getitem__ (DIN.py:84-86).
// Math (per sample b, history rows r = 0..L-1, A attention units):
//   z[r][n] = U[b][n] + sum_k W1k[n][k] K[r][k]        (U = q W1q^T + b1, caller)
//   s[r]    = b2 + sum_n w2[n] relu(z[r][n])
//   alpha   = softmax_r(s)  over ALL L rows, zero padding rows included (DIN.py:108)
//   pooled  = sum_r alpha[r] K[r][:]
// Backward (embeddings are frozen inputs in the reference, so only parameter
// gradients): dalpha_r = dpooled . K[r]; ds_r = alpha_r (dalpha_r - sum alpha dalpha);
//   dz = ds_r w2[n] [z > 0];  dW1k = sum dz^T K;  dw2 = sum ds relu(z);
//   db2 = sum ds;  dU[b] = sum_r dz[r][:]  (caller: dW1q = dU^T q, db1 = sum dU).
//
// Layout: one 256-thread workgroup (4 waves) per sample at a time, looping
// over samples (persistent grid).  The sample's key rows are gathered from HBM
// into an LDS image (bf16: XOR-swizzled 16-B chunks; f32: rows padded by one
// word).  Wave w owns attention units [32w, 32w+32): the z GEMM runs on MFMA
// (bf16: v_mfma_f32_32x32x16_bf16, f32: v_mfma_f32_32x32x2_f32) with the
// W1k slice as A (rows = units) and the key rows as B (cols = history rows),
// so the w2-weighted ReLU reduction over units is lane-local.  In the
// backward the same GEMM is recomputed in the transposed orientation so the
// dz accumulator feeds the dW1k MFMA directly as its A operand; the key rows
// come back as the B operand through ds_read_b64_tr_b16 (bf16) transposed reads.
#include <math.h>

#include "nrk_common.h"

namespace nrk {

template <int CPR>
__device__ __forceinline__ int kswz(int row) {
  if constexpr (CPR >= 16) return row & 15;
  else return (row / (16 / CPR)) & (CPR - 1);
}

// ----------------------------------------------------------- LDS images --
template <bool BF16, int D>
struct KImg;

template <int D>
struct KImg<true, D> {  // bf16 rows of D elements, 16-B chunks XOR-swizzled
  static constexpr int CPR = D / 8;
  static constexpr int ROW_BYTES = 2 * D;
  __device__ static size_t bytes(int Lp) { return (size_t)Lp * ROW_BYTES; }
  // byte offset of element (row, col)
  __device__ static int off(int row, int col) {
    return row * ROW_BYTES + 16 * ((col >> 3) ^ kswz<CPR>(row)) + 2 * (col & 7);
  }
  // stage rows [0, Lp): rows < L from the source, others zero
  __device__ static void stage(unsigned char* img, const void* src_v, const int32_t* ids, int64_t n_table,
                               int64_t b, int L, int Lp) {
    const uint16_t* src = static_cast<const uint16_t*>(src_v);
    for (int f = threadIdx.x; f < Lp * CPR; f += blockDim.x) {
      const int row = f / CPR, cc = f % CPR;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (row < L) {
        const uint16_t* p = nullptr;
        if (ids) {
          const int32_t id = ids[b * L + row];
          if (id >= 0 && id < n_table) p = src + (int64_t)id * D;
        } else {
          p = src + (b * L + row) * (int64_t)D;
        }
        if (p) v = *reinterpret_cast<const uint4*>(p + cc * 8);
      }
      *reinterpret_cast<uint4*>(img + row * ROW_BYTES + 16 * (cc ^ kswz<CPR>(row))) = v;
    }
  }
  __device__ static float2 pair(const unsigned char* img, int row, int col) {  // col even
    const uint32_t u = *reinterpret_cast<const uint32_t*>(img + off(row, col));
    return make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xFFFF0000u));
  }
};

template <int D>
struct KImg<false, D> {  // f32 rows padded to D+1 words (conflict-free column reads)
  static constexpr int STRIDE = D + 1;
  __device__ static size_t bytes(int Lp) { return (size_t)Lp * STRIDE * 4; }
  __device__ static int off(int row, int col) { return 4 * (row * STRIDE + col); }
  __device__ static void stage(unsigned char* img, const void* src_v, const int32_t* ids, int64_t n_table,
                               int64_t b, int L, int Lp) {
    const float* src = static_cast<const float*>(src_v);
    float* out = reinterpret_cast<float*>(img);
    constexpr int C4 = D / 4;
    for (int f = threadIdx.x; f < Lp * C4; f += blockDim.x) {
      const int row = f / C4, cc = f % C4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < L) {
        const float* p = nullptr;
        if (ids) {
          const int32_t id = ids[b * L + row];
          if (id >= 0 && id < n_table) p = src + (int64_t)id * D;
        } else {
          p = src + (b * L + row) * (int64_t)D;
        }
        if (p) v = *reinterpret_cast<const float4*>(p + cc * 4);
      }
      float* o = out + row * STRIDE + cc * 4;
      o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    }
  }
  __device__ static float2 pair(const unsigned char* img, int row, int col) {
    const float* p = reinterpret_cast<const float*>(img + off(row, col));
    return make_float2(p[0], p[1]);
  }
};

// ------------------------------------------------------ MFMA fragments --
// W1k fragment of wave-slice rows n = 32*ws + (lane&31), all k.
template <bool BF16, int D>
struct WFrag;

template <int D>
struct WFrag<true, D> {
  static constexpr int KS = D / 16;
  bf16x8 f[KS];
  __device__ void load(const void* W, int n_row, int h) {
    const uint16_t* p = static_cast<const uint16_t*>(W) + (int64_t)n_row * D + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) f[s] = *reinterpret_cast<const bf16x8*>(p + 16 * s);
  }
};

template <int D>
struct WFrag<false, D> {  // f32: fragments are re-read from L1/L2 inside the k loop
  const float* p;
  __device__ void load(const void* W, int n_row, int h) {
    p = static_cast<const float*>(W) + (int64_t)n_row * D + h;
  }
};

// acc += W-slice (rows n) x K-tile^T (cols r)       [forward orientation]
// acc += K-tile (rows r) x W-slice^T (cols n)       [backward orientation]
template <bool BF16, int D, bool KROWS_AS_A>
__device__ __forceinline__ void zgemm(f32x16& acc, const WFrag<BF16, D>& wf, const unsigned char* img, int row0,
                                      int lane) {
  const int r = lane & 31, h = lane >> 5;
  if constexpr (BF16) {
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(img + KImg<true, D>::off(row0 + r, 16 * s + 8 * h));
      if constexpr (KROWS_AS_A)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, wf.f[s], acc, 0, 0, 0);
      else
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf.f[s], kf, acc, 0, 0, 0);
    }
  } else {
    const float* krow = reinterpret_cast<const float*>(img + KImg<false, D>::off(row0 + r, h));
#pragma unroll 8
    for (int s = 0; s < D / 2; ++s) {
      const float kv = krow[2 * s];
      const float wv = wf.p[2 * s];
      if constexpr (KROWS_AS_A)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(kv, wv, acc, 0, 0, 0);
      else
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv, kv, acc, 0, 0, 0);
    }
  }
}

__device__ __forceinline__ int acc_row(int g, int h) { return (g & 3) + 8 * (g >> 2) + 4 * h; }

// ================================================================ forward ==
template <bool BF16, int D>
__global__ __launch_bounds__(256) void din_fwd_kernel(const void* __restrict__ keys, const int32_t* __restrict__ ids,
                                                      int64_t n_table, const float* __restrict__ U,
                                                      const void* __restrict__ W1k, const float* __restrict__ w2,
                                                      float b2, int B, int L, int A, float* __restrict__ pooled,
                                                      float* __restrict__ alpha) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  using Img = KImg<BF16, D>;
  const int Lp = (L + 31) & ~31, nct = Lp >> 5, nsl = A >> 5;
  unsigned char* img = smem;
  float* spart = reinterpret_cast<float*>(smem + align_up(Img::bytes(Lp), 16));  // [4][Lp]
  float* salpha = spart + 4 * Lp;                                                // [Lp]
  constexpr int NPAIR = D / 2, G = 256 / NPAIR;
  float* spool = salpha + Lp;  // [G][D]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;

  WFrag<BF16, D> wf;
  float w2v[16];
  if (w < nsl) {
    wf.load(W1k, 32 * w + r, h);
#pragma unroll
    for (int g = 0; g < 16; ++g) w2v[g] = w2[32 * w + acc_row(g, h)];
  }

  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    Img::stage(img, keys, ids, n_table, b, L, Lp);
    __syncthreads();
    if (w < nsl) {
      float u[16];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 v = *reinterpret_cast<const float4*>(U + b * A + 32 * w + 8 * j + 4 * h);
        u[4 * j] = v.x; u[4 * j + 1] = v.y; u[4 * j + 2] = v.z; u[4 * j + 3] = v.w;
      }
      for (int ct = 0; ct < nct; ++ct) {
        f32x16 acc;
#pragma unroll
        for (int g = 0; g < 16; ++g) acc[g] = u[g];
        zgemm<BF16, D, false>(acc, wf, img, 32 * ct, lane);
        float part = 0.f;
#pragma unroll
        for (int g = 0; g < 16; ++g) part = fmaf(w2v[g], fmaxf(acc[g], 0.f), part);
        part += __shfl_xor(part, 32, 64);
        if (h == 0) spart[w * Lp + 32 * ct + r] = part;
      }
    }
    __syncthreads();
    if (w == 0) {  // softmax over the L rows (padding rows of the history included)
      float sv[2];
      float m = -INFINITY;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = lane + 64 * i;
        float s = -INFINITY;
        if (row < L) {
          s = b2;
          for (int ww = 0; ww < nsl; ++ww) s += spart[ww * Lp + row];
        }
        sv[i] = s;
        m = fmaxf(m, s);
      }
      m = wave_max(m);
      float e0 = lane < L ? expf(sv[0] - m) : 0.f;
      float e1 = lane + 64 < L ? expf(sv[1] - m) : 0.f;
      const float sum = wave_sum(e0 + e1);
      if (lane < Lp) salpha[lane] = e0 / sum;
      if (lane + 64 < Lp) salpha[lane + 64] = e1 / sum;
      if (lane < L) alpha[b * L + lane] = e0 / sum;
      if (lane + 64 < L) alpha[b * L + lane + 64] = e1 / sum;
    }
    __syncthreads();
    {
      const int p = tid % NPAIR, rg = tid / NPAIR;
      float a0 = 0.f, a1 = 0.f;
      for (int row = rg; row < L; row += G) {
        const float al = salpha[row];
        const float2 kv = Img::pair(img, row, 2 * p);
        a0 = fmaf(al, kv.x, a0);
        a1 = fmaf(al, kv.y, a1);
      }
      spool[rg * D + 2 * p] = a0;
      spool[rg * D + 2 * p + 1] = a1;
    }
    __syncthreads();
    for (int c = tid; c < D; c += 256) {
      float s = 0.f;
      for (int g = 0; g < G; ++g) s += spool[g * D + c];
      pooled[b * D + c] = s;
    }
    // the next sample's staging overwrites img/spool only after this barrier
    __syncthreads();
  }
}

// ---------------------------------------------- forward, wave per sample --
// bf16 fast path (D <= 128): one WAVE owns one sample at a time, so there are
// no workgroup barriers.  W1k for all A units lives in registers (A/32 x D/16
// fragments); the sample's Lp key rows are gathered by id straight into the
// wave's LDS slice with global_load_lds (padding / invalid ids read a zero
// row); z = U + W1k K^T on MFMA per (32-row, 32-unit) tile; softmax and the
// alpha-weighted pool stay inside the wave.
__device__ __attribute__((aligned(16))) uint16_t g_zero_row[256];  // zero-initialised code-object global

template <int D, int NA, int NBUF>
__global__ __launch_bounds__(256, 2) void din_fwd_wave_kernel(const uint16_t* __restrict__ table,
                                                               const int32_t* __restrict__ ids, int64_t n_table,
                                                               const float* __restrict__ U,
                                                               const uint16_t* __restrict__ W1k,
                                                               const float* __restrict__ w2, int B, int L,
                                                               float* __restrict__ pooled,
                                                               float* __restrict__ alpha) {
  constexpr int CPR = D / 8, KS = D / 16, A = 32 * NA;
  constexpr int DPL = D / 64;         // pooled dims per lane
  constexpr int AP = (A + 63) & ~63;  // U slot padded to whole 64-lane DMA pieces
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int Lp = (L + 31) & ~31, nct = Lp >> 5;
  // LDS: w2 [AP] (shared) | per wave, NBUF slots of {U row [AP] f32, key image [Lp][D] bf16}
  const int slot_f = AP + Lp * D / 2;  // floats per slot
  float* w2s = reinterpret_cast<float*>(smem);
  float* wbase = w2s + AP + (size_t)wv * NBUF * slot_f;
  typedef __attribute__((address_space(3))) void* lds_ptr;
  for (int i = threadIdx.x; i < A; i += 256) w2s[i] = w2[i];
  __syncthreads();

  bf16x8 wf[NA][KS];
#pragma unroll
  for (int t = 0; t < NA; ++t)
#pragma unroll
    for (int s = 0; s < KS; ++s)
      wf[t][s] = *reinterpret_cast<const bf16x8*>(W1k + (int64_t)(32 * t + r) * D + 16 * s + 8 * h);

  const int nw = gridDim.x * 4;
  auto load_ids = [&](int b, int32_t& i0, int32_t& i1) {
    i0 = (b < B && lane < L) ? ids[(int64_t)b * L + lane] : -1;
    i1 = (b < B && lane + 64 < L) ? ids[(int64_t)b * L + lane + 64] : -1;
  };
  // gather sample b's key rows + U row into slot `sl` (asynchronous LDS-DMA)
  auto issue = [&](int b, int sl, int32_t i0, int32_t i1) {
    float* us = wbase + sl * slot_f;
    uint16_t* img = reinterpret_cast<uint16_t*>(us + AP);
    const int npieces = Lp * CPR / 64;
    for (int u = 0; u < npieces; ++u) {
      const int p = u * 64 + lane;
      const int row = p / CPR, pc = p % CPR;
      const int cc = pc ^ kswz<CPR>(row);
      const int ida = __shfl(i0, row & 63, 64), idb = __shfl(i1, row & 63, 64);  // both: source lanes differ
      const int idr = row < 64 ? ida : idb;
      const uint16_t* src = (row < L && idr >= 0 && idr < n_table) ? table + (int64_t)idr * D + cc * 8 : g_zero_row;
      __builtin_amdgcn_global_load_lds(src, (lds_ptr)(img + u * 64 * 8), 16, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < AP / 64; ++u) {
      const int i = u * 64 + lane;
      __builtin_amdgcn_global_load_lds(U + (int64_t)b * A + (i < A ? i : 0), (lds_ptr)(us + u * 64), 4, 0, 0);
    }
  };

  int b = blockIdx.x * 4 + wv;
  int32_t c0, c1, n0 = -1, n1 = -1;
  load_ids(b, c0, c1);
  if (b < B) issue(b, 0, c0, c1);
  if (NBUF == 2) load_ids(b + nw, n0, n1);
  int sl = 0;
  for (; b < B; b += nw) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this sample's rows (and the next ids) landed
    const int bn = b + nw;
    if constexpr (NBUF == 2) {
      if (bn < B) issue(bn, sl ^ 1, n0, n1);
      load_ids(bn + nw, n0, n1);
    }
    const float* us = wbase + sl * slot_f;
    const uint16_t* img = reinterpret_cast<const uint16_t*>(us + AP);

    // ---- scores: s[row] = sum_n w2[n] relu(U[n] + W1k[n] . K[row])
    float sc[4];  // row 32c + r (halves combined), c < nct
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      sc[c] = -INFINITY;
      if (c < nct) {
        bf16x8 kf[KS];
        const int row = 32 * c + r;
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2)
          kf[s2] = *reinterpret_cast<const bf16x8*>(img + row * D + 8 * ((2 * s2 + h) ^ kswz<CPR>(row)));
        float part = 0.f;
#pragma unroll
        for (int t = 0; t < NA; ++t) {
          f32x16 acc;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float4 uv = *reinterpret_cast<const float4*>(us + 32 * t + 8 * j + 4 * h);
            acc[4 * j] = uv.x; acc[4 * j + 1] = uv.y; acc[4 * j + 2] = uv.z; acc[4 * j + 3] = uv.w;
          }
#pragma unroll
          for (int s2 = 0; s2 < KS; ++s2)
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[t][s2], kf[s2], acc, 0, 0, 0);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float4 wv4 = *reinterpret_cast<const float4*>(w2s + 32 * t + 8 * j + 4 * h);
            part = fmaf(wv4.x, fmaxf(acc[4 * j], 0.f), part);
            part = fmaf(wv4.y, fmaxf(acc[4 * j + 1], 0.f), part);
            part = fmaf(wv4.z, fmaxf(acc[4 * j + 2], 0.f), part);
            part = fmaf(wv4.w, fmaxf(acc[4 * j + 3], 0.f), part);
          }
        }
        part += __shfl_xor(part, 32, 64);
        sc[c] = (row < L) ? part : -INFINITY;
      }
    }
    // ---- softmax over the L rows (padding rows of the history included)
    float m = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
    m = wave_max(m);
    float e[4], sum = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      e[c] = c < nct && 32 * c + r < L ? expf(sc[c] - m) : 0.f;
      sum += h == 0 ? e[c] : 0.f;
    }
    sum = wave_sum(sum);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      e[c] = e[c] / sum;
      if (h == 0 && c < nct && 32 * c + r < L) alpha[(int64_t)b * L + 32 * c + r] = e[c];
    }
    // ---- pooled = sum_rows alpha[row] K[row][:]
    float acc2[DPL];
#pragma unroll
    for (int j = 0; j < DPL; ++j) acc2[j] = 0.f;
    for (int row = 0; row < L; ++row) {
      const float ar = __builtin_amdgcn_readlane(__float_as_int(row < 32 ? e[0] : row < 64 ? e[1] : row < 96 ? e[2] : e[3]),
                                                 row & 31);
      const float al = __int_as_float(ar);
      if constexpr (DPL == 2) {
        const uint32_t u = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const unsigned char*>(img) +
                                                              KImg<true, D>::off(row, 2 * lane));
        acc2[0] = fmaf(al, __uint_as_float(u << 16), acc2[0]);
        acc2[1] = fmaf(al, __uint_as_float(u & 0xFFFF0000u), acc2[1]);
      } else {
        const uint16_t u = *reinterpret_cast<const uint16_t*>(reinterpret_cast<const unsigned char*>(img) +
                                                              KImg<true, D>::off(row, lane));
        acc2[0] = fmaf(al, bf16_to_f32(u), acc2[0]);
      }
    }
    if constexpr (DPL == 2) {
      *reinterpret_cast<float2*>(pooled + (int64_t)b * D + 2 * lane) = make_float2(acc2[0], acc2[1]);
    } else {
      pooled[(int64_t)b * D + lane] = acc2[0];
    }
    // slot reuse: every LDS read of this sample is done before the DMA after next
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (NBUF == 2) {
      sl ^= 1;
    } else {
      load_ids(bn, c0, c1);
      if (bn < B) issue(bn, 0, c0, c1);
    }
  }
}

// =============================================================== backward ==
// Workgroup slab layout (floats): dW1k [A][D], then dw2 [A], then db2 [1].
__host__ __device__ __forceinline__ size_t slab_floats(int A, int D) { return (size_t)A * D + A + 4; }

template <bool BF16, int D>
__global__ __launch_bounds__(256) void din_bwd_kernel(
    const void* __restrict__ keys, const int32_t* __restrict__ ids, int64_t n_table, const float* __restrict__ U,
    const void* __restrict__ W1k, const float* __restrict__ w2, int B, int L, int A,
    const float* __restrict__ dpooled, const float* __restrict__ alpha, float* __restrict__ dU,
    float* __restrict__ slabs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  using Img = KImg<BF16, D>;
  constexpr int NCT = D / 32;  // output column tiles of dW1k
  const int Lp = (L + 31) & ~31, nct = Lp >> 5, nsl = A >> 5;
  unsigned char* img = smem;
  float* sdp = reinterpret_cast<float*>(smem + align_up(Img::bytes(Lp), 16));  // [D]
  float* sal = sdp + D;                                                         // [Lp]
  float* sda = sal + Lp;                                                        // [Lp] dalpha
  float* sds = sda + Lp;                                                        // [Lp] ds
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;

  WFrag<BF16, D> wf;
  float w2n = 0.f;
  if (w < nsl) {
    wf.load(W1k, 32 * w + r, h);
    w2n = w2[32 * w + r];
  }
  f32x16 dw[NCT];
#pragma unroll
  for (int c = 0; c < NCT; ++c)
#pragma unroll
    for (int g = 0; g < 16; ++g) dw[c][g] = 0.f;
  float dw2_acc = 0.f, db2_acc = 0.f;

  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    Img::stage(img, keys, ids, n_table, b, L, Lp);
    for (int c = tid; c < D; c += 256) sdp[c] = dpooled[b * D + c];
    for (int i = tid; i < Lp; i += 256) sal[i] = i < L ? alpha[b * L + i] : 0.f;
    __syncthreads();
    // dalpha_r = dpooled . K[r]   (4 threads per row)
    for (int base = 0; base < Lp; base += 64) {
      const int row = base + (tid >> 2), q = tid & 3;
      float acc = 0.f;
      if (row < Lp) {
        for (int c = q * (D / 4); c < (q + 1) * (D / 4); c += 2) {
          const float2 kv = Img::pair(img, row, c);
          acc = fmaf(sdp[c], kv.x, acc);
          acc = fmaf(sdp[c + 1], kv.y, acc);
        }
      }
      acc += __shfl_xor(acc, 1, 64);
      acc += __shfl_xor(acc, 2, 64);
      if (row < Lp && q == 0) sda[row] = acc;
    }
    __syncthreads();
    if (w == 0) {
      float t = 0.f;
      for (int i = lane; i < L; i += 64) t += sal[i] * sda[i];
      const float cdot = wave_sum(t);
      for (int i = lane; i < Lp; i += 64) {
        const float ds = i < L ? sal[i] * (sda[i] - cdot) : 0.f;
        sds[i] = ds;
        db2_acc += ds;
      }
    }
    __syncthreads();
    if (w < nsl) {
      const float un = U[b * A + 32 * w + r];
      float du = 0.f;
      for (int ct = 0; ct < nct; ++ct) {
        f32x16 acc;
#pragma unroll
        for (int g = 0; g < 16; ++g) acc[g] = un;
        zgemm<BF16, D, true>(acc, wf, img, 32 * ct, lane);  // acc[g] = z[row(g)][n]
        f32x16 dz;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const float ds = sds[32 * ct + acc_row(g, h)];
          const float z = acc[g];
          dw2_acc = fmaf(ds, fmaxf(z, 0.f), dw2_acc);
          const float v = z > 0.f ? ds * w2n : 0.f;
          dz[g] = v;
          du += v;
        }
        // dW1k[n][c] += sum_rows dz[row][n] K[row][c]
        if constexpr (BF16) {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            bf16x8 af;
#pragma unroll
            for (int j = 0; j < 8; ++j) af[j] = (short)f32_to_bf16_rne(dz[8 * s + j]);
            // B operand: lane (c, h) element j = K[16s + 8(j>>2) + 4h + (j&3)][c]
            const int grp = lane >> 4, i16 = lane & 15;
            const int rowq = 32 * ct + 16 * s + 4 * h + (i16 >> 2);
#pragma unroll
            for (int c = 0; c < NCT; ++c) {
              const int col = 32 * c + 16 * (grp & 1) + 4 * (i16 & 3);
              typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
              const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                  (lds_bf16x4*)(img + KImg<true, D>::off(rowq, col)));
              const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                  (lds_bf16x4*)(img + KImg<true, D>::off(rowq + 8, col)));
              bf16x8 bf;
              bf[0] = lo[0]; bf[1] = lo[1]; bf[2] = lo[2]; bf[3] = lo[3];
              bf[4] = hi[0]; bf[5] = hi[1]; bf[6] = hi[2]; bf[7] = hi[3];
              dw[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, dw[c], 0, 0, 0);
            }
          }
        } else {
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            const int row = 32 * ct + acc_row(s, h);
            const float* krow = reinterpret_cast<const float*>(img + KImg<false, D>::off(row, 0));
#pragma unroll
            for (int c = 0; c < NCT; ++c)
              dw[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(dz[s], krow[32 * c + r], dw[c], 0, 0, 0);
          }
        }
      }
      du += __shfl_xor(du, 32, 64);
      if (h == 0) dU[b * A + 32 * w + r] = du;
    }
    __syncthreads();
  }

  // per-workgroup partial sums -> slab (reduced by din_bwd_reduce_kernel)
  float* slab = slabs + (size_t)blockIdx.x * slab_floats(A, D);
  if (w < nsl) {
#pragma unroll
    for (int c = 0; c < NCT; ++c)
#pragma unroll
      for (int g = 0; g < 16; ++g) slab[(size_t)(32 * w + acc_row(g, h)) * D + 32 * c + r] = dw[c][g];
    const float t = dw2_acc + __shfl_xor(dw2_acc, 32, 64);
    if (h == 0) slab[(size_t)A * D + 32 * w + r] = t;
  }
  if (w == 0) {
    const float t = wave_sum(db2_acc);
    if (lane == 0) slab[(size_t)A * D + A] = t;
  }
}

// Backward, bf16 pipelined (D <= 128): wave w owns units [32w, 32w+32) and
// accumulates its dW1k slice over all of the workgroup's samples.  Per sample
// the four waves stage {key rows, dpooled, alpha} into an LDS slot with
// global_load_lds, one sample AHEAD (two slots), so there is ONE barrier per
// sample.  dalpha / ds are computed inside every wave from the same key-row
// fragments that feed the z recompute (no cross-wave exchange).
template <int D>
__global__ __launch_bounds__(256, 1) void din_bwd_pipe_kernel(
    const uint16_t* __restrict__ table, const int32_t* __restrict__ ids, int64_t n_table, const float* __restrict__ U,
    const uint16_t* __restrict__ W1k, const float* __restrict__ w2, int B, int L, int A,
    const float* __restrict__ dpooled, const float* __restrict__ alpha, float* __restrict__ dU,
    float* __restrict__ slabs) {
  constexpr int CPR = D / 8, KS = D / 16, NCT = D / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  const int Lp = (L + 31) & ~31, nct = Lp >> 5;
  const int nsl = A >> 5;
  // slot layout (floats): dpooled [D] | alpha [128] | key image [Lp][D] bf16;  plus per-wave ds [4][128]
  const int slot_f = D + 128 + Lp * D / 2;
  float* slot0 = reinterpret_cast<float*>(smem);
  float* dsbuf = slot0 + 2 * slot_f + w * 128;
  typedef __attribute__((address_space(3))) void* lds_ptr;

  WFrag<true, D> wf;
  float w2n = 0.f;
  if (w < nsl) {
    wf.load(W1k, 32 * w + r, h);
    w2n = w2[32 * w + r];
  }
  f32x16 dw[NCT];
#pragma unroll
  for (int c = 0; c < NCT; ++c)
#pragma unroll
    for (int g = 0; g < 16; ++g) dw[c][g] = 0.f;
  float dw2_acc = 0.f, db2_acc = 0.f;

  // cooperative stage of sample b into slot sl (every thread issues its share)
  auto issue = [&](int64_t b, int sl) {
    float* sp = slot0 + sl * slot_f;
    uint16_t* img = reinterpret_cast<uint16_t*>(sp + D + 128);
    const int npieces = Lp * CPR / 64;  // 1-KiB DMA pieces, spread over the 4 waves
    for (int u = w; u < npieces; u += 4) {
      const int p = u * 64 + lane;
      const int row = p / CPR, pc = p % CPR;
      const int cc = pc ^ kswz<CPR>(row);
      const int32_t idr = row < L ? ids[b * L + row] : -1;
      const uint16_t* src = (idr >= 0 && idr < n_table) ? table + (int64_t)idr * D + cc * 8 : g_zero_row;
      __builtin_amdgcn_global_load_lds(src, (lds_ptr)(img + u * 64 * 8), 16, 0, 0);
    }
    if (w == 0) {
#pragma unroll
      for (int u = 0; u < D / 64; ++u)
        __builtin_amdgcn_global_load_lds(dpooled + b * D + u * 64 + lane, (lds_ptr)(sp + u * 64), 4, 0, 0);
    } else if (w == 1) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = u * 64 + lane;
        __builtin_amdgcn_global_load_lds(alpha + b * L + (i < L ? i : 0), (lds_ptr)(sp + D + u * 64), 4, 0, 0);
      }
    }
  };

  int64_t b = blockIdx.x;
  if (b < B) issue(b, 0);
  int sl = 0;
  float un = (w < nsl && b < B) ? U[b * A + 32 * w + r] : 0.f;
  for (; b < B; b += gridDim.x) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // slot sl landed for every wave; slot sl^1 is free
    const int64_t bn = b + gridDim.x;
    if (bn < B) issue(bn, sl ^ 1);
    const float un_next = (w < nsl && bn < B) ? U[bn * A + 32 * w + r] : 0.f;

    const float* sp = slot0 + sl * slot_f;
    const float* sdp = sp;
    const float* sal = sp + D;
    const unsigned char* img = reinterpret_cast<const unsigned char*>(sp + D + 128);
    if (w < nsl) {
      // key-row fragments of every 32-row tile (rows 32c + r, k = 16s + 8h ..), reused twice
      // dalpha[row] = dpooled . K[row]  (halves over h combined)
      float da[4];
      bf16x8 kf[4][KS];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        da[c] = 0.f;
        if (c < nct) {
          const int row = 32 * c + r;
#pragma unroll
          for (int s2 = 0; s2 < KS; ++s2) {
            kf[c][s2] = *reinterpret_cast<const bf16x8*>(img + KImg<true, D>::off(row, 16 * s2 + 8 * h));
#pragma unroll
            for (int j = 0; j < 8; ++j)
              da[c] = fmaf(sdp[16 * s2 + 8 * h + j], bf16_to_f32((uint16_t)kf[c][s2][j]), da[c]);
          }
          da[c] += __shfl_xor(da[c], 32, 64);
        }
      }
      // ds = alpha (dalpha - sum alpha dalpha); rows >= L contribute nothing
      float t = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int row = 32 * c + r;
        t += (c < nct && row < L && h == 0) ? sal[row] * da[c] : 0.f;
      }
      const float cdot = wave_sum(t);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int row = 32 * c + r;
        if (c < nct && h == 0) {
          const float ds = row < L ? sal[row] * (da[c] - cdot) : 0.f;
          dsbuf[row] = ds;
          if (w == 0) db2_acc += ds;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      float du = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c < nct) {
          f32x16 acc;
#pragma unroll
          for (int g = 0; g < 16; ++g) acc[g] = un;
#pragma unroll
          for (int s2 = 0; s2 < KS; ++s2) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[c][s2], wf.f[s2], acc, 0, 0, 0);
          f32x16 dz;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float4 d4 = *reinterpret_cast<const float4*>(dsbuf + 32 * c + 8 * j + 4 * h);
            const float dsv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int g = 4 * j + i;
              const float z = acc[g];
              dw2_acc = fmaf(dsv[i], fmaxf(z, 0.f), dw2_acc);
              const float v = z > 0.f ? dsv[i] * w2n : 0.f;
              dz[g] = v;
              du += v;
            }
          }
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            bf16x8 af;
#pragma unroll
            for (int j = 0; j < 8; ++j) af[j] = (short)f32_to_bf16_rne(dz[8 * s + j]);
            const int grp = lane >> 4, i16 = lane & 15;
            const int rowq = 32 * c + 16 * s + 4 * h + (i16 >> 2);
#pragma unroll
            for (int cc = 0; cc < NCT; ++cc) {
              const int col = 32 * cc + 16 * (grp & 1) + 4 * (i16 & 3);
              typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
              const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + KImg<true, D>::off(rowq, col)));
              const bf16x4 hi =
                  __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + KImg<true, D>::off(rowq + 8, col)));
              bf16x8 bfr;
              bfr[0] = lo[0]; bfr[1] = lo[1]; bfr[2] = lo[2]; bfr[3] = lo[3];
              bfr[4] = hi[0]; bfr[5] = hi[1]; bfr[6] = hi[2]; bfr[7] = hi[3];
              dw[cc] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, dw[cc], 0, 0, 0);
            }
          }
        }
      }
      du += __shfl_xor(du, 32, 64);
      if (h == 0) dU[b * A + 32 * w + r] = du;
    }
    un = un_next;
    sl ^= 1;
  }

  float* slab = slabs + (size_t)blockIdx.x * slab_floats(A, D);
  if (w < nsl) {
#pragma unroll
    for (int c = 0; c < NCT; ++c)
#pragma unroll
      for (int g = 0; g < 16; ++g) slab[(size_t)(32 * w + acc_row(g, h)) * D + 32 * c + r] = dw[c][g];
    const float t = dw2_acc + __shfl_xor(dw2_acc, 32, 64);
    if (h == 0) slab[(size_t)A * D + 32 * w + r] = t;
  }
  if (w == 0) {
    const float t = wave_sum(db2_acc);
    if (lane == 0) slab[(size_t)A * D + A] = t;
  }
}

// Sum the per-workgroup slabs in a fixed order (deterministic): a block owns
// 64 consecutive outputs; its 4 waves each sum every 4th slab, then combine.
__global__ __launch_bounds__(256) void din_bwd_reduce_kernel(const float* __restrict__ slabs, int nslab, int A, int D,
                                                             float* __restrict__ dW1k, float* __restrict__ dw2,
                                                             float* __restrict__ db2) {
  __shared__ float part[4][64];
  const size_t n = slab_floats(A, D);
  const size_t nout = (size_t)A * D + A + 1;
  const int o = threadIdx.x & 63, g = threadIdx.x >> 6;
  const size_t i = (size_t)blockIdx.x * 64 + o;
  float s = 0.f;
  if (i < nout)
    for (int j = g; j < nslab; j += 4) s += slabs[(size_t)j * n + i];
  part[g][o] = s;
  __syncthreads();
  if (g == 0 && i < nout) {
    const float t = (part[0][o] + part[1][o]) + (part[2][o] + part[3][o]);
    if (i < (size_t)A * D) dW1k[i] = t;
    else if (i < (size_t)A * D + A) dw2[i - (size_t)A * D] = t;
    else db2[0] = t;
  }
}

// ================================================================ gather ==
template <bool BF16>
__global__ void gather_rows_kernel(const void* __restrict__ table, int64_t n_table, const int32_t* __restrict__ ids,
                                   int64_t n, int d, float* __restrict__ out) {
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const int32_t id = ids[row];
  const bool ok = id >= 0 && id < n_table;
  for (int c = lane; c < d; c += 64) {
    float v = 0.f;
    if (ok) {
      if constexpr (BF16) v = bf16_to_f32(static_cast<const uint16_t*>(table)[(int64_t)id * d + c]);
      else v = static_cast<const float*>(table)[(int64_t)id * d + c];
    }
    out[row * d + c] = v;
  }
}

}  // namespace nrk

using namespace nrk;

namespace {

int din_grid(int B, bool bwd) {
  // forward: many small workgroups; backward: one workgroup per CU (its
  // registers allow one wave per SIMD) so the per-workgroup gradient slabs
  // stay few
  const char* e = getenv(bwd ? "NRK_DIN_BWD_WGS" : "NRK_DIN_WGS");
  int cap = e && *e ? atoi(e) : (bwd ? 256 : 1024);
  return B < cap ? B : cap;
}

size_t fwd_smem(bool bf16, int d, int L) {
  const int Lp = (L + 31) & ~31;
  const size_t img = bf16 ? (size_t)Lp * d * 2 : (size_t)Lp * (d + 1) * 4;
  const int G = 256 / (d / 2);
  return align_up(img, 16) + (size_t)(4 * Lp + Lp + G * d) * 4;
}

size_t bwd_smem(bool bf16, int d, int L) {
  const int Lp = (L + 31) & ~31;
  const size_t img = bf16 ? (size_t)Lp * d * 2 : (size_t)Lp * (d + 1) * 4;
  return align_up(img, 16) + (size_t)(d + 3 * Lp) * 4;
}

int check_common(const void* keys, int32_t dtype, int32_t B, int32_t L, int32_t d, int32_t A) {
  NRK_CHECK_ARG(keys != nullptr || B == 0, "din: null keys/table");
  NRK_CHECK_ARG(dtype == NRK_DTYPE_F32 || dtype == NRK_DTYPE_BF16, "din: bad dtype %d", dtype);
  NRK_CHECK_ARG(d == 32 || d == 64 || d == 128 || d == 256, "din: emb_dim %d unsupported (32, 64, 128, 256; "
                "the Python layer zero-pads other widths)", d);
  NRK_CHECK_ARG(A >= 32 && A <= 128 && A % 32 == 0, "din: attn_units %d unsupported (32..128 step 32)", A);
  NRK_CHECK_ARG(L >= 1 && L <= 128, "din: history length %d unsupported (1..128)", L);
  NRK_CHECK_ARG(B >= 0, "din: bad batch %d", B);
  return NRK_OK;
}

}  // namespace

#define NRK_DIN_DISPATCH(BF, DD, ...)                          \
  do {                                                         \
    if (BF) {                                                  \
      if (DD == 32) { constexpr bool kBF = true; constexpr int kD = 32; __VA_ARGS__; }   \
      else if (DD == 64) { constexpr bool kBF = true; constexpr int kD = 64; __VA_ARGS__; }   \
      else if (DD == 128) { constexpr bool kBF = true; constexpr int kD = 128; __VA_ARGS__; } \
      else { constexpr bool kBF = true; constexpr int kD = 256; __VA_ARGS__; }           \
    } else {                                                   \
      if (DD == 32) { constexpr bool kBF = false; constexpr int kD = 32; __VA_ARGS__; }  \
      else if (DD == 64) { constexpr bool kBF = false; constexpr int kD = 64; __VA_ARGS__; }  \
      else if (DD == 128) { constexpr bool kBF = false; constexpr int kD = 128; __VA_ARGS__; } \
      else { constexpr bool kBF = false; constexpr int kD = 256; __VA_ARGS__; }          \
    }                                                          \
  } while (0)

extern "C" int nrk_din_attn_fwd(const void* keys, const int32_t* hist_ids, int64_t n_table, int32_t dtype,
                                const float* U, const void* W1k, const float* w2, float b2, int32_t B, int32_t L,
                                int32_t d, int32_t A, float* pooled, float* alpha, void* stream) {
  int rc = check_common(keys, dtype, B, L, d, A);
  if (rc) return rc;
  if (B == 0) return NRK_OK;
  NRK_CHECK_ARG(U && W1k && w2 && pooled && alpha, "din_fwd: null pointer");
  const bool bf = dtype == NRK_DTYPE_BF16;
  const size_t smem = fwd_smem(bf, d, L);
  NRK_CHECK_ARG(smem <= 160 * 1024, "din_fwd: L=%d d=%d needs %zu B LDS", L, d, smem);
  const char* ew = getenv("NRK_DIN_WAVE_FWD");
  const bool wave_ok = bf && hist_ids && (d == 64 || d == 128) && (ew == nullptr || atoi(ew) != 0);
  if (wave_ok) {
    const int Lp = (L + 31) & ~31;
    const size_t AP = (size_t)((A + 63) & ~63);
    const size_t slot = AP * 4 + (size_t)Lp * d * 2;
    const bool dbl = AP * 4 + 4 * 2 * slot <= 150 * 1024;
    const size_t wsm = AP * 4 + 4 * (dbl ? 2 : 1) * slot;
    int grid = (int)cdiv(B, 4);
    const int cap = dbl ? 256 : 512;
    if (grid > cap) grid = cap;
    const uint16_t* tb = static_cast<const uint16_t*>(keys);
    const uint16_t* wk = static_cast<const uint16_t*>(W1k);
    hipStream_t st = (hipStream_t)stream;
#define NRK_FWD_WAVE(DD, NN)                                                                                        \
  do {                                                                                                              \
    if (dbl)                                                                                                        \
      hipLaunchKernelGGL((din_fwd_wave_kernel<DD, NN, 2>), dim3(grid), dim3(256), wsm, st, tb, hist_ids, n_table, U, wk, \
                         w2, B, L, pooled, alpha);                                                                  \
    else                                                                                                            \
      hipLaunchKernelGGL((din_fwd_wave_kernel<DD, NN, 1>), dim3(grid), dim3(256), wsm, st, tb, hist_ids, n_table, U, wk, \
                         w2, B, L, pooled, alpha);                                                                  \
  } while (0)
    const int na = A / 32;
    if (d == 128) {
      if (na == 1) NRK_FWD_WAVE(128, 1); else if (na == 2) NRK_FWD_WAVE(128, 2);
      else if (na == 3) NRK_FWD_WAVE(128, 3); else NRK_FWD_WAVE(128, 4);
    } else {
      if (na == 1) NRK_FWD_WAVE(64, 1); else if (na == 2) NRK_FWD_WAVE(64, 2);
      else if (na == 3) NRK_FWD_WAVE(64, 3); else NRK_FWD_WAVE(64, 4);
    }
#undef NRK_FWD_WAVE
  } else {
    NRK_DIN_DISPATCH(bf, d, {
      hipLaunchKernelGGL((din_fwd_kernel<kBF, kD>), dim3(din_grid(B, false)), dim3(256), smem, (hipStream_t)stream,
                         keys, hist_ids, n_table, U, W1k, w2, b2, B, L, A, pooled, alpha);
    });
  }
  NRK_CHECK_LAUNCH("din_fwd_kernel");
  return NRK_OK;
}

extern "C" int nrk_din_attn_bwd_workspace(int32_t B, int32_t d, int32_t A, size_t* ws_bytes) {
  NRK_CHECK_ARG(ws_bytes != nullptr, "din_bwd_workspace: null");
  *ws_bytes = (size_t)(B > 0 ? din_grid(B, true) : 1) * slab_floats(A, d) * 4;
  return NRK_OK;
}

extern "C" int nrk_din_attn_bwd(const void* keys, const int32_t* hist_ids, int64_t n_table, int32_t dtype,
                                const float* U, const void* W1k, const float* w2, float b2, int32_t B, int32_t L,
                                int32_t d, int32_t A, const float* dpooled, const float* alpha, float* dU,
                                float* dW1k, float* dw2, float* db2, void* ws, size_t ws_bytes, void* stream) {
  (void)b2;
  int rc = check_common(keys, dtype, B, L, d, A);
  if (rc) return rc;
  NRK_CHECK_ARG(dW1k && dw2 && db2, "din_bwd: null gradient pointer");
  hipStream_t st = (hipStream_t)stream;
  if (B == 0) {
    if (hipMemsetAsync(dW1k, 0, (size_t)A * d * 4, st) != hipSuccess || hipMemsetAsync(dw2, 0, (size_t)A * 4, st) ||
        hipMemsetAsync(db2, 0, 4, st))
      return fail(NRK_ELAUNCH, "din_bwd: memset failed");
    return NRK_OK;
  }
  NRK_CHECK_ARG(U && W1k && w2 && dpooled && alpha && dU && ws, "din_bwd: null pointer");
  const int grid = din_grid(B, true);
  const size_t need = (size_t)grid * slab_floats(A, d) * 4;
  if (ws_bytes < need) return fail(NRK_EWORKSPACE, "din_bwd: workspace %zu < %zu", ws_bytes, need);
  const bool bf = dtype == NRK_DTYPE_BF16;
  const size_t smem = bwd_smem(bf, d, L);
  NRK_CHECK_ARG(smem <= 160 * 1024, "din_bwd: L=%d d=%d needs %zu B LDS", L, d, smem);
  float* slabs = static_cast<float*>(ws);
  const char* ep = getenv("NRK_DIN_PIPE_BWD");
  const bool pipe_ok = bf && hist_ids && (d == 64 || d == 128) && (ep == nullptr || atoi(ep) != 0);
  if (pipe_ok) {
    const int Lp = (L + 31) & ~31;
    const size_t psm = (size_t)(2 * (d + 128 + Lp * d / 2) + 4 * 128) * 4;
    NRK_CHECK_ARG(psm <= 160 * 1024, "din_bwd: L=%d d=%d needs %zu B LDS", L, d, psm);
    if (d == 128)
      hipLaunchKernelGGL(din_bwd_pipe_kernel<128>, dim3(grid), dim3(256), psm, st, static_cast<const uint16_t*>(keys),
                         hist_ids, n_table, U, static_cast<const uint16_t*>(W1k), w2, B, L, A, dpooled, alpha, dU, slabs);
    else
      hipLaunchKernelGGL(din_bwd_pipe_kernel<64>, dim3(grid), dim3(256), psm, st, static_cast<const uint16_t*>(keys),
                         hist_ids, n_table, U, static_cast<const uint16_t*>(W1k), w2, B, L, A, dpooled, alpha, dU, slabs);
  } else {
    NRK_DIN_DISPATCH(bf, d, {
      hipLaunchKernelGGL((din_bwd_kernel<kBF, kD>), dim3(grid), dim3(256), smem, st, keys, hist_ids, n_table, U, W1k,
                         w2, B, L, A, dpooled, alpha, dU, slabs);
    });
  }
  NRK_CHECK_LAUNCH("din_bwd_kernel");
  const size_t nout = (size_t)A * d + A + 1;
  hipLaunchKernelGGL(din_bwd_reduce_kernel, dim3((unsigned)cdiv((int64_t)nout, 64)), dim3(256), 0, st, slabs, grid, A,
                     d, dW1k, dw2, db2);
  NRK_CHECK_LAUNCH("din_bwd_reduce_kernel");
  return NRK_OK;
}

extern "C" int nrk_gather_rows(const void* table, int64_t n_table, int32_t dtype, const int32_t* ids, int64_t n,
                               int32_t d, float* out, void* stream) {
  NRK_CHECK_ARG(dtype == NRK_DTYPE_F32 || dtype == NRK_DTYPE_BF16, "gather_rows: bad dtype %d", dtype);
  NRK_CHECK_ARG(d > 0 && n >= 0, "gather_rows: bad shape");
  if (n == 0) return NRK_OK;
  NRK_CHECK_ARG(table && ids && out, "gather_rows: null pointer");
  const unsigned grid = (unsigned)cdiv(n, 4);
  if (dtype == NRK_DTYPE_BF16)
    hipLaunchKernelGGL(gather_rows_kernel<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, table, n_table, ids, n,
                       d, out);
  else
    hipLaunchKernelGGL(gather_rows_kernel<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, table, n_table, ids,
                       n, d, out);
  NRK_CHECK_LAUNCH("gather_rows_kernel");
  return NRK_OK;
}
