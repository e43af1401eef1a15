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
// Zero rows for padding slots / invalid ids (zero-initialised code-object
// global).  Padding is ~60% of the slots at L=50 with uniform history lengths;
// reading ONE zero row from every CU serialises on one L2 channel per XCD, so
// each (sample, row) picks one of 256 distinct zero rows.
__device__ __attribute__((aligned(16))) uint16_t g_zero_rows[256 * 256];
__device__ __forceinline__ const uint16_t* zero_row(int64_t b, int row) {
  return g_zero_rows + (((int)b * 37 + row) & 255) * 256;
}

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
  const int Lp = (L + 31) & ~31;
  // LDS: w2 [AP] (shared) | per wave, NBUF slots of {U row [AP] f32, key image [Lp][D] bf16} | ids [4][128]
  const int slot_f = AP + Lp * D / 2;  // floats per slot
  float* w2s = reinterpret_cast<float*>(smem);
  float* wbase = w2s + AP + (size_t)wv * NBUF * slot_f;
  int32_t* idtab = reinterpret_cast<int32_t*>(w2s + AP + 4 * (size_t)NBUF * slot_f) + wv * 128;  // [128] per wave
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
  // ids of sample b's slots (lane, 64 + lane) and the wave-uniform masks of
  // its valid slots (padding slots hold zero keys and share one logit)
  auto load_ids = [&](int b, int32_t& i0, int32_t& i1, uint64_t& v0, uint64_t& v1) {
    i0 = (b < B && lane < L) ? ids[(int64_t)b * L + lane] : -1;
    i1 = (b < B && lane + 64 < L) ? ids[(int64_t)b * L + lane + 64] : -1;
    v0 = __ballot(i0 >= 0 && i0 < n_table);
    v1 = __ballot(i1 >= 0 && i1 < n_table);
  };
  // gather sample b's key rows, valid slots first (compacted row j <- the
  // (j+1)-th valid slot), zero rows after, + U row into slot `sl` (LDS-DMA);
  // only the 32-row tiles holding the valid rows and the padding row
  auto issue = [&](int b, int sl, int32_t i0, int32_t i1, uint64_t v0, uint64_t v1) {
    float* us = wbase + sl * slot_f;
    uint16_t* img = reinterpret_cast<uint16_t*>(us + AP);
    const int n0 = __popcll(v0), nv = n0 + __popcll(v1);
    const int ntile = (nv + (nv < L ? 1 : 0) + 31) >> 5;
    const int npieces = 32 * ntile * CPR / 64;
    {  // compacted id table of this wave, written by some lanes, read by others below
      const uint64_t below = (1ull << lane) - 1;
      if ((v0 >> lane) & 1) idtab[__popcll(v0 & below)] = i0;
      if ((v1 >> lane) & 1) idtab[n0 + __popcll(v1 & below)] = i1;
      // explicit fence: the LDS stores have completed (lgkmcnt 0) and the
      // compiler may not move the reads across (wave barrier + memory clobber)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
    for (int u = 0; u < npieces; ++u) {
      const int p = u * 64 + lane;
      const int row = p / CPR, pc = p % CPR;
      const int cc = pc ^ kswz<CPR>(row);
      const uint16_t* src = row < nv ? table + (int64_t)idtab[row] * D + cc * 8 : zero_row(b, row) + cc * 8;
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
  uint64_t cv0, cv1, nv0 = 0, nv1 = 0;
  load_ids(b, c0, c1, cv0, cv1);
  if (b < B) issue(b, 0, c0, c1, cv0, cv1);
  if (NBUF == 2) load_ids(b + nw, n0, n1, nv0, nv1);
  int sl = 0;
  for (; b < B; b += nw) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this sample's rows (and the next ids) landed
    const int bn = b + nw;
    // this sample: compacted valid rows [0, nv), the padding row nv (zero
    // key, npad = L - nv slots) when nv < L, nct tiles of 32 rows
    const uint64_t sv0 = cv0, sv1 = cv1;
    const int sn0 = __popcll(sv0), nv = sn0 + __popcll(sv1), npad = L - nv, nr = nv + (npad > 0 ? 1 : 0);
    const int nct = (nr + 31) >> 5;
    if constexpr (NBUF == 2) {
      if (bn < B) issue(bn, sl ^ 1, n0, n1, nv0, nv1);
      cv0 = nv0;
      cv1 = nv1;
      load_ids(bn + nw, n0, n1, nv0, nv1);
    } else {
      // the next sample's ids: loads issued now, consumed (ballots) after this
      // sample's math, so their latency hides behind it
      n0 = (bn < B && lane < L) ? ids[(int64_t)bn * L + lane] : -1;
      n1 = (bn < B && lane + 64 < L) ? ids[(int64_t)bn * L + lane + 64] : -1;
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
        part = half_swap_sum(part);
        sc[c] = (row < nr) ? part : -INFINITY;
      }
    }
    // ---- softmax over the L slots (DIN.py:108, padding included): rows < nv
    // once each, the padding row nv for its npad slots
    float m = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
    m = wave_max_fast(m);
    float e[4], sum = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int row = 32 * c + r;
      e[c] = c < nct && row < nr ? expf(sc[c] - m) : 0.f;
      sum += h == 0 ? (row < nv ? e[c] : (float)npad * e[c]) : 0.f;
    }
    sum = wave_sum_fast(sum);
#pragma unroll
    for (int c = 0; c < 4; ++c) e[c] = e[c] / sum;
    {  // alpha in slot order: a valid slot's compacted row, or the padding row
      auto erow = [&](int row) {
        float v = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float t = __shfl(e[c], row & 31, 64);
          if ((row >> 5) == c) v = t;
        }
        return v;
      };
      const uint64_t below = (1ull << lane) - 1;
      const bool ok0 = (sv0 >> lane) & 1, ok1 = (sv1 >> lane) & 1;
      const float a0 = erow(ok0 ? __popcll(sv0 & below) : nv);
      const float a1 = erow(ok1 ? sn0 + __popcll(sv1 & below) : nv);
      if (lane < L) alpha[(int64_t)b * L + lane] = a0;
      if (64 + lane < L) alpha[(int64_t)b * L + 64 + lane] = a1;
    }
    // ---- pooled = sum_rows alpha[row] K[row][:] over the valid rows
    // rows in groups of 8 up to round_up(nv, 8) <= 32 nct: rows >= nv are zero
    // rows, so the 8 LDS reads of a group issue back to back
    float acc2[DPL];
#pragma unroll
    for (int j = 0; j < DPL; ++j) acc2[j] = 0.f;
    const int L8 = (nv + 7) & ~7;
    for (int row0 = 0; row0 < L8; row0 += 8) {
      const int c = row0 >> 5;
      const float ec = c == 0 ? e[0] : c == 1 ? e[1] : c == 2 ? e[2] : e[3];
      uint32_t u[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (DPL == 2)
          u[i] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const unsigned char*>(img) +
                                                    KImg<true, D>::off(row0 + i, 2 * lane));
        else
          u[i] = *reinterpret_cast<const uint16_t*>(reinterpret_cast<const unsigned char*>(img) +
                                                    KImg<true, D>::off(row0 + i, lane));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float al = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ec), (row0 + i) & 31));
        if constexpr (DPL == 2) {
          acc2[0] = fmaf(al, __uint_as_float(u[i] << 16), acc2[0]);
          acc2[1] = fmaf(al, __uint_as_float(u[i] & 0xFFFF0000u), acc2[1]);
        } else {
          acc2[0] = fmaf(al, bf16_to_f32((uint16_t)u[i]), acc2[0]);
        }
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
      c0 = n0;
      c1 = n1;
      cv0 = __ballot(c0 >= 0 && c0 < n_table);
      cv1 = __ballot(c1 >= 0 && c1 < n_table);
      if (bn < B) issue(bn, 0, c0, c1, cv0, cv1);
    }
  }
}

// Forward at D = 256 (the reference's own training width, DIN.py:16 with the
// 256-d corpus of embedding_generate.py:14): the W1k fragments of all A = 128
// units would take 256 VGPRs, so a PAIR of waves shares one sample: wave half
// hu keeps the unit tiles t = hu, hu + 2, ... (the d = 128 kernel's register
// budget), both gather half of the key rows into the pair's LDS image, the
// partial scores of the two halves meet in LDS (summed in a fixed order, so
// both waves hold identical scores), both run the softmax, and each pools its
// half of the 256 columns.  Four waves = two samples per workgroup, two
// workgroups per CU (LDS).  Same math and padding-row compaction as
// din_fwd_wave_kernel.
template <int D, int NA, int MINB = 2>
__global__ __launch_bounds__(256, MINB) void din_fwd_pair_kernel(const uint16_t* __restrict__ table,
                                                               const int32_t* __restrict__ ids, int64_t n_table,
                                                               const float* __restrict__ U,
                                                               const uint16_t* __restrict__ W1k,
                                                               const float* __restrict__ w2, int B, int L,
                                                               float* __restrict__ pooled,
                                                               float* __restrict__ alpha) {
  constexpr int CPR = D / 8, KS = D / 16, A = 32 * NA;
  constexpr int NAH = (NA + 1) / 2;   // unit tiles per wave half
  constexpr int DH = D / 2, DPL = DH / 64;  // pooled columns per wave half / per lane
  static_assert(DPL == 2 || DPL == 1, "pair kernel: D = 128 or 256");
  constexpr int AP = (A + 63) & ~63;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int pr = wv >> 1, hu = wv & 1;
  const int r = lane & 31, h = lane >> 5;
  const int Lp = (L + 31) & ~31;
  // LDS: w2 [AP] | per pair {U row [AP] f32, key image [Lp][D] bf16} | per wave idtab [128] | per pair xch [2][128]
  const int slot_f = AP + Lp * D / 2;
  float* w2s = reinterpret_cast<float*>(smem);
  float* us = w2s + AP + (size_t)pr * slot_f;
  int32_t* idtab = reinterpret_cast<int32_t*>(w2s + AP + 2 * (size_t)slot_f) + wv * 128;
  float* xch = reinterpret_cast<float*>(w2s + AP + 2 * (size_t)slot_f + 4 * 128) + pr * 256;
  typedef __attribute__((address_space(3))) void* lds_ptr;
  for (int i = threadIdx.x; i < A; i += 256) w2s[i] = w2[i];
  __syncthreads();

  bf16x8 wf[NAH][KS];
#pragma unroll
  for (int i = 0; i < NAH; ++i) {
    const int t = hu + 2 * i < NA ? hu + 2 * i : 0;
#pragma unroll
    for (int s = 0; s < KS; ++s)
      wf[i][s] = *reinterpret_cast<const bf16x8*>(W1k + (int64_t)(32 * t + r) * D + 16 * s + 8 * h);
  }

  const int nw = gridDim.x * 2;  // samples in flight over the grid (one per pair)
  auto load_ids = [&](int b, int32_t& i0, int32_t& i1, uint64_t& v0, uint64_t& v1) {
    i0 = (b < B && lane < L) ? ids[(int64_t)b * L + lane] : -1;
    i1 = (b < B && lane + 64 < L) ? ids[(int64_t)b * L + lane + 64] : -1;
    v0 = __ballot(i0 >= 0 && i0 < n_table);
    v1 = __ballot(i1 >= 0 && i1 < n_table);
  };
  // this wave's half of sample b's key pieces (compacted valid rows, then the
  // padding row), and the U row (wave half 0)
  auto issue = [&](int b, int32_t i0, int32_t i1, uint64_t v0, uint64_t v1) {
    uint16_t* img = reinterpret_cast<uint16_t*>(us + AP);
    const int n0 = __popcll(v0), nv = n0 + __popcll(v1);
    const int ntile = (nv + (nv < L ? 1 : 0) + 31) >> 5;
    const int npieces = 32 * ntile * CPR / 64;
    {
      const uint64_t below = (1ull << lane) - 1;
      if ((v0 >> lane) & 1) idtab[__popcll(v0 & below)] = i0;
      if ((v1 >> lane) & 1) idtab[n0 + __popcll(v1 & below)] = i1;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
    for (int u = hu; u < npieces; u += 2) {
      const int p = u * 64 + lane;
      const int row = p / CPR, pc = p % CPR;
      const int cc = pc ^ kswz<CPR>(row);
      const uint16_t* src = row < nv ? table + (int64_t)idtab[row] * D + cc * 8 : zero_row(b, row) + cc * 8;
      __builtin_amdgcn_global_load_lds(src, (lds_ptr)(img + u * 64 * 8), 16, 0, 0);
    }
    if (hu == 0) {
#pragma unroll
      for (int u = 0; u < AP / 64; ++u) {
        const int i = u * 64 + lane;
        __builtin_amdgcn_global_load_lds(U + (int64_t)b * A + (i < A ? i : 0), (lds_ptr)(us + u * 64), 4, 0, 0);
      }
    }
  };

  // trip count uniform over the workgroup (barriers): pair 0's samples lead
  const int b0 = blockIdx.x * 2;
  int b = b0 + pr;
  int32_t c0, c1;
  uint64_t cv0, cv1;
  load_ids(b, c0, c1, cv0, cv1);
  if (b < B) issue(b, c0, c1, cv0, cv1);
  for (int bl = b0; bl < B; bl += nw, b += nw) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // both halves of every pair's image (and U row) landed
    const bool act = b < B;
    const uint64_t sv0 = cv0, sv1 = cv1;
    const int sn0 = __popcll(sv0), nv = sn0 + __popcll(sv1), npad = L - nv, nr = nv + (npad > 0 ? 1 : 0);
    const int nct = act ? (nr + 31) >> 5 : 0;
    const uint16_t* img = reinterpret_cast<const uint16_t*>(us + AP);
    // ---- partial scores over this half's units
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c < nct) {
        const int row = 32 * c + r;
        // k-outer: one key fragment live at a time, the half's unit tiles side by side
        f32x16 acc[NAH];
#pragma unroll
        for (int i = 0; i < NAH; ++i) {
          const int t = hu + 2 * i < NA ? hu + 2 * i : 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float4 uv = *reinterpret_cast<const float4*>(us + 32 * t + 8 * j + 4 * h);
            acc[i][4 * j] = uv.x; acc[i][4 * j + 1] = uv.y; acc[i][4 * j + 2] = uv.z; acc[i][4 * j + 3] = uv.w;
          }
        }
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(img + row * D + 8 * ((2 * s2 + h) ^ kswz<CPR>(row)));
#pragma unroll
          for (int i = 0; i < NAH; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i][s2], kf, acc[i], 0, 0, 0);
        }
        float part = 0.f;
#pragma unroll
        for (int i = 0; i < NAH; ++i) {
          const int t = hu + 2 * i;
          if (t >= NA) continue;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float4 wv4 = *reinterpret_cast<const float4*>(w2s + 32 * t + 8 * j + 4 * h);
            part = fmaf(wv4.x, fmaxf(acc[i][4 * j], 0.f), part);
            part = fmaf(wv4.y, fmaxf(acc[i][4 * j + 1], 0.f), part);
            part = fmaf(wv4.z, fmaxf(acc[i][4 * j + 2], 0.f), part);
            part = fmaf(wv4.w, fmaxf(acc[i][4 * j + 3], 0.f), part);
          }
        }
        part = half_swap_sum(part);
        if (h == 0) xch[hu * 128 + row] = part;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();  // both halves' partial scores
    float sc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int row = 32 * c + r;
      sc[c] = (c < nct && row < nr) ? xch[row] + xch[128 + row] : -INFINITY;
    }
    float m = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
    m = wave_max_fast(m);
    float e[4], sum = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int row = 32 * c + r;
      e[c] = c < nct && row < nr ? expf(sc[c] - m) : 0.f;
      sum += h == 0 ? (row < nv ? e[c] : (float)npad * e[c]) : 0.f;
    }
    sum = wave_sum_fast(sum);
#pragma unroll
    for (int c = 0; c < 4; ++c) e[c] = e[c] / sum;
    if (act && hu == 0) {
      auto erow = [&](int row) {
        float v = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float t = __shfl(e[c], row & 31, 64);
          if ((row >> 5) == c) v = t;
        }
        return v;
      };
      const uint64_t below = (1ull << lane) - 1;
      const bool ok0 = (sv0 >> lane) & 1, ok1 = (sv1 >> lane) & 1;
      const float a0 = erow(ok0 ? __popcll(sv0 & below) : nv);
      const float a1 = erow(ok1 ? sn0 + __popcll(sv1 & below) : nv);
      if (lane < L) alpha[(int64_t)b * L + lane] = a0;
      if (64 + lane < L) alpha[(int64_t)b * L + 64 + lane] = a1;
    }
    if (act) {  // ---- pooled, this half's DH columns
      float acc2[DPL];
#pragma unroll
      for (int j = 0; j < DPL; ++j) acc2[j] = 0.f;
      const int L8 = (nv + 7) & ~7;
      for (int row0 = 0; row0 < L8; row0 += 8) {
        const int c = row0 >> 5;
        const float ec = c == 0 ? e[0] : c == 1 ? e[1] : c == 2 ? e[2] : e[3];
        uint32_t u[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if constexpr (DPL == 2)
            u[i] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const unsigned char*>(img) +
                                                      KImg<true, D>::off(row0 + i, DH * hu + 2 * lane));
          else
            u[i] = *reinterpret_cast<const uint16_t*>(reinterpret_cast<const unsigned char*>(img) +
                                                      KImg<true, D>::off(row0 + i, DH * hu + lane));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float al = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ec), (row0 + i) & 31));
          if constexpr (DPL == 2) {
            acc2[0] = fmaf(al, __uint_as_float(u[i] << 16), acc2[0]);
            acc2[1] = fmaf(al, __uint_as_float(u[i] & 0xFFFF0000u), acc2[1]);
          } else {
            acc2[0] = fmaf(al, __uint_as_float(u[i] << 16), acc2[0]);
          }
        }
      }
      if constexpr (DPL == 2)
        *reinterpret_cast<float2*>(pooled + (int64_t)b * D + DH * hu + 2 * lane) = make_float2(acc2[0], acc2[1]);
      else
        pooled[(int64_t)b * D + DH * hu + lane] = acc2[0];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();  // every read of the pair's image and exchange is done: refill
    load_ids(b + nw, c0, c1, cv0, cv1);
    if (b + nw < B) issue(b + nw, c0, c1, cv0, cv1);
  }
}

// =============================================================== backward ==
// Workgroup slab layout (floats): dW1k [A][D], then dw2 [A], then db2 [1].
// The pipelined backward with the query (nrk_din_attn_bwd_params) appends
// dW1q [A][D] and db1 [A] at slab_q_off.
__host__ __device__ __forceinline__ size_t slab_q_off(int A, int D) { return ((size_t)A * D + A + 4 + 31) / 32 * 32; }
// slab stride rounded up to 32 floats: every slab starts on a 128-B line, so the
// parameter reduction's 64-float output windows read 2 whole lines per slab (an
// unaligned stride made it 3, the boundary line shared with a block on another
// XCD: 26.5 MB fetched per launch for 16.9 MB of slabs at B = 4096)
__host__ __device__ __forceinline__ size_t slab_floats(int A, int D) {
  return (slab_q_off(A, D) + (size_t)A * D + A + 4 + 31) / 32 * 32;
}

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
        // dW1k[n][c] += sum_rows dz[row][n] K[row][c]; dz enters as bf16 hi + lo
        // (this generic kernel is off the timed path: near-fp32 gradients)
        if constexpr (BF16) {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            bf16x8 af, afl;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const uint16_t hb = f32_to_bf16_rne(dz[8 * s + j]);
              af[j] = (short)hb;
              afl[j] = (short)f32_to_bf16_rne(dz[8 * s + j] - bf16_to_f32(hb));
            }
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
              dw[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afl, bf, dw[c], 0, 0, 0);
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
    float* __restrict__ slabs, const float* __restrict__ q, int dq) {
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
  // query half of W1 (q != nullptr): dW1q = sum_b dU[b] q[b]^T on f32 MFMA,
  // two samples per 32x32x2 step (lanes h = 0 / 1 carry the older / newer
  // sample), and db1 = sum_b dU[b]
  f32x16 dwq[NCT];
#pragma unroll
  for (int c = 0; c < NCT; ++c)
#pragma unroll
    for (int g = 0; g < 16; ++g) dwq[c][g] = 0.f;
  float db1_acc = 0.f, du_prev = 0.f;
  float qprev[NCT];
#pragma unroll
  for (int c = 0; c < NCT; ++c) qprev[c] = 0.f;
  int npair = 0;

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
      const uint16_t* src = (idr >= 0 && idr < n_table) ? table + (int64_t)idr * D + cc * 8 : zero_row(b, row) + cc * 8;
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
    float qcur[NCT];
    if (q != nullptr) {
#pragma unroll
      for (int c = 0; c < NCT; ++c) qcur[c] = 32 * c + r < dq ? q[b * dq + 32 * c + r] : 0.f;
    }
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
      if (h == 0 && dU != nullptr) dU[b * A + 32 * w + r] = du;
      if (q != nullptr) {
        db1_acc += du;
        if (npair & 1) {
          const float av = h ? du : du_prev;
#pragma unroll
          for (int c = 0; c < NCT; ++c)
            dwq[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, h ? qcur[c] : qprev[c], dwq[c], 0, 0, 0);
        }
        du_prev = du;
#pragma unroll
        for (int c = 0; c < NCT; ++c) qprev[c] = qcur[c];
        ++npair;
      }
    }
    un = un_next;
    sl ^= 1;
  }
  if (q != nullptr && w < nsl && (npair & 1)) {  // odd tail: the newer-sample half is zero
    const float av = h ? 0.f : du_prev;
#pragma unroll
    for (int c = 0; c < NCT; ++c) dwq[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, h ? 0.f : qprev[c], dwq[c], 0, 0, 0);
  }

  float* slab = slabs + (size_t)blockIdx.x * slab_floats(A, D);
  if (w < nsl) {
#pragma unroll
    for (int c = 0; c < NCT; ++c)
#pragma unroll
      for (int g = 0; g < 16; ++g) slab[(size_t)(32 * w + acc_row(g, h)) * D + 32 * c + r] = dw[c][g];
    const float t = dw2_acc + __shfl_xor(dw2_acc, 32, 64);
    if (h == 0) slab[(size_t)A * D + 32 * w + r] = t;
    if (q != nullptr) {
      float* sq = slab + slab_q_off(A, D);
#pragma unroll
      for (int c = 0; c < NCT; ++c)
#pragma unroll
        for (int g = 0; g < 16; ++g) sq[(size_t)(32 * w + acc_row(g, h)) * D + 32 * c + r] = dwq[c][g];
      if (h == 0) sq[(size_t)A * D + 32 * w + r] = db1_acc;
    }
  }
  if (w == 0) {
    const float t = wave_sum(db2_acc);
    if (lane == 0) slab[(size_t)A * D + A] = t;
  }
}

// Backward for the fused train step (query half folded in, no dU output),
// pipelined TWO samples ahead with every per-sample input moved by LDS-DMA
// issued from inline asm (hipcc neither sees nor waits for it, so no
// conservative vmcnt(0) lands in front of the LDS reads of the current
// sample): three LDS slots of {dpooled, alpha, U row, q row, key image} and
// a per-wave ring of history ids one sample further ahead.  Each wave issues
// the same N_D DMA ops per iteration (out-of-range samples / rows read
// clamped addresses or the zero row), so the waits are counted vmcnt:
//   top of iteration: vmcnt(N_D)  -> the DMA group of this sample landed,
//   then s_waitcnt lgkmcnt(0) + raw s_barrier (never __syncthreads, whose
//   fence would drain every DMA in flight);
//   before issuing: vmcnt(N_D)    -> the ids of the sample being issued landed.
// LP = padded history rows (32, 64 or 128; rows >= L are zero rows).
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_hw;
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)p;
}
__device__ __forceinline__ void glds16_asm(const void* gsrc, uint32_t lds_dst) {
  lds_dst = __builtin_amdgcn_readfirstlane(lds_dst);  // wave-uniform by construction
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
__device__ __forceinline__ void glds4_asm(const void* gsrc, uint32_t lds_dst) {
  lds_dst = __builtin_amdgcn_readfirstlane(lds_dst);  // wave-uniform by construction
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

// Where the fused train step's attention backward finds dpooled's inputs when
// it forms dpooled itself (FDP): the head's state after nrk_din_head_train
// (nrk_din_head_ws_views) and the forward's pooled rows.  stat0 / sum5 / bn0w /
// w1 are indexed over the head's 2d input columns (the pooled half from d).
struct DpSrc {
  const float* pooled;  // [B][D]
  const float* da1;     // [B][32]
  const float* w1;      // fc.1 weight [32][2D]
  const float* stat0;   // {mean [2D], invstd [2D]}
  const double* sum5;   // {sum dh0 [2D], sum dh0 xhat0 [2D]}
  const float* bn0w;    // fc.0 weight [2D]
  float invB;
};

template <int D, int LP, int NSLOT>
__global__ __launch_bounds__(256, 1) void din_bwd_deep_kernel(
    const uint16_t* __restrict__ table, const int32_t* __restrict__ ids, int64_t n_table, const float* __restrict__ U,
    const uint16_t* __restrict__ W1k, const float* __restrict__ w2, int B, int L, int A,
    const float* __restrict__ dpooled, const float* __restrict__ alpha, float* __restrict__ slabs,
    const float* __restrict__ q, int dq) {
  constexpr int CPR = D / 8, KS = D / 16, NCT = D / 32, NC = LP / 32;
  constexpr int NPW = LP * CPR / 256;  // key-image DMA pieces per wave
  constexpr int N_IDS = LP > 64 ? 2 : 1;
  constexpr int N_D = NPW + 2 + N_IDS;  // per wave and iteration: keys, two small pieces, the ids pieces
  constexpr int P = NSLOT - 1;          // data groups in flight ahead of the sample computed
  constexpr int X = 3, RING = X + 1;    // ids are fetched X iterations before their data group
  static_assert(NPW >= 1 && P >= 2 && P <= X && X * N_D < 64, "vmcnt range");
  // slot (floats): dpooled [128] | alpha [128] | U [128] | q [128] | key image [LP][D] bf16
  constexpr int SLOT_F = 4 * 128 + LP * D / 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nsl = A >> 5;
  float* slot0 = reinterpret_cast<float*>(smem);
  int32_t* idring = reinterpret_cast<int32_t*>(slot0 + NSLOT * SLOT_F) + w * RING * 128;  // [RING][128] per wave
  float* dsbuf = reinterpret_cast<float*>(reinterpret_cast<int32_t*>(slot0 + NSLOT * SLOT_F) + 4 * RING * 128) + w * 128;
  float* dabuf = reinterpret_cast<float*>(reinterpret_cast<int32_t*>(slot0 + NSLOT * SLOT_F) + 4 * RING * 128) + 4 * 128;

  WFrag<true, D> wf;
  const int wu = w < nsl ? w : 0;
  wf.load(W1k, 32 * wu + r, h);
  const float w2n = w2[32 * wu + r];
#pragma unroll
  for (int s2 = 0; s2 < KS; ++s2) asm volatile("" ::"v"(wf.f[s2]));  // hipcc's waits for these land here
  asm volatile("" ::"v"(w2n));
  f32x16 dw[NCT], dwq[NCT];
#pragma unroll
  for (int c = 0; c < NCT; ++c)
#pragma unroll
    for (int g = 0; g < 16; ++g) dw[c][g] = dwq[c][g] = 0.f;
  float dw2_acc = 0.f, db2_acc = 0.f, db1_acc = 0.f;

  // ids of sample b (all LP rows; clamped) into ring entry e of this wave
  auto issue_ids = [&](int64_t b, int e) {
    const int64_t bc = b < B ? b : 0;
    const int i = lane < LP ? lane : 0;
    glds4_asm(ids + bc * L + (i < L ? i : 0), lds_u32(idring + e * 128));
    if constexpr (LP > 64) glds4_asm(ids + bc * L + (64 + lane < L ? 64 + lane : 0), lds_u32(idring + e * 128 + 64));
  };
  // key rows + small pieces of sample b (its ids in ring entry e) into slot sl
  auto issue_data = [&](int64_t b, int sl, int e) {
    float* sp = slot0 + sl * SLOT_F;
    uint16_t* img = reinterpret_cast<uint16_t*>(sp + 4 * 128);
#pragma unroll
    for (int k = 0; k < NPW; ++k) {
      const int u = w + 4 * k;
      const int p = u * 64 + lane;
      const int row = p / CPR, pc = p % CPR;
      const int cc = pc ^ kswz<CPR>(row);
      const int32_t idv0 = idring[e * 128 + row];
      const int32_t idr = row < L && b < B ? idv0 : -1;
      const uint16_t* src = (idr >= 0 && idr < n_table) ? table + (int64_t)idr * D + cc * 8 : zero_row(b, row) + cc * 8;
      glds16_asm(src, lds_u32(img + u * 64 * 8));
    }
    const int64_t bc = b < B ? b : 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // small pieces 2w, 2w+1 of [dp0, dp1, al0, al1, u0, u1, q0, q1]
      const int pc = 2 * w + k, kind = pc >> 1, part = pc & 1;
      const int i = part * 64 + lane;
      const float* base = kind == 0 ? dpooled + bc * D : kind == 1 ? alpha + bc * L : kind == 2 ? U + bc * A : q + bc * dq;
      const int lim = kind == 0 ? D : kind == 1 ? L : kind == 2 ? A : dq;
      glds4_asm(base + (i < lim ? i : 0), lds_u32(sp + kind * 128 + part * 64));
    }
  };

  const int64_t grid = gridDim.x;
  int64_t b = blockIdx.x;
#pragma unroll
  for (int k = 0; k < X; ++k) issue_ids(b + k * grid, k);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int k = 0; k < P; ++k) {
    issue_ids(b + (k + X) * grid, (k + X) % RING);
    issue_data(b + k * grid, k, k);
  }
  int sl = 0, e = P % RING;  // e: ring entry holding the ids of sample b + P grid
  for (; b < B; b += grid) {
    // this wave's DMA group of sample b landed; all waves' after the barrier; slot of b - grid is free
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"((P - 1) * N_D) : "memory");
    issue_ids(b + (P + X) * grid, e + X < RING ? e + X : e + X - RING);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(X * N_D) : "memory");  // ids of b + P grid landed
    issue_data(b + P * grid, sl + P < NSLOT ? sl + P : sl + P - NSLOT, e);
    e = e + 1 < RING ? e + 1 : 0;

    const float* sp = slot0 + sl * SLOT_F;
    const float* sdp = sp;
    const float* sal = sp + 128;
    const float* sU = sp + 256;
    const float* sq = sp + 384;
    const unsigned char* img = reinterpret_cast<const unsigned char*>(sp + 512);
    {  // dalpha[row] = dpooled . K[row], split over the waves: wave w owns rows [w R, (w+1) R)
      constexpr int R = LP / 4, LPR = 64 / R, CH = CPR / LPR;
      const int row = w * R + lane / LPR, part = lane % LPR;
      float acc = 0.f;
#pragma unroll
      for (int ch = 0; ch < CH; ++ch) {
        const int cc = part * CH + ch;
        const uint4 kv = *reinterpret_cast<const uint4*>(img + row * 2 * D + 16 * (cc ^ kswz<CPR>(row)));
        const float4 d0 = *reinterpret_cast<const float4*>(sdp + 8 * cc);
        const float4 d1 = *reinterpret_cast<const float4*>(sdp + 8 * cc + 4);
        acc = fmaf(d0.x, __uint_as_float(kv.x << 16), acc);
        acc = fmaf(d0.y, __uint_as_float(kv.x & 0xFFFF0000u), acc);
        acc = fmaf(d0.z, __uint_as_float(kv.y << 16), acc);
        acc = fmaf(d0.w, __uint_as_float(kv.y & 0xFFFF0000u), acc);
        acc = fmaf(d1.x, __uint_as_float(kv.z << 16), acc);
        acc = fmaf(d1.y, __uint_as_float(kv.z & 0xFFFF0000u), acc);
        acc = fmaf(d1.z, __uint_as_float(kv.w << 16), acc);
        acc = fmaf(d1.w, __uint_as_float(kv.w & 0xFFFF0000u), acc);
      }
#pragma unroll
      for (int o = 1; o < LPR; o <<= 1) acc += __shfl_xor(acc, o, 64);
      if (part == 0) dabuf[row] = acc;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (w < nsl) {
      const float un = sU[32 * w + r];
      float qcur[NCT];
#pragma unroll
      for (int c = 0; c < NCT; ++c) qcur[c] = 32 * c + r < dq ? sq[32 * c + r] : 0.f;
      float da[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) da[c] = dabuf[32 * c + r];
      float t = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int row = 32 * c + r;
        t += (row < L && h == 0) ? sal[row] * da[c] : 0.f;
      }
      const float cdot = wave_sum(t);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int row = 32 * c + r;
        if (h == 0) {
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
      for (int c = 0; c < NC; ++c) {
        f32x16 acc;
#pragma unroll
        for (int g = 0; g < 16; ++g) acc[g] = un;
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(img + KImg<true, D>::off(32 * c + r, 16 * s2 + 8 * h));
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, wf.f[s2], acc, 0, 0, 0);
        }
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
          for (int j = 0; j < 4; ++j) {  // v_cvt_pk_bf16_f32 (round to nearest even)
            const bf16x2_hw pk = {(__bf16)dz[8 * s + 2 * j], (__bf16)dz[8 * s + 2 * j + 1]};
            const uint32_t u = __builtin_bit_cast(uint32_t, pk);
            af[2 * j] = (short)(u & 0xFFFF);
            af[2 * j + 1] = (short)(u >> 16);
          }
          const int grp = lane >> 4, i16 = lane & 15;
          const int rowq = 32 * c + 16 * s + 4 * h + (i16 >> 2);
#pragma unroll
          for (int cc = 0; cc < NCT; ++cc) {
            const int col = 32 * cc + 16 * (grp & 1) + 4 * (i16 & 3);
            typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
            const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + KImg<true, D>::off(rowq, col)));
            const bf16x4 hi =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + KImg<true, D>::off(rowq + 8, col)));
            const bf16x8 bfr = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
            dw[cc] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, dw[cc], 0, 0, 0);
          }
        }
      }
      du += __shfl_xor(du, 32, 64);
      db1_acc += du;
      // dW1q += dU q^T: one sample per 32x32x2 step (k = 1 half zero), no branch
#pragma unroll
      for (int c = 0; c < NCT; ++c)
        dwq[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(h ? 0.f : du, h ? 0.f : qcur[c], dwq[c], 0, 0, 0);
    }
    sl = sl == NSLOT - 1 ? 0 : sl + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup exits
  float* slab = slabs + (size_t)blockIdx.x * slab_floats(A, D);
  if (w < nsl) {
    float* sqs = slab + slab_q_off(A, D);
#pragma unroll
    for (int c = 0; c < NCT; ++c)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        slab[(size_t)(32 * w + acc_row(g, h)) * D + 32 * c + r] = dw[c][g];
        sqs[(size_t)(32 * w + acc_row(g, h)) * D + 32 * c + r] = dwq[c][g];
      }
    const float t = dw2_acc + __shfl_xor(dw2_acc, 32, 64);
    if (h == 0) {
      slab[(size_t)A * D + 32 * w + r] = t;
      sqs[(size_t)A * D + 32 * w + r] = db1_acc;
    }
  }
  if (w == 0) {
    const float t = wave_sum(db2_acc);
    if (lane == 0) slab[(size_t)A * D + A] = t;
  }
}

// 8-wave variant (two waves per SIMD): waves w and w + 4 own the same 32
// units (us = w & 3) and split the sample's 32-row history tiles (rg = w >> 2
// takes tiles rg, rg + 2, ...); each accumulates its rows' share of every
// gradient, and the pairs are combined in a fixed order after the loop.
template <int D, int LP, int NSLOT, bool FQ, bool FDP>
__global__ __launch_bounds__(512, 1) void din_bwd_deep8_kernel(
    const uint16_t* __restrict__ table, const int32_t* __restrict__ ids, int64_t n_table, const float* __restrict__ U,
    const uint16_t* __restrict__ W1k, const float* __restrict__ w2, int B, int L, int A,
    const float* __restrict__ dpooled, const float* __restrict__ alpha, float* __restrict__ slabs,
    const float* __restrict__ q, int dq, float* __restrict__ dUp, float* __restrict__ dummy, DpSrc dps) {
  constexpr int CPR = D / 8, KS = D / 16, NCT = D / 32, NC = LP / 32;
  constexpr int NPW = LP * CPR / 512;  // key-image DMA pieces per wave
  constexpr int N_IDS = LP > 64 ? 2 : 1;
  // per wave and iteration: [the dU store,] keys, one small piece, ids.  FQ: dW1q is folded in here
  // (the samples' dU and q rows staged in LDS, one f32 MFMA pass after the loop; the host uses FQ
  // only when a workgroup has <= 16 samples: a flush inside the loop spilled 56 VGPRs), no dU stores
  constexpr int N_D = (FQ ? 0 : 1) + NPW + 1 + N_IDS;
  constexpr int P = NSLOT - 1;          // data groups in flight ahead of the sample computed
  constexpr int X = P > 3 ? P : 3, RING = X + 1;  // ids are fetched X iterations before their data group
  static_assert(NPW >= 0 && P >= 2 && P <= X && X * N_D < 64, "vmcnt range");
  // slot (floats): dpooled [128] | alpha [128] | U [128] | q [128] | key image [LP][D] bf16
  constexpr int SLOT_F = 4 * 128 + LP * D / 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int us = w & 3, rg = w >> 2;
  const int nsl = A >> 5;
  float* slot0 = reinterpret_cast<float*>(smem);
  int32_t* idring = reinterpret_cast<int32_t*>(slot0 + NSLOT * SLOT_F) + w * RING * 128;  // [RING][128] per wave
  float* dsbuf = reinterpret_cast<float*>(reinterpret_cast<int32_t*>(slot0 + NSLOT * SLOT_F) + 8 * RING * 128) + w * 128;
  float* dabuf = reinterpret_cast<float*>(reinterpret_cast<int32_t*>(slot0 + NSLOT * SLOT_F) + 8 * RING * 128) + 8 * 128;
  float* dul = dabuf + 128;                       // FQ: [16][2 row groups][128] dU rows of the samples
  float* ql = dul + (FQ ? 16 * 2 * 128 : 0);      // FQ: [16][128] their query rows
  // FDP: dpooled formed here from the head's state (BN0 backward of da1 W1[:, d:]), no
  // separate launch: W1p [32][D] (fc.1 weight, pooled half), per pooled column {mean,
  // invstd, gamma, sum dh0 / B, sum dh0 xhat0 / B}, and this sample's dpooled [D]
  float* w1p = ql + (FQ ? 16 * 128 : 0);
  float* colc = w1p + (FDP ? 32 * D : 0);
  float* dpl = colc + 5 * D;
  static_assert(!FDP || LP <= 64, "FDP: the da1 row takes the second alpha piece");
  if constexpr (FDP) {
    for (int i = tid; i < 32 * D; i += 512) w1p[i] = dps.w1[(size_t)(i / D) * 2 * D + D + i % D];
    for (int c = tid; c < D; c += 512) {
      colc[c] = dps.stat0[D + c];
      colc[D + c] = dps.stat0[3 * D + c];
      colc[2 * D + c] = dps.bn0w[D + c];
      colc[3 * D + c] = (float)dps.sum5[D + c] * dps.invB;
      colc[4 * D + c] = (float)dps.sum5[3 * D + c] * dps.invB;
    }
    // ordered before the first use by the loop's barriers
  }

  WFrag<true, D> wf;
  const int wu = us < nsl ? us : 0;
  wf.load(W1k, 32 * wu + r, h);
  const float w2n = w2[32 * wu + r];
#pragma unroll
  for (int s2 = 0; s2 < KS; ++s2) asm volatile("" ::"v"(wf.f[s2]));  // hipcc's waits for these land here
  asm volatile("" ::"v"(w2n));
  f32x16 dw[NCT];
#pragma unroll
  for (int c = 0; c < NCT; ++c)
#pragma unroll
    for (int g = 0; g < 16; ++g) dw[c][g] = 0.f;
  float dw2_acc = 0.f, db2_acc = 0.f, db1_acc = 0.f;
  // this wave's rows' share of dU of the previous sample, stored (asm, counted
  // in the vmcnt plan) at the top of the next iteration; dW1q = sum dU q^T is
  // formed from these rows by din_dwq_kernel
  float du_keep = 0.f;
  int64_t b_keep = -1;
  float* const dmy = dummy + (size_t)blockIdx.x * 512 + tid;
  auto store_du = [&]() {
    if constexpr (!FQ) {
      float* dst = (b_keep >= 0 && us < nsl && h == 0) ? dUp + ((size_t)rg * B + b_keep) * A + 32 * us + r : dmy;
      asm volatile("global_store_dword %0, %1, off" ::"v"(dst), "v"(du_keep) : "memory");
    }
  };
  // FQ: dW1q partial of the staged samples [0, ns) into this workgroup's slab:
  // wave (us, rg) owns tiles n = 32 us.., k = 32 (rg + 2 j)..
  float* const sqs_slab = slabs + (size_t)blockIdx.x * slab_floats(A, D) + slab_q_off(A, D);
  auto flush_q = [&](int ns) {
    if (us < nsl) {
#pragma unroll
      for (int j = 0; j < (NCT + 1) / 2; ++j) {
        const int tk = rg + 2 * j;
        if (tk >= NCT) continue;
        f32x16 acc;
#pragma unroll
        for (int g = 0; g < 16; ++g) acc[g] = 0.f;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const int sm = 2 * kk + h;
          const float av = sm < ns ? dul[sm * 256 + 32 * us + r] + dul[sm * 256 + 128 + 32 * us + r] : 0.f;
          const float bv = sm < ns ? ql[sm * 128 + 32 * tk + r] : 0.f;
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
        }
#pragma unroll
        for (int g = 0; g < 16; ++g) sqs_slab[(size_t)(32 * us + acc_row(g, h)) * D + 32 * tk + r] = acc[g];
      }
    }
  };
  int it = 0;  // samples of this workgroup so far

  // ids of sample b (all LP rows; clamped) into ring entry e of this wave
  auto issue_ids = [&](int64_t b, int e) {
    const int64_t bc = b < B ? b : 0;
    const int i = lane < LP ? lane : 0;
    glds4_asm(ids + bc * L + (i < L ? i : 0), lds_u32(idring + e * 128));
    if constexpr (LP > 64) glds4_asm(ids + bc * L + (64 + lane < L ? 64 + lane : 0), lds_u32(idring + e * 128 + 64));
  };
  // key rows + small pieces of sample b (its ids in ring entry e) into slot sl
  auto issue_data = [&](int64_t b, int sl, int e) {
    float* sp = slot0 + sl * SLOT_F;
    uint16_t* img = reinterpret_cast<uint16_t*>(sp + 4 * 128);
#pragma unroll
    for (int k = 0; k < NPW; ++k) {
      const int u = w + 8 * k;
      const int p = u * 64 + lane;
      const int row = p / CPR, pc = p % CPR;
      const int cc = pc ^ kswz<CPR>(row);
      const int32_t idv0 = idring[e * 128 + row];
      const int32_t idr = row < L && b < B ? idv0 : -1;
      const uint16_t* src = (idr >= 0 && idr < n_table) ? table + (int64_t)idr * D + cc * 8 : zero_row(b, row) + cc * 8;
      glds16_asm(src, lds_u32(img + u * 64 * 8));
    }
    const int64_t bc = b < B ? b : 0;
    {  // small piece w of [dp0, dp1, al0, al1, u0, u1, q0, q1]
       // (FDP: pooled instead of dpooled, and the da1 row [32] in the al1 piece)
      const int pc = w, kind = pc >> 1, part = pc & 1;
      const int i = part * 64 + lane;
      const float* base = kind == 0 ? (FDP ? dps.pooled : dpooled) + bc * D : kind == 1 ? alpha + bc * L
                          : kind == 2 ? U + bc * A : q + bc * dq;
      int lim = kind == 0 ? D : kind == 1 ? L : kind == 2 ? A : dq;
      if (FDP && pc == 3) {
        base = dps.da1 + bc * 32;
        lim = 32;
      }
      const int ii = FDP && pc == 3 ? lane : i;
      glds4_asm(base + (ii < lim ? ii : 0), lds_u32(sp + kind * 128 + part * 64));
    }
  };

  const int64_t grid = gridDim.x;
  int64_t b = blockIdx.x;
#pragma unroll
  for (int k = 0; k < X; ++k) issue_ids(b + k * grid, k);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int k = 0; k < P; ++k) {
    store_du();  // nothing to store yet: the dummy slot (keeps every group the same size)
    issue_ids(b + (k + X) * grid, (k + X) % RING);
    issue_data(b + k * grid, k, k);
  }
  int sl = 0, e = P % RING;  // e: ring entry holding the ids of sample b + P grid
  for (; b < B; b += grid) {
    // this wave's DMA group of sample b landed; all waves' after the barrier; slot of b - grid is free
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"((P - 1) * N_D) : "memory");
    store_du();
    issue_ids(b + (P + X) * grid, e + X < RING ? e + X : e + X - RING);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(X * N_D) : "memory");  // ids of b + P grid landed
    issue_data(b + P * grid, sl + P < NSLOT ? sl + P : sl + P - NSLOT, e);
    e = e + 1 < RING ? e + 1 : 0;

    const float* sp = slot0 + sl * SLOT_F;
    const float* sdp = FDP ? dpl : sp;
    const float* sal = sp + 128;
    const float* sU = sp + 256;
    const unsigned char* img = reinterpret_cast<const unsigned char*>(sp + 512);
    if constexpr (FDP) {  // dpooled[c] = iv g (sum_j da1[j] W1p[j][c] - sb - xhat sg), xhat = (pooled - m) iv
      if (tid < D) {
        const float* da1s = sp + 192;
        float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
#pragma unroll
        for (int j = 0; j < 32; j += 4) {
          c0 = fmaf(da1s[j], w1p[j * D + tid], c0);
          c1 = fmaf(da1s[j + 1], w1p[(j + 1) * D + tid], c1);
          c2 = fmaf(da1s[j + 2], w1p[(j + 2) * D + tid], c2);
          c3 = fmaf(da1s[j + 3], w1p[(j + 3) * D + tid], c3);
        }
        const float acc = (c0 + c1) + (c2 + c3);
        const float m = colc[tid], iv = colc[D + tid], gw = colc[2 * D + tid];
        const float xhat = (sp[tid] - m) * iv;
        dpl[tid] = iv * gw * (acc - colc[3 * D + tid] - xhat * colc[4 * D + tid]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    {  // dalpha[row] = dpooled . K[row], split over the waves: wave w owns rows [w R, (w+1) R)
      constexpr int R = LP / 8, LPR = 64 / R, CH = CPR / LPR;
      const int row = w * R + lane / LPR, part = lane % LPR;
      float acc = 0.f;
#pragma unroll
      for (int ch = 0; ch < CH; ++ch) {
        const int cc = part * CH + ch;
        const uint4 kv = *reinterpret_cast<const uint4*>(img + row * 2 * D + 16 * (cc ^ kswz<CPR>(row)));
        const float4 d0 = *reinterpret_cast<const float4*>(sdp + 8 * cc);
        const float4 d1 = *reinterpret_cast<const float4*>(sdp + 8 * cc + 4);
        acc = fmaf(d0.x, __uint_as_float(kv.x << 16), acc);
        acc = fmaf(d0.y, __uint_as_float(kv.x & 0xFFFF0000u), acc);
        acc = fmaf(d0.z, __uint_as_float(kv.y << 16), acc);
        acc = fmaf(d0.w, __uint_as_float(kv.y & 0xFFFF0000u), acc);
        acc = fmaf(d1.x, __uint_as_float(kv.z << 16), acc);
        acc = fmaf(d1.y, __uint_as_float(kv.z & 0xFFFF0000u), acc);
        acc = fmaf(d1.z, __uint_as_float(kv.w << 16), acc);
        acc = fmaf(d1.w, __uint_as_float(kv.w & 0xFFFF0000u), acc);
      }
      acc = group_sum<LPR>(acc);
      if (part == 0) dabuf[row] = acc;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float du = 0.f;
    if (us < nsl && rg < NC) {
      const float un = sU[32 * us + r];
      float da[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) da[c] = dabuf[32 * c + r];
      float t = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int row = 32 * c + r;
        t += (row < L && h == 0) ? sal[row] * da[c] : 0.f;
      }
      const float cdot = wave_sum_fast(t);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int row = 32 * c + r;
        if (h == 0 && (c & 1) == rg) {
          const float ds = row < L ? sal[row] * (da[c] - cdot) : 0.f;
          dsbuf[row] = ds;
          if (us == 0) db2_acc += ds;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if ((c & 1) != rg) continue;
        f32x16 acc;
#pragma unroll
        for (int g = 0; g < 16; ++g) acc[g] = un;
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(img + KImg<true, D>::off(32 * c + r, 16 * s2 + 8 * h));
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, wf.f[s2], acc, 0, 0, 0);
        }
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
          for (int j = 0; j < 4; ++j) {  // v_cvt_pk_bf16_f32 (round to nearest even)
            const bf16x2_hw pk = {(__bf16)dz[8 * s + 2 * j], (__bf16)dz[8 * s + 2 * j + 1]};
            const uint32_t u = __builtin_bit_cast(uint32_t, pk);
            af[2 * j] = (short)(u & 0xFFFF);
            af[2 * j + 1] = (short)(u >> 16);
          }
          const int grp = lane >> 4, i16 = lane & 15;
          const int rowq = 32 * c + 16 * s + 4 * h + (i16 >> 2);
#pragma unroll
          for (int cc = 0; cc < NCT; ++cc) {
            const int col = 32 * cc + 16 * (grp & 1) + 4 * (i16 & 3);
            typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
            const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + KImg<true, D>::off(rowq, col)));
            const bf16x4 hi =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + KImg<true, D>::off(rowq + 8, col)));
            const bf16x8 bfr = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
            dw[cc] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, dw[cc], 0, 0, 0);
          }
        }
      }
      du = half_swap_sum(du);
      db1_acc += du;
    }
    if constexpr (FQ) {  // stage this sample's dU rows (both row groups) and query row
      if (h == 0 && us < nsl && it < 16) dul[it * 256 + rg * 128 + 32 * us + r] = du;
      if (lane < 16 && it < 16) ql[it * 128 + 16 * w + lane] = sp[384 + 16 * w + lane];
    }
    ++it;
    du_keep = du;
    b_keep = b;
    sl = sl == NSLOT - 1 ? 0 : sl + 1;
  }
  store_du();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup exits
  if constexpr (FQ) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (it > 0) flush_q(it);
    else if (us < nsl) {  // no sample: a zero dW1q partial
      for (int i = lane; i < 32 * D; i += 64) sqs_slab[(size_t)(32 * us) * D + i] = 0.f;
    }
  }
  // combine the row-group pairs (rg 1 into rg 0, fixed order) through LDS
  float* xch = slot0;  // [4 unit slices][32][D] f32, reused for dW1k then dW1q
  const bool act = us < nsl;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (rg == 1 && act) {
#pragma unroll
    for (int c = 0; c < NCT; ++c)
#pragma unroll
      for (int g = 0; g < 16; ++g) xch[(size_t)(32 * us + acc_row(g, h)) * D + 32 * c + r] = dw[c][g];
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (rg == 0 && act) {
#pragma unroll
    for (int c = 0; c < NCT; ++c)
#pragma unroll
      for (int g = 0; g < 16; ++g) dw[c][g] += xch[(size_t)(32 * us + acc_row(g, h)) * D + 32 * c + r];
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  float* xs = slot0 + 4 * 32 * D;  // [4][32] dw2, [4][32] db1, [1] db2 of the rg = 1 waves
  {
    const float t2 = dw2_acc + __shfl_xor(dw2_acc, 32, 64);
    const float tb2 = wave_sum(db2_acc);
    if (rg == 1 && act && h == 0) {
      xs[32 * us + r] = t2;
      xs[128 + 32 * us + r] = db1_acc;
    }
    if (rg == 1 && us == 0 && lane == 0) xs[256] = tb2;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float* slab = slabs + (size_t)blockIdx.x * slab_floats(A, D);
    if (rg == 0 && act) {
      float* sqs = slab + slab_q_off(A, D);
#pragma unroll
      for (int c = 0; c < NCT; ++c)
#pragma unroll
        for (int g = 0; g < 16; ++g) slab[(size_t)(32 * us + acc_row(g, h)) * D + 32 * c + r] = dw[c][g];
      if (h == 0) {
        slab[(size_t)A * D + 32 * us + r] = t2 + xs[32 * us + r];
        sqs[(size_t)A * D + 32 * us + r] = db1_acc + xs[128 + 32 * us + r];
      }
    }
    if (rg == 0 && us == 0 && lane == 0) slab[(size_t)A * D + A] = tb2 + xs[256];
  }
}

// Two-stream form of the head-fused 8-wave backward (FQ + FDP, LP <= 64): the
// workgroup's samples alternate between two groups of four waves (g = w >> 2),
// each group runs ONE sample per iteration with all four waves (us = w & 3: 32
// attention units each, every row tile of the sample), so one barrier-separated
// iteration advances two samples and a sample whose second row tile holds only
// zero keys (padding, rows >= L) costs its group one tile, not a partner wave's
// idle tile.  The per-group dW1k / dw2 / db1 accumulators meet in a fixed order
// at the end, as the row-group pairs of din_bwd_deep8_kernel do.
template <int D, int LP>
__global__ __launch_bounds__(512, 1) void din_bwd_deep8g_kernel(
    const uint16_t* __restrict__ table, const int32_t* __restrict__ ids, int64_t n_table, const float* __restrict__ U,
    const uint16_t* __restrict__ W1k, const float* __restrict__ w2, int B, int L, int A,
    const float* __restrict__ alpha, float* __restrict__ slabs, const float* __restrict__ q, int dq, DpSrc dps) {
  constexpr int CPR = D / 8, KS = D / 16, NCT = D / 32, NC = LP / 32;
  constexpr int NPW = LP * CPR / 256;  // key-image DMA pieces per wave (four waves per sample)
  static_assert(LP <= 64 && NPW >= 1, "deep8g: LP <= 64, L D >= 2048");
  constexpr int N_D = NPW + 2 + 1;     // per wave and iteration: keys, two small pieces, ids
  constexpr int NSLOT = 3, P = NSLOT - 1, X = 3, RING = X + 1;
  static_assert(X * N_D < 64, "vmcnt range");
  // slot (floats): pooled [128] | alpha [64], da1 [32..] | U [128] | q [128] | key image [LP][D] bf16
  constexpr int SLOT_F = 4 * 128 + LP * D / 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int us = w & 3, g = w >> 2, gt = tid & 255;
  const int nsl = A >> 5;
  float* slot0 = reinterpret_cast<float*>(smem) + g * NSLOT * SLOT_F;  // this group's slots
  int32_t* const ring0 = reinterpret_cast<int32_t*>(reinterpret_cast<float*>(smem) + 2 * NSLOT * SLOT_F);
  int32_t* idring = ring0 + w * RING * 64;                                  // [RING][64] per wave
  float* dsbuf = reinterpret_cast<float*>(ring0 + 8 * RING * 64) + w * 64;  // [64] per wave
  float* dabuf = reinterpret_cast<float*>(ring0 + 8 * RING * 64) + 8 * 64 + g * 64;  // [64] per group
  float* dul = reinterpret_cast<float*>(ring0 + 8 * RING * 64) + 8 * 64 + 2 * 64;    // [16][128] dU rows
  float* ql = dul + 16 * 128;                                                        // [16][128] query rows
  float* dpl = ql + 16 * 128;                                                        // [2 groups][D]
  float* w1p = dpl + 2 * D;                                                          // [32][D] fc.1 pooled half
  float* colc = w1p + 32 * D;                                                        // [5][D]
  for (int i = tid; i < 32 * D; i += 512) w1p[i] = dps.w1[(size_t)(i / D) * 2 * D + D + i % D];
  for (int c = tid; c < D; c += 512) {
    colc[c] = dps.stat0[D + c];
    colc[D + c] = dps.stat0[3 * D + c];
    colc[2 * D + c] = dps.bn0w[D + c];
    colc[3 * D + c] = (float)dps.sum5[D + c] * dps.invB;
    colc[4 * D + c] = (float)dps.sum5[3 * D + c] * dps.invB;
  }
  WFrag<true, D> wf;
  const int wu = us < nsl ? us : 0;
  wf.load(W1k, 32 * wu + r, h);
  const float w2n = w2[32 * wu + r];
  f32x16 dw[NCT];
#pragma unroll
  for (int c = 0; c < NCT; ++c)
#pragma unroll
    for (int gg = 0; gg < 16; ++gg) dw[c][gg] = 0.f;
  float dw2_acc = 0.f, db2_acc = 0.f, db1_acc = 0.f;
  float* const sqs_slab = slabs + (size_t)blockIdx.x * slab_floats(A, D) + slab_q_off(A, D);

  // this wave's two small pieces of [pooled0, pooled1, alpha, da1, u0, u1, q0, q1]: kind us
  const float* const sbase = us == 0 ? dps.pooled : us == 2 ? U : q;
  const int sstride = us == 0 ? D : us == 2 ? A : dq;
  uint32_t zmask = 0;  // per slot 2 bits: row tile c holds only zero keys (z = U, no dW1k term)
  auto issue_ids = [&](int64_t b, int e) {
    const int64_t bc = b < B ? b : 0;
    const int i = lane < L ? lane : 0;
    glds4_asm(ids + bc * L + i, lds_u32(idring + e * 64));
  };
  auto issue_data = [&](int64_t b, int sl, int e) {
    float* sp = slot0 + sl * SLOT_F;
    uint16_t* img = reinterpret_cast<uint16_t*>(sp + 4 * 128);
#pragma unroll
    for (int k = 0; k < NPW; ++k) {
      const int u = us + 4 * k;
      const int p = u * 64 + lane;
      const int row = p / CPR, pc = p % CPR;
      const int cc = pc ^ kswz<CPR>(row);
      const int32_t idv0 = idring[e * 64 + row];
      const int32_t idr = row < L && b < B ? idv0 : -1;
      const uint16_t* src = (idr >= 0 && idr < n_table) ? table + (int64_t)idr * D + cc * 8 : zero_row(b, row) + cc * 8;
      glds16_asm(src, lds_u32(img + u * 64 * 8));
    }
    const int64_t bc = b < B ? b : 0;
    if (us == 1) {  // alpha [L], da1 [32]
      glds4_asm(alpha + bc * L + (lane < L ? lane : 0), lds_u32(sp + 128));
      glds4_asm(dps.da1 + bc * 32 + (lane < 32 ? lane : 0), lds_u32(sp + 192));
    } else {
#pragma unroll
      for (int part = 0; part < 2; ++part) {
        const int i = part * 64 + lane;
        glds4_asm(sbase + bc * sstride + (i < sstride ? i : 0), lds_u32(sp + us * 128 + part * 64));
      }
    }
    const int32_t idl = idring[e * 64 + lane];
    const uint64_t vm = __ballot(lane < L && b < B && idl >= 0 && idl < n_table);
    const uint32_t zb = ((uint32_t)vm == 0u ? 1u : 0u) | ((uint32_t)(vm >> 32) == 0u ? 2u : 0u);
    zmask = (zmask & ~(3u << (2 * sl))) | (zb << (2 * sl));
  };

  const int64_t grid = gridDim.x;
  const int64_t b0 = blockIdx.x;
  const int ns_wg = b0 < B ? (int)((B - b0 + grid - 1) / grid) : 0;  // samples of this workgroup
  const int n_it = (ns_wg + 1) >> 1;
  auto sample = [&](int j) { return b0 + (int64_t)(2 * j + g) * grid; };  // group g's j-th sample
#pragma unroll
  for (int k = 0; k < X; ++k) issue_ids(sample(k), k);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int k = 0; k < P; ++k) {
    issue_ids(sample(k + X), (k + X) % RING);
    issue_data(sample(k), k, k);
  }
  int sl = 0, e = P % RING;  // e: ring entry holding the ids of sample(j + P)
  for (int j = 0; j < n_it; ++j) {
    // this wave's DMA group of sample(j) landed; all waves' after the barrier; slot of sample(j - 1) is free
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"((P - 1) * N_D) : "memory");
    issue_ids(sample(j + P + X), e + X < RING ? e + X : e + X - RING);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(X * N_D) : "memory");  // ids of sample(j + P) landed
    issue_data(sample(j + P), sl + P < NSLOT ? sl + P : sl + P - NSLOT, e);
    e = e + 1 < RING ? e + 1 : 0;

    const int64_t bs = sample(j);
    const bool act = bs < B;  // group 1 may run past the workgroup's last sample
    const float* sp = slot0 + sl * SLOT_F;
    const float* sal = sp + 128;
    const float* sU = sp + 256;
    const unsigned char* img = reinterpret_cast<const unsigned char*>(sp + 512);
    float* sdp = dpl + g * D;
    if (gt < D) {  // dpooled[c] = iv g (sum_j da1[j] W1p[j][c] - sb - xhat sg), xhat = (pooled - m) iv
      const float* da1s = sp + 192;
      float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
#pragma unroll
      for (int jj = 0; jj < 32; jj += 4) {
        c0 = fmaf(da1s[jj], w1p[jj * D + gt], c0);
        c1 = fmaf(da1s[jj + 1], w1p[(jj + 1) * D + gt], c1);
        c2 = fmaf(da1s[jj + 2], w1p[(jj + 2) * D + gt], c2);
        c3 = fmaf(da1s[jj + 3], w1p[(jj + 3) * D + gt], c3);
      }
      const float acc = (c0 + c1) + (c2 + c3);
      const float m = colc[gt], iv = colc[D + gt], gw = colc[2 * D + gt];
      const float xhat = (sp[gt] - m) * iv;
      sdp[gt] = iv * gw * (acc - colc[3 * D + gt] - xhat * colc[4 * D + gt]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    {  // dalpha[row] = dpooled . K[row]: wave us of the group owns rows [us R, (us+1) R)
      constexpr int R = LP / 4, LPR = 64 / R, CH = CPR / LPR;
      const int row = us * R + lane / LPR, part = lane % LPR;
      float acc = 0.f;
#pragma unroll
      for (int ch = 0; ch < CH; ++ch) {
        const int cc = part * CH + ch;
        const uint4 kv = *reinterpret_cast<const uint4*>(img + row * 2 * D + 16 * (cc ^ kswz<CPR>(row)));
        const float4 d0 = *reinterpret_cast<const float4*>(sdp + 8 * cc);
        const float4 d1 = *reinterpret_cast<const float4*>(sdp + 8 * cc + 4);
        acc = fmaf(d0.x, __uint_as_float(kv.x << 16), acc);
        acc = fmaf(d0.y, __uint_as_float(kv.x & 0xFFFF0000u), acc);
        acc = fmaf(d0.z, __uint_as_float(kv.y << 16), acc);
        acc = fmaf(d0.w, __uint_as_float(kv.y & 0xFFFF0000u), acc);
        acc = fmaf(d1.x, __uint_as_float(kv.z << 16), acc);
        acc = fmaf(d1.y, __uint_as_float(kv.z & 0xFFFF0000u), acc);
        acc = fmaf(d1.z, __uint_as_float(kv.w << 16), acc);
        acc = fmaf(d1.w, __uint_as_float(kv.w & 0xFFFF0000u), acc);
      }
      acc = group_sum<LPR>(acc);
      if (part == 0) dabuf[row] = acc;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float du = 0.f;
    if (act && us < nsl) {
      const float un = sU[32 * us + r];
      float da[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) da[c] = dabuf[32 * c + r];
      float t = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int row = 32 * c + r;
        t += (row < L && h == 0) ? sal[row] * da[c] : 0.f;
      }
      const float cdot = wave_sum_fast(t);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int row = 32 * c + r;
        if (h == 0) {
          const float ds = row < L ? sal[row] * (da[c] - cdot) : 0.f;
          dsbuf[row] = ds;
          if (us == 0) db2_acc += ds;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 1
      for (int c = 0; c < NC; ++c) {  // (not unrolled: the two tiles' registers would overlap)
        const bool kz = (zmask >> (2 * sl + c)) & 1u;  // zero keys: z = U exactly, no dW1k term
        f32x16 acc;
#pragma unroll
        for (int gg = 0; gg < 16; ++gg) acc[gg] = un;
        if (!kz) {
#pragma unroll
          for (int s2 = 0; s2 < KS; ++s2) {
            const bf16x8 kf = *reinterpret_cast<const bf16x8*>(img + KImg<true, D>::off(32 * c + r, 16 * s2 + 8 * h));
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, wf.f[s2], acc, 0, 0, 0);
          }
        }
        f32x16 dz;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float4 d4 = *reinterpret_cast<const float4*>(dsbuf + 32 * c + 8 * jj + 4 * h);
          const float dsv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
          for (int i2 = 0; i2 < 4; ++i2) {
            const int gg = 4 * jj + i2;
            const float z = acc[gg];
            dw2_acc = fmaf(dsv[i2], fmaxf(z, 0.f), dw2_acc);
            const float v = z > 0.f ? dsv[i2] * w2n : 0.f;
            dz[gg] = v;
            du += v;
          }
        }
        if (kz) continue;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 af;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {  // v_cvt_pk_bf16_f32 (round to nearest even)
            const bf16x2_hw pk = {(__bf16)dz[8 * s + 2 * jj], (__bf16)dz[8 * s + 2 * jj + 1]};
            const uint32_t u = __builtin_bit_cast(uint32_t, pk);
            af[2 * jj] = (short)(u & 0xFFFF);
            af[2 * jj + 1] = (short)(u >> 16);
          }
          const int grp = lane >> 4, i16 = lane & 15;
          const int rowq = 32 * c + 16 * s + 4 * h + (i16 >> 2);
#pragma unroll
          for (int cc = 0; cc < NCT; ++cc) {
            const int col = 32 * cc + 16 * (grp & 1) + 4 * (i16 & 3);
            typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
            const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + KImg<true, D>::off(rowq, col)));
            const bf16x4 hi =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + KImg<true, D>::off(rowq + 8, col)));
            const bf16x8 bfr = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
            dw[cc] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, dw[cc], 0, 0, 0);
          }
        }
      }
      du = half_swap_sum(du);
      db1_acc += du;
    }
    {  // stage this sample's dU row and query row (sample index 2 j + g of the workgroup; host: <= 16)
      const int si = 2 * j + g;
      if (act && si < 16) {
        if (h == 0 && us < nsl) dul[si * 128 + 32 * us + r] = du;
        if (lane < 32) ql[si * 128 + 32 * us + lane] = sp[384 + 32 * us + lane];
      }
    }
    sl = sl == NSLOT - 1 ? 0 : sl + 1;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");  // no LDS-DMA lands after this
  {  // dW1q partial of the staged samples: wave (us, g) owns tiles n = 32 us.., k = 32 (g + 2 jj)..
    const int ns = ns_wg < 16 ? ns_wg : 16;
    if (us < nsl) {
#pragma unroll
      for (int jj = 0; jj < (NCT + 1) / 2; ++jj) {
        const int tk = g + 2 * jj;
        if (tk >= NCT) continue;
        f32x16 acc;
#pragma unroll
        for (int gg = 0; gg < 16; ++gg) acc[gg] = 0.f;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const int sm = 2 * kk + h;
          const float av = sm < ns ? dul[sm * 128 + 32 * us + r] : 0.f;
          const float bv = sm < ns ? ql[sm * 128 + 32 * tk + r] : 0.f;
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
        }
#pragma unroll
        for (int gg = 0; gg < 16; ++gg) sqs_slab[(size_t)(32 * us + acc_row(gg, h)) * D + 32 * tk + r] = acc[gg];
      }
    }
  }
  // combine the groups (g 1 into g 0, fixed order) through LDS
  float* xch = reinterpret_cast<float*>(smem);  // [4 unit slices][32][D] f32
  const bool wact = us < nsl;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (g == 1 && wact) {
#pragma unroll
    for (int c = 0; c < NCT; ++c)
#pragma unroll
      for (int gg = 0; gg < 16; ++gg) xch[(size_t)(32 * us + acc_row(gg, h)) * D + 32 * c + r] = dw[c][gg];
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (g == 0 && wact) {
#pragma unroll
    for (int c = 0; c < NCT; ++c)
#pragma unroll
      for (int gg = 0; gg < 16; ++gg) dw[c][gg] += xch[(size_t)(32 * us + acc_row(gg, h)) * D + 32 * c + r];
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  float* xs = xch + 4 * 32 * D;  // [4][32] dw2, [4][32] db1, [1] db2 of group 1
  {
    const float t2 = half_swap_sum(dw2_acc);
    const float tb2 = wave_sum_fast(db2_acc);
    if (g == 1 && wact && h == 0) {
      xs[32 * us + r] = t2;
      xs[128 + 32 * us + r] = db1_acc;
    }
    if (g == 1 && us == 0 && lane == 0) xs[256] = tb2;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float* slab = slabs + (size_t)blockIdx.x * slab_floats(A, D);
    if (g == 0 && wact) {
      float* sqs = slab + slab_q_off(A, D);
#pragma unroll
      for (int c = 0; c < NCT; ++c)
#pragma unroll
        for (int gg = 0; gg < 16; ++gg) slab[(size_t)(32 * us + acc_row(gg, h)) * D + 32 * c + r] = dw[c][gg];
      if (h == 0) {
        slab[(size_t)A * D + 32 * us + r] = t2 + xs[32 * us + r];
        sqs[(size_t)A * D + 32 * us + r] = db1_acc + xs[128 + 32 * us + r];
      }
    }
    if (g == 0 && us == 0 && lane == 0) slab[(size_t)A * D + A] = tb2 + xs[256];
  }
}

// D = 256 variant of the 8-wave backward (the reference's training width):
// waves w and w + 4 own the same 32 units (us = w & 3) and split the 256
// COLUMNS (ch = w >> 2 takes [128 ch, 128 ch + 128)) instead of the rows, so
// each keeps the d = 128 register budget (W1k fragments of its half, dW1k
// accumulators of its half).  z needs the full 256-term reduction: each wave
// forms its half's partial z of both row tiles on MFMA, the partials meet in
// LDS (summed ch 0 + ch 1 in that order by both waves, so both hold the same
// z), then both form dz and accumulate dW1k for their columns; the ch = 0 wave
// also accumulates dw2, db1 and the sample's dU row (its partner stores zeros
// in the second dU half the dW1q kernel adds).  Small pieces per sample:
// dpooled [256] (4 pieces), alpha [LP <= 64] (1), U [128] (2), one unused.
//
// SPLIT (histories of 65..128 rows, LP = 64): every sample runs as two
// half-samples (rows [0, 64) and [64, L)).  Past the softmax the backward is
// row-local, so the halves only share the softmax term cdot = sum_l alpha_l
// dalpha_l, which din_cdot_kernel forms beforehand (cdv[b], loaded into the
// alpha slot's second half by the otherwise unused small piece); half h's dU
// row goes to dUp[h] (the dW1q kernel adds both), its other partials to the
// same accumulators as any sample's.
template <int D, int LP, int NSLOT, bool SPLIT = false>
__global__ __launch_bounds__(512, 1) void din_bwd_deep8c_kernel(
    const uint16_t* __restrict__ table, const int32_t* __restrict__ ids, int64_t n_table, const float* __restrict__ U,
    const uint16_t* __restrict__ W1k, const float* __restrict__ w2, int B, int L, int A,
    const float* __restrict__ dpooled, const float* __restrict__ alpha, float* __restrict__ slabs,
    float* __restrict__ dUp, float* __restrict__ dummy, const float* __restrict__ cdv = nullptr) {
  static_assert(D == 256 && LP <= 64 && (!SPLIT || LP == 64), "deep8c: D = 256, LP <= 64 (SPLIT: 64)");
  constexpr int DH = D / 2;
  constexpr int CPR = D / 8, KSH = DH / 16, NCTH = DH / 32, NC = LP / 32;
  constexpr int NPW = LP * CPR / 512;  // key-image DMA pieces per wave
  constexpr int N_D = 1 + NPW + 1 + 1;  // per wave and iteration: the dU store, keys, one small piece, ids
  constexpr int P = NSLOT - 1;
  constexpr int X = P > 3 ? P : 3, RING = X + 1;
  static_assert(NPW >= 1 && P >= 2 && P <= X && X * N_D < 64, "vmcnt range");
  // slot (floats): dpooled [256] | alpha [128] | U [128] | key image [LP][D] bf16
  constexpr int SLOT_F = 4 * 128 + LP * D / 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int us = w & 3, ch = w >> 2;
  const int nsl = A >> 5;
  float* slot0 = reinterpret_cast<float*>(smem);
  int32_t* idring = reinterpret_cast<int32_t*>(slot0 + NSLOT * SLOT_F) + w * RING * 64;  // [RING][64] per wave
  float* dsbuf = reinterpret_cast<float*>(reinterpret_cast<int32_t*>(slot0 + NSLOT * SLOT_F) + 8 * RING * 64) + w * 64;
  float* dabuf = reinterpret_cast<float*>(reinterpret_cast<int32_t*>(slot0 + NSLOT * SLOT_F) + 8 * RING * 64) + 8 * 64;
  float* xz = dabuf + 64;  // [4 unit slices][2 halves][1024] partial z of one row tile, lane-major
  float* xzw = xz + (size_t)(us * 2 + ch) * 1024;
  const float* xz0 = xz + (size_t)(us * 2) * 1024;
  const float* xz1 = xz + (size_t)(us * 2 + 1) * 1024;

  const int wu = us < nsl ? us : 0;
  bf16x8 wf[KSH];
  {
    const uint16_t* p = W1k + (int64_t)(32 * wu + r) * D + DH * ch + 8 * h;
#pragma unroll
    for (int s2 = 0; s2 < KSH; ++s2) wf[s2] = *reinterpret_cast<const bf16x8*>(p + 16 * s2);
  }
  const float w2n = w2[32 * wu + r];
#pragma unroll
  for (int s2 = 0; s2 < KSH; ++s2) asm volatile("" ::"v"(wf[s2]));
  asm volatile("" ::"v"(w2n));
  f32x16 dw[NCTH];
#pragma unroll
  for (int c = 0; c < NCTH; ++c)
#pragma unroll
    for (int g = 0; g < 16; ++g) dw[c][g] = 0.f;
  float dw2_acc = 0.f, db2_acc = 0.f, db1_acc = 0.f;
  float du_keep = 0.f;
  int64_t b_keep = -1;
  float* const dmy = dummy + (size_t)blockIdx.x * 512 + tid;
  // work items: samples, or (SPLIT) half-samples v -> sample v >> 1, rows [64 (v & 1), ...)
  const int64_t NV = SPLIT ? 2 * (int64_t)B : B;
  auto rows_of = [&](int64_t v) { return SPLIT ? min(LP, L - 64 * (int)(v & 1)) : L; };
  auto row0_of = [&](int64_t v) { return SPLIT ? 64 * (int)(v & 1) : 0; };
  auto store_du = [&]() {  // half ch of dUp: the ch = 0 wave's full row sum, zeros from ch = 1
    const int64_t bs = SPLIT ? b_keep >> 1 : b_keep;
    const int part = SPLIT ? (int)(b_keep & 1) : ch;
    float* dst = (b_keep >= 0 && us < nsl && h == 0 && (!SPLIT || ch == 0))
                     ? dUp + ((size_t)part * B + bs) * A + 32 * us + r : dmy;
    const float v = ch == 0 ? du_keep : 0.f;
    asm volatile("global_store_dword %0, %1, off" ::"v"(dst), "v"(v) : "memory");
  };
  auto issue_ids = [&](int64_t b, int e) {
    const int64_t vc = b < NV ? b : 0;
    const int64_t bc = SPLIT ? vc >> 1 : vc;
    const int le = rows_of(vc), r0 = row0_of(vc);
    const int i = lane < LP ? lane : 0;
    glds4_asm(ids + bc * L + r0 + (i < le ? i : 0), lds_u32(idring + e * 64));
  };
  auto issue_data = [&](int64_t b, int sl, int e) {
    const int64_t vc = b < NV ? b : 0;
    const int le = rows_of(vc), r0 = row0_of(vc);
    float* sp = slot0 + sl * SLOT_F;
    uint16_t* img = reinterpret_cast<uint16_t*>(sp + 4 * 128);
#pragma unroll
    for (int k = 0; k < NPW; ++k) {
      const int u = w + 8 * k;
      const int p = u * 64 + lane;
      const int row = p / CPR, pc = p % CPR;
      const int cc = pc ^ kswz<CPR>(row);
      const int32_t idv0 = idring[e * 64 + row];
      const int32_t idr = row < le && b < NV ? idv0 : -1;
      const uint16_t* src = (idr >= 0 && idr < n_table) ? table + (int64_t)idr * D + cc * 8 : zero_row(b, row) + cc * 8;
      glds16_asm(src, lds_u32(img + u * 64 * 8));
    }
    const int64_t bc = SPLIT ? vc >> 1 : vc;
    {  // small piece w of [dp0, dp1, dp2, dp3, al0, u0, u1, (u1 again: unused slot | SPLIT: cdot)]
      const float* base;
      int i, lim;
      float* dst;
      if (w < 4) { base = dpooled + bc * D; i = 64 * w + lane; lim = D; dst = sp + 64 * w; }
      else if (w == 4) { base = alpha + bc * L + r0; i = lane; lim = le; dst = sp + 256; }
      else { base = U + bc * A; i = 64 * ((w - 5) & 1) + lane; lim = A; dst = sp + 384 + 64 * ((w - 5) & 1); }
      if (w == 7) dst = sp + 320;  // the alpha slot's unused second half (LP <= 64)
      if (SPLIT && w == 7) { base = cdv + bc; i = 0; lim = 1; }
      glds4_asm(base + (i < lim ? i : 0), lds_u32(dst));
    }
  };

  const int64_t grid = gridDim.x;
  int64_t b = blockIdx.x;
#pragma unroll
  for (int k = 0; k < X; ++k) issue_ids(b + k * grid, k);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int k = 0; k < P; ++k) {
    store_du();
    issue_ids(b + (k + X) * grid, (k + X) % RING);
    issue_data(b + k * grid, k, k);
  }
  int sl = 0, e = P % RING;
  for (; b < NV; b += grid) {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"((P - 1) * N_D) : "memory");
    store_du();
    issue_ids(b + (P + X) * grid, e + X < RING ? e + X : e + X - RING);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(X * N_D) : "memory");
    issue_data(b + P * grid, sl + P < NSLOT ? sl + P : sl + P - NSLOT, e);
    e = e + 1 < RING ? e + 1 : 0;

    const float* sp = slot0 + sl * SLOT_F;
    const float* sdp = sp;
    const float* sal = sp + 256;
    const float* sU = sp + 384;
    const unsigned char* img = reinterpret_cast<const unsigned char*>(sp + 512);
    const int Le = rows_of(b);
    {  // dalpha[row] = dpooled . K[row]: wave w owns rows [w R, (w+1) R)
      constexpr int R = LP / 8, LPR = 64 / R, CHK = CPR / LPR;
      const int row = w * R + lane / LPR, part = lane % LPR;
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < CHK; ++k) {
        const int cc = part * CHK + k;
        const uint4 kv = *reinterpret_cast<const uint4*>(img + row * 2 * D + 16 * (cc ^ kswz<CPR>(row)));
        const float4 d0 = *reinterpret_cast<const float4*>(sdp + 8 * cc);
        const float4 d1 = *reinterpret_cast<const float4*>(sdp + 8 * cc + 4);
        acc = fmaf(d0.x, __uint_as_float(kv.x << 16), acc);
        acc = fmaf(d0.y, __uint_as_float(kv.x & 0xFFFF0000u), acc);
        acc = fmaf(d0.z, __uint_as_float(kv.y << 16), acc);
        acc = fmaf(d0.w, __uint_as_float(kv.y & 0xFFFF0000u), acc);
        acc = fmaf(d1.x, __uint_as_float(kv.z << 16), acc);
        acc = fmaf(d1.y, __uint_as_float(kv.z & 0xFFFF0000u), acc);
        acc = fmaf(d1.z, __uint_as_float(kv.w << 16), acc);
        acc = fmaf(d1.w, __uint_as_float(kv.w & 0xFFFF0000u), acc);
      }
      acc = group_sum<LPR>(acc);
      if (part == 0) dabuf[row] = acc;
    }
    // partial z of this half's columns for row tile c (MFMA), exchanged through LDS
    auto zpart = [&](int c) {
      f32x16 acc;
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[g] = 0.f;
#pragma unroll
      for (int s2 = 0; s2 < KSH; ++s2) {
        const bf16x8 kf =
            *reinterpret_cast<const bf16x8*>(img + KImg<true, D>::off(32 * c + r, DH * ch + 16 * s2 + 8 * h));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, wf[s2], acc, 0, 0, 0);
      }
      return acc;
    };
    auto zput = [&](const f32x16& acc) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<float4*>(xzw + j * 256 + 4 * lane) =
            make_float4(acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3]);
    };
    zput(zpart(0));
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // dalpha and both halves' partial z
    float du = 0.f;
    {  // every wave runs the tile loop (its barriers); a wave without units (A < 128) stores nothing
      const float un = sU[32 * wu + r];
      float da[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) da[c] = dabuf[32 * c + r];
      float t = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int row = 32 * c + r;
        t += (row < Le && h == 0) ? sal[row] * da[c] : 0.f;
      }
      const float cdot = SPLIT ? sal[64] : wave_sum_fast(t);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int row = 32 * c + r;
        if (h == 0) {
          const float ds = row < Le ? sal[row] * (da[c] - cdot) : 0.f;
          dsbuf[row] = ds;
          if (w == 0) db2_acc += ds;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (c > 0) {  // every partner has read tile c - 1's partial: publish tile c's
          const f32x16 zp = zpart(c);
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
          zput(zp);
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        f32x16 dz;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 p0 = *reinterpret_cast<const float4*>(xz0 + j * 256 + 4 * lane);
          const float4 p1 = *reinterpret_cast<const float4*>(xz1 + j * 256 + 4 * lane);
          const float4 d4 = *reinterpret_cast<const float4*>(dsbuf + 32 * c + 8 * j + 4 * h);
          const float zz[4] = {un + (p0.x + p1.x), un + (p0.y + p1.y), un + (p0.z + p1.z), un + (p0.w + p1.w)};
          const float dsv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int g = 4 * j + i;
            const float z = zz[i];
            if (ch == 0) dw2_acc = fmaf(dsv[i], fmaxf(z, 0.f), dw2_acc);
            const float v = z > 0.f ? dsv[i] * w2n : 0.f;
            dz[g] = v;
            du += v;
          }
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 af, afl;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bf16x2_hw pk = {(__bf16)dz[8 * s + 2 * j], (__bf16)dz[8 * s + 2 * j + 1]};
            const uint32_t u = __builtin_bit_cast(uint32_t, pk);
            af[2 * j] = (short)(u & 0xFFFF);
            af[2 * j + 1] = (short)(u >> 16);
            if constexpr (SPLIT) {  // dz as bf16 hi + lo: 96..128 rows of bf16 dz round past 2e-3 of dW1k
              const bf16x2_hw pl = {(__bf16)(dz[8 * s + 2 * j] - (float)pk[0]),
                                    (__bf16)(dz[8 * s + 2 * j + 1] - (float)pk[1])};
              const uint32_t ul = __builtin_bit_cast(uint32_t, pl);
              afl[2 * j] = (short)(ul & 0xFFFF);
              afl[2 * j + 1] = (short)(ul >> 16);
            }
          }
          const int grp = lane >> 4, i16 = lane & 15;
          const int rowq = 32 * c + 16 * s + 4 * h + (i16 >> 2);
#pragma unroll
          for (int cc = 0; cc < NCTH; ++cc) {
            const int col = DH * ch + 32 * cc + 16 * (grp & 1) + 4 * (i16 & 3);
            typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
            const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + KImg<true, D>::off(rowq, col)));
            const bf16x4 hi =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + KImg<true, D>::off(rowq + 8, col)));
            const bf16x8 bfr = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
            dw[cc] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, dw[cc], 0, 0, 0);
            if constexpr (SPLIT) dw[cc] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afl, bfr, dw[cc], 0, 0, 0);
          }
        }
      }
      du = half_swap_sum(du);
      if (ch == 0) db1_acc += du;
    }
    du_keep = du;
    b_keep = b;
    sl = sl == NSLOT - 1 ? 0 : sl + 1;
  }
  store_du();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup exits
  float* slab = slabs + (size_t)blockIdx.x * slab_floats(A, D);
  if (us < nsl) {
#pragma unroll
    for (int c = 0; c < NCTH; ++c)
#pragma unroll
      for (int g = 0; g < 16; ++g) slab[(size_t)(32 * us + acc_row(g, h)) * D + DH * ch + 32 * c + r] = dw[c][g];
    const float t2 = dw2_acc + __shfl_xor(dw2_acc, 32, 64);
    if (ch == 0 && h == 0) {
      slab[(size_t)A * D + 32 * us + r] = t2;
      slab[slab_q_off(A, D) + (size_t)A * D + 32 * us + r] = db1_acc;
    }
  }
  if (w == 0) {
    const float tb2 = wave_sum(db2_acc);
    if (lane == 0) slab[(size_t)A * D + A] = tb2;
  }
}

// Softmax term of the SPLIT backward (d = 256, L 65..128): cd[b] = sum_l
// alpha[b][l] (dpooled[b] . K[b][l]) over the bf16 key rows (an invalid id is a
// zero row).  One wave per sample, a lane per 4 columns; the per-lane partial
// is linear in the rows, so the wave reduces once at the end.
template <int D>
__global__ __launch_bounds__(256) void din_cdot_kernel(const uint16_t* __restrict__ table,
                                                       const int32_t* __restrict__ ids, int64_t n_table,
                                                       const float* __restrict__ dpooled,
                                                       const float* __restrict__ alpha, int B, int L,
                                                       float* __restrict__ cd) {
  static_assert(D == 256, "din_cdot: D = 256");
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float4 dp = *reinterpret_cast<const float4*>(dpooled + b * D + 4 * lane);
  const int32_t id0 = lane < L ? ids[b * L + lane] : -1;
  const int32_t id1 = lane + 64 < L ? ids[b * L + 64 + lane] : -1;
  const float a0 = lane < L ? alpha[b * L + lane] : 0.f;
  const float a1 = lane + 64 < L ? alpha[b * L + 64 + lane] : 0.f;
  float t = 0.f;
#pragma unroll 8
  for (int l = 0; l < L; ++l) {
    const int32_t id = __builtin_amdgcn_readlane(l < 64 ? id0 : id1, l & 63);
    const float al = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(l < 64 ? a0 : a1), l & 63));
    const bool ok = id >= 0 && id < n_table;
    const uint2 kv = *reinterpret_cast<const uint2*>(table + (int64_t)(ok ? id : 0) * D + 4 * lane);
    float s = dp.x * __uint_as_float(kv.x << 16);
    s = fmaf(dp.y, __uint_as_float(kv.x & 0xFFFF0000u), s);
    s = fmaf(dp.z, __uint_as_float(kv.y << 16), s);
    s = fmaf(dp.w, __uint_as_float(kv.y & 0xFFFF0000u), s);
    t = fmaf(ok ? al : 0.f, s, t);
  }
  t = wave_sum(t);
  if (lane == 0) cd[b] = t;
}

// The same term from the forward's pooled rows: sum_l alpha_l (dp . k_l) =
// dp . (sum_l alpha_l k_l) = dp . pooled (equal up to the fp32 rounding of the
// two summation orders).  One wave per sample.
template <int D>
__global__ __launch_bounds__(256) void din_cdot_pooled_kernel(const float* __restrict__ dpooled,
                                                              const float* __restrict__ pooled, int B,
                                                              float* __restrict__ cd) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  float t = 0.f;
#pragma unroll
  for (int c = 0; c < D / 256; ++c) {
    const float4 x = *reinterpret_cast<const float4*>(dpooled + b * D + 256 * c + 4 * lane);
    const float4 y = *reinterpret_cast<const float4*>(pooled + b * D + 256 * c + 4 * lane);
    t = fmaf(x.x, y.x, fmaf(x.y, y.y, fmaf(x.z, y.z, fmaf(x.w, y.w, t))));
  }
  t = wave_sum(t);
  if (lane == 0) cd[b] = t;
}

// dW1q partial tiles for nrk_din_attn_bwd_params (8-wave backward):
//   part[kc][n][k] = sum over the samples b of chunk kc and both row groups
//   of dUp[rg][b][n] q[b][k], on f32 MFMA (lane half h = row group).
// grid (A/32 x D/32 tiles, KC chunks); 4 waves split a chunk's samples.
__global__ __launch_bounds__(256) void din_dwq_kernel(const float* __restrict__ dUp, const float* __restrict__ q, int B,
                                                      int A, int dq, int D, int kchunk, float* __restrict__ part) {
  __shared__ float red[4][32][33];
  const int nt = D / 32;
  const int tn = blockIdx.x / nt, tk = blockIdx.x % nt, kc = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 31, h = lane >> 5;
  f32x16 acc;
#pragma unroll
  for (int g = 0; g < 16; ++g) acc[g] = 0.f;
  const int b0 = kc * kchunk, b1 = min(B, b0 + kchunk);
  const int col = 32 * tk + i;
  const bool colok = col < dq;
  for (int bb = b0 + w; bb < b1; bb += 4 * 8) {
    float av[8], bv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int b = bb + 4 * u;
      const bool ok = b < b1;
      av[u] = ok ? dUp[((size_t)h * B + b) * A + 32 * tn + i] : 0.f;
      bv[u] = ok && colok ? q[(size_t)b * dq + col] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
  }
#pragma unroll
  for (int g = 0; g < 16; ++g) red[w][acc_row(g, h)][i] = acc[g];
  __syncthreads();
  for (int o = threadIdx.x; o < 32 * 32; o += 256) {
    const int rr = o >> 5, cc = o & 31;
    const float v = (red[0][rr][cc] + red[1][rr][cc]) + (red[2][rr][cc] + red[3][rr][cc]);
    part[((size_t)kc * A + 32 * tn + rr) * D + 32 * tk + cc] = v;
  }
}

// Parameter gradients of the whole attention layer from the slabs (fixed
// slab order, deterministic), written straight into the model's gradient
// tensors: gW1 (A, 2d) = [dW1q | dW1k[:, :d]], gb1, gw2, gb2.  A block owns
// 64 consecutive outputs of the layout {dW1q, dW1k, db1, dw2, db2}; its 8
// waves each sum every 8th slab with 4 loads in flight, then combine.
// norm_part (optional): gW1 is then the base of the model's flat gradient
// buffer of n_flat floats ([gW1 | gb1 | gw2 | gb2 | the head's gradients, final
// already]); block i also writes the fp64 sum of squares of flat entries
// [64 i, 64 i + 64) to norm_part[i] (blocks past the attention outputs only read
// the head's), so clip_grad_norm_ needs no second pass over the gradients.
__global__ __launch_bounds__(512) void din_bwd_reduce_params_kernel(const float* __restrict__ slabs, int nslab, int A,
                                                                    int D, int d, float* __restrict__ gW1,
                                                                    float* __restrict__ gb1, float* __restrict__ gw2,
                                                                    float* __restrict__ gb2,
                                                                    const float* __restrict__ qpart, int nkc,
                                                                    int64_t n_flat, double* __restrict__ norm_part) {
  __shared__ float part[8][64];
  const size_t n = slab_floats(A, D);
  const size_t nw = (size_t)A * d;  // per half of W1
  const size_t nout = 2 * nw + A + A + 1;
  const int o = threadIdx.x & 63, g = threadIdx.x >> 6;
  const size_t i = (size_t)blockIdx.x * 64 + o;
  size_t src = 0;
  if (i < nout) {
    if (i < 2 * nw) {
      const size_t row = i / (2 * (size_t)d);
      const int col = (int)(i % (2 * (size_t)d));
      src = col < d ? slab_q_off(A, D) + row * D + col : row * D + (col - d);
    } else if (i < 2 * nw + A) {
      src = slab_q_off(A, D) + (size_t)A * D + (i - 2 * nw);
    } else if (i < 2 * nw + 2 * A) {
      src = (size_t)A * D + (i - 2 * nw - A);
    } else {
      src = (size_t)A * D + A;
    }
  }
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (qpart != nullptr && i < 2 * nw && (int)(i % (2 * (size_t)d)) < d) {  // dW1q from din_dwq_kernel's chunks
    const size_t row = i / (2 * (size_t)d), col = i % (2 * (size_t)d);
    for (int kc = g; kc < nkc; kc += 8) s0 += qpart[((size_t)kc * A + row) * D + col];
  } else if (i < nout) {
    int j = g;
    for (; j + 24 < nslab; j += 32) {
      s0 += slabs[(size_t)j * n + src];
      s1 += slabs[(size_t)(j + 8) * n + src];
      s2 += slabs[(size_t)(j + 16) * n + src];
      s3 += slabs[(size_t)(j + 24) * n + src];
    }
    for (; j < nslab; j += 8) s0 += slabs[(size_t)j * n + src];
  }
  part[g][o] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (g == 0) {
    float t = 0.f;
    if (i < nout) {
      t = ((part[0][o] + part[1][o]) + (part[2][o] + part[3][o])) +
          ((part[4][o] + part[5][o]) + (part[6][o] + part[7][o]));
      if (i < 2 * nw) gW1[i] = t;
      else if (i < 2 * nw + A) gb1[i - 2 * nw] = t;
      else if (i < 2 * nw + 2 * A) gw2[i - 2 * nw - A] = t;
      else gb2[0] = t;
    } else if (norm_part != nullptr && (int64_t)i < n_flat) {
      t = gW1[i];  // a head gradient (flat buffer)
    }
    if (norm_part != nullptr) {
      const double sq = wave_sum((double)t * (double)t);
      if (o == 0) norm_part[blockIdx.x] = sq;
    }
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

// w = hi + mid + lo exactly, each part a bf16 (truncation split: hi keeps w's top
// 8 significant bits, w - hi is exact in f32 with <= 16 of them, mid its top 8,
// the remaining <= 8 bits are exactly a bf16), so q·hi + q·mid + q·lo are exact
// f32 products for a bf16 q.  Six integer/float ops instead of three RNE roundings.
__device__ __forceinline__ void split3_bf16(float w, short* hi, short* mid, short* lo) {
  const uint32_t hb = __float_as_uint(w) & 0xFFFF0000u;
  const float rem = w - __uint_as_float(hb);
  const uint32_t mb = __float_as_uint(rem) & 0xFFFF0000u;
  const float low = rem - __uint_as_float(mb);
  *hi = (short)(hb >> 16);
  *mid = (short)(mb >> 16);
  *lo = (short)(__float_as_uint(low) >> 16);
}

// ========================================================== train batch ==
// One DIN train batch assembled from the device-resident click log, replacing
// TrainDataset.__getitem__'s CPU gather (DIN.py:81-92) and the query half of
// the attention MLP (DIN.py:105-106): for the 32 samples of a block,
//   rows idx[b] -> history ids, target id, label;  q[b] = f32(table[target]);
//   U[b] = W1q q[b] + b1  on bf16 MFMA.  q is exact in bf16 (a bf16 table row)
//   and W1q is split three ways (hi + mid + lo bf16), so every product is the
//   exact f32 product of the f32 weight and q, accumulated in f32;
//   W1k (the key half of W1) -> bf16 for the attention kernels (grid-strided).
template <int D, bool DO_U>
__global__ __launch_bounds__(256) void din_batch_kernel(const int64_t* __restrict__ idx, int B,
                                                        const int32_t* __restrict__ hist_all,
                                                        const int32_t* __restrict__ tgt_all,
                                                        const float* __restrict__ lab_all, int64_t n_rows, int L,
                                                        const uint16_t* __restrict__ table, int64_t n_table,
                                                        const float* __restrict__ W1, const float* __restrict__ b1,
                                                        int A, int32_t* __restrict__ hist, float* __restrict__ q,
                                                        float* __restrict__ y, float* __restrict__ U,
                                                        uint16_t* __restrict__ W1k_bf) {
  constexpr int KS = D / 16;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
  const int b0 = blockIdx.x * 32;
  __shared__ int64_t s_row[32];
  __shared__ int32_t s_tgt[32];
  if (tid < 32) {
    const int b = b0 + tid;
    int64_t row = -1;
    int32_t t = -1;
    if (b < B) {
      row = idx[b];
      float lab = 0.f;
      if (row >= 0 && row < n_rows) {
        t = tgt_all[row];
        lab = lab_all[row];
      } else {
        row = -1;
      }
      y[b] = lab;
    }
    s_row[tid] = row;
    s_tgt[tid] = t;
  }
  if constexpr (DO_U) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + tid; e < (int64_t)A * D; e += (int64_t)gridDim.x * 256) {
      const int64_t n = e / D, k = e % D;
      W1k_bf[e] = f32_to_bf16_rne(W1[n * 2 * D + D + k]);
    }
  }
  __syncthreads();
  for (int e0 = tid; e0 < 32 * L; e0 += 8 * 256) {  // 8 loads in flight per thread
    int32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * 256;
      const int i = e / L, j = e % L;
      v[u] = (e < 32 * L && s_row[i < 32 ? i : 0] >= 0) ? hist_all[s_row[i] * L + j] : -1;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * 256;
      const int i = e / L, j = e % L, b = b0 + i;
      if (e < 32 * L && b < B) hist[(int64_t)b * L + j] = v[u];
    }
  }
  const int b = b0 + r;
  const int32_t t = s_tgt[r];
  const bool ok = b < B && t >= 0 && t < n_table;
  bf16x8 qf[KS];
#pragma unroll
  for (int s2 = 0; s2 < KS; ++s2) {
    if (ok) {
      qf[s2] = *reinterpret_cast<const bf16x8*>(table + (int64_t)t * D + 16 * s2 + 8 * h);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[s2][j] = 0;
    }
  }
  if (b < B) {
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) {
      if ((s2 & 3) != w) continue;
      float4 lo4, hi4;
      lo4.x = bf16_to_f32((uint16_t)qf[s2][0]); lo4.y = bf16_to_f32((uint16_t)qf[s2][1]);
      lo4.z = bf16_to_f32((uint16_t)qf[s2][2]); lo4.w = bf16_to_f32((uint16_t)qf[s2][3]);
      hi4.x = bf16_to_f32((uint16_t)qf[s2][4]); hi4.y = bf16_to_f32((uint16_t)qf[s2][5]);
      hi4.z = bf16_to_f32((uint16_t)qf[s2][6]); hi4.w = bf16_to_f32((uint16_t)qf[s2][7]);
      float* o = q + (int64_t)b * D + 16 * s2 + 8 * h;
      *reinterpret_cast<float4*>(o) = lo4;
      *reinterpret_cast<float4*>(o + 4) = hi4;
    }
  }
  if constexpr (!DO_U) return;
  for (int ws = w; ws < A / 32; ws += 4) {
    f32x16 acc;
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[g] = 0.f;
    const float* wrow = W1 + (int64_t)(32 * ws + r) * 2 * D;
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) {
      const float4 w0 = *reinterpret_cast<const float4*>(wrow + 16 * s2 + 8 * h);
      const float4 w1 = *reinterpret_cast<const float4*>(wrow + 16 * s2 + 8 * h + 4);
      const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      bf16x8 fh, fm, fl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        short h1, m1, l1;
        split3_bf16(wv[j], &h1, &m1, &l1);
        fh[j] = h1;
        fm[j] = m1;
        fl[j] = l1;
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fl, qf[s2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fm, qf[s2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fh, qf[s2], acc, 0, 0, 0);
    }
    if (b < B) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int n = 32 * ws + acc_row(g, h);
        U[(int64_t)b * A + n] = acc[g] + b1[n];
      }
    }
  }
}

// The per-step half of the train batch when the gathers of several steps ran
// ahead (nrk_din_batch with W1 == NULL over K steps' rows): U = q W1q^T + b1
// from the gathered f32 query rows (bf16-exact: rows of a bf16 table) and
// W1k -> bf16, the same MFMA split as din_batch_kernel.
template <int D>
__global__ __launch_bounds__(256) void din_u_kernel(const float* __restrict__ q, int B, const float* __restrict__ W1,
                                                    const float* __restrict__ b1, int A, float* __restrict__ U,
                                                    uint16_t* __restrict__ W1k_bf) {
  // U = q W1q^T + b1 for 16 samples per block on v_mfma_f32_16x16x32_bf16 (256
  // blocks at B = 4096; the 32x32x16 form had 128): q is exact in bf16, W1q
  // enters as hi + mid + lo bf16 parts (truncation: every product is the exact
  // f32 product).  Wave w owns the 16-unit tiles w, w + 4, ...
  constexpr int KS = D / 32;
  constexpr int MAXT = 2;  // A <= 128: at most two of the A / 16 unit tiles per wave
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l15 = lane & 15, l4 = lane >> 4;
  const int b0 = blockIdx.x * 16;
  const int b = b0 + l15;
  // every load of the block in flight before any math: the query rows, then both
  // unit tiles' W1q rows and biases (L2-resident after the first blocks)
  float4 qlo[KS], qhi[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    qlo[s] = make_float4(0.f, 0.f, 0.f, 0.f);
    qhi[s] = qlo[s];
    if (b < B) {
      qlo[s] = *reinterpret_cast<const float4*>(q + (int64_t)b * D + 32 * s + 8 * l4);
      qhi[s] = *reinterpret_cast<const float4*>(q + (int64_t)b * D + 32 * s + 8 * l4 + 4);
    }
  }
  float4 wv0[MAXT][KS], wv1[MAXT][KS];
  float bv[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int ut = w + 4 * t;
    const int u = 16 * (ut < A / 16 ? ut : 0) + l15;
    bv[t] = b1[u];
    const float* wrow = W1 + (int64_t)u * 2 * D + 8 * l4;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      wv0[t][s] = *reinterpret_cast<const float4*>(wrow + 32 * s);
      wv1[t][s] = *reinterpret_cast<const float4*>(wrow + 32 * s + 4);
    }
  }
  for (int64_t e = (int64_t)blockIdx.x * 256 + tid; e < (int64_t)A * D; e += (int64_t)gridDim.x * 256) {
    const int64_t n = e / D, k = e % D;
    W1k_bf[e] = f32_to_bf16_rne(W1[n * 2 * D + D + k]);
  }
  bf16x8 qf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    qf[s][0] = (short)f32_to_bf16_rne(qlo[s].x); qf[s][1] = (short)f32_to_bf16_rne(qlo[s].y);
    qf[s][2] = (short)f32_to_bf16_rne(qlo[s].z); qf[s][3] = (short)f32_to_bf16_rne(qlo[s].w);
    qf[s][4] = (short)f32_to_bf16_rne(qhi[s].x); qf[s][5] = (short)f32_to_bf16_rne(qhi[s].y);
    qf[s][6] = (short)f32_to_bf16_rne(qhi[s].z); qf[s][7] = (short)f32_to_bf16_rne(qhi[s].w);
  }
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int ut = w + 4 * t;
    if (ut >= A / 16) break;
    const int u = 16 * ut + l15;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const float wv[8] = {wv0[t][s].x, wv0[t][s].y, wv0[t][s].z, wv0[t][s].w,
                           wv1[t][s].x, wv1[t][s].y, wv1[t][s].z, wv1[t][s].w};
      bf16x8 fh, fm, fl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        short h1, m1, l1;
        split3_bf16(wv[j], &h1, &m1, &l1);
        fh[j] = h1;
        fm[j] = m1;
        fl[j] = l1;
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[s], fl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[s], fm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[s], fh, acc, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int bb = b0 + 4 * l4 + i;
      if (bb < B) U[(int64_t)bb * A + u] = acc[i] + bv[t];
    }
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
  const int cap = bwd ? 256 : 1024;
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
  const bool wave_ok = bf && hist_ids && (d == 64 || d == 128);
  const size_t pair_sm = ((size_t)((A + 63) & ~63) * 3 + (size_t)((L + 31) & ~31) * d + 4 * 128 + 2 * 256) * 4;
  if (bf && hist_ids && d == 256 && pair_sm <= 160 * 1024) {
    // a wave pair per sample: L <= 64 two WGs per CU; L 65..128 (twice the key image) one
    const bool two = pair_sm <= 80 * 1024;
    const size_t psm = pair_sm;
    int grid = (int)cdiv(B, 2);
    if (grid > (two ? 512 : 256)) grid = two ? 512 : 256;
    const uint16_t* tb = static_cast<const uint16_t*>(keys);
    const uint16_t* wk = static_cast<const uint16_t*>(W1k);
    hipStream_t st = (hipStream_t)stream;
    const int na = A / 32;
#define NRK_FWD_PAIR(NN)                                                                                          \
  do {                                                                                                            \
    if (two)                                                                                                      \
      hipLaunchKernelGGL((din_fwd_pair_kernel<256, NN>), dim3(grid), dim3(256), psm, st, tb, hist_ids, n_table, U, \
                         wk, w2, B, L, pooled, alpha);                                                            \
    else                                                                                                          \
      hipLaunchKernelGGL((din_fwd_pair_kernel<256, NN, 1>), dim3(grid), dim3(256), psm, st, tb, hist_ids, n_table, \
                         U, wk, w2, B, L, pooled, alpha);                                                         \
  } while (0)
    if (na == 1) NRK_FWD_PAIR(1); else if (na == 2) NRK_FWD_PAIR(2); else if (na == 3) NRK_FWD_PAIR(3);
    else NRK_FWD_PAIR(4);
#undef NRK_FWD_PAIR
    NRK_CHECK_LAUNCH("din_fwd_pair_kernel");
    return NRK_OK;
  }
  // d = 128: a wave pair per sample (each wave half the unit tiles: 168 VGPRs, three
  // workgroups = 12 waves per CU): 153.4 -> 151.5 us per train step against one wave
  // per sample at 8 waves per CU (profiles/r03_din_fwd_pair_ab.log)
  if (wave_ok && d == 128) {
    const size_t psm = pair_sm;
    // histories of 65..128 slots (twice the key image): fewer workgroups per CU
    NRK_CHECK_ARG(psm <= 160 * 1024, "din_fwd: L=%d d=%d needs %zu B LDS (pair)", L, d, psm);
    const int per_cu = (int)((160 * 1024) / psm) < 3 ? (int)((160 * 1024) / psm) : 3;
    int grid = (int)cdiv(B, 2);
    if (grid > 256 * per_cu) grid = 256 * per_cu;
    const uint16_t* tb = static_cast<const uint16_t*>(keys);
    const uint16_t* wk = static_cast<const uint16_t*>(W1k);
    hipStream_t st = (hipStream_t)stream;
    const int na = A / 32;
#define NRK_FWD_PAIR(NN)                                                                                          \
  hipLaunchKernelGGL((din_fwd_pair_kernel<128, NN, 3>), dim3(grid), dim3(256), psm, st, tb, hist_ids, n_table, U, wk, \
                     w2, B, L, pooled, alpha)
    if (na == 1) NRK_FWD_PAIR(1); else if (na == 2) NRK_FWD_PAIR(2); else if (na == 3) NRK_FWD_PAIR(3);
    else NRK_FWD_PAIR(4);
#undef NRK_FWD_PAIR
    NRK_CHECK_LAUNCH("din_fwd_pair_kernel");
    return NRK_OK;
  }
  if (wave_ok) {  // d = 64: one wave per sample
    const int Lp = (L + 31) & ~31;
    const size_t AP = (size_t)((A + 63) & ~63);
    const size_t slot = AP * 4 + (size_t)Lp * d * 2;
    // single-buffered slots, two workgroups per CU: measured faster than
    // double-buffered ones at one per CU (41 vs 51 us at B=4096, L=50, d=128)
    const size_t wsm = AP * 4 + 4 * slot + 4 * 128 * 4;  // + the waves' compacted id tables
    int grid = (int)cdiv(B, 4);
    if (grid > 512) grid = 512;
    const uint16_t* tb = static_cast<const uint16_t*>(keys);
    const uint16_t* wk = static_cast<const uint16_t*>(W1k);
    hipStream_t st = (hipStream_t)stream;
    const int na = A / 32;
#define NRK_FWD_WAVE(NN)                                                                                            \
  hipLaunchKernelGGL((din_fwd_wave_kernel<64, NN, 1>), dim3(grid), dim3(256), wsm, st, tb, hist_ids, n_table, U, wk,  \
                     w2, B, L, pooled, alpha)
    if (na == 1) NRK_FWD_WAVE(1); else if (na == 2) NRK_FWD_WAVE(2); else if (na == 3) NRK_FWD_WAVE(3);
    else NRK_FWD_WAVE(4);
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

constexpr int DWQ_KC = 64;  // sample chunks of din_dwq_kernel

// workspace: slabs | dU rows of both row groups [2][B][A] | dW1q chunks [KC][A][d] | dummy store slots
size_t bwd_ws_parts(int B, int d, int A, size_t off[4]) {
  const int grid = B > 0 ? din_grid(B, true) : 1;
  off[0] = 0;
  off[1] = align_up((size_t)grid * slab_floats(A, d) * 4, 256);
  off[2] = align_up(off[1] + (size_t)2 * B * A * 4, 256);
  off[3] = align_up(off[2] + (size_t)DWQ_KC * A * d * 4, 256);
  return off[3] + (size_t)grid * 512 * 4;
}

extern "C" int nrk_din_attn_bwd_workspace(int32_t B, int32_t d, int32_t A, size_t* ws_bytes) {
  NRK_CHECK_ARG(ws_bytes != nullptr, "din_bwd_workspace: null");
  size_t off[4];
  *ws_bytes = bwd_ws_parts(B, d, A, off);
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
  const bool pipe_ok = bf && hist_ids && (d == 64 || d == 128);
  if (pipe_ok) {
    const int Lp = (L + 31) & ~31;
    const size_t psm = (size_t)(2 * (d + 128 + Lp * d / 2) + 4 * 128) * 4;
    NRK_CHECK_ARG(psm <= 160 * 1024, "din_bwd: L=%d d=%d needs %zu B LDS", L, d, psm);
    if (d == 128)
      hipLaunchKernelGGL(din_bwd_pipe_kernel<128>, dim3(grid), dim3(256), psm, st, static_cast<const uint16_t*>(keys),
                         hist_ids, n_table, U, static_cast<const uint16_t*>(W1k), w2, B, L, A, dpooled, alpha, dU, slabs,
                         nullptr, 0);
    else
      hipLaunchKernelGGL(din_bwd_pipe_kernel<64>, dim3(grid), dim3(256), psm, st, static_cast<const uint16_t*>(keys),
                         hist_ids, n_table, U, static_cast<const uint16_t*>(W1k), w2, B, L, A, dpooled, alpha, dU, slabs,
                         nullptr, 0);
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

extern "C" int nrk_din_batch(const int64_t* idx, int32_t B, const int32_t* hist_all, const int32_t* tgt_all,
                             const float* lab_all, int64_t n_rows, int32_t L, const void* table, int64_t n_table,
                             int32_t dtype, int32_t d, const float* W1, const float* b1, int32_t A, int32_t* hist,
                             float* q, float* y, float* U, void* W1k_bf16, void* stream) {
  NRK_CHECK_ARG(dtype == NRK_DTYPE_BF16, "din_batch: the table must be bf16");
  NRK_CHECK_ARG(d == 64 || d == 128 || d == 256, "din_batch: emb_dim %d unsupported (64, 128, 256)", d);
  NRK_CHECK_ARG(A >= 32 && A <= 128 && A % 32 == 0, "din_batch: attn_units %d unsupported (32..128 step 32)", A);
  NRK_CHECK_ARG(L >= 1 && L <= 128 && B >= 0, "din_batch: bad L=%d / B=%d", L, B);
  if (B == 0) return NRK_OK;
  const bool do_u = W1 != nullptr;  // W1 == NULL: the gathers only (several steps' rows ahead; nrk_din_batch_u)
  NRK_CHECK_ARG(idx && hist_all && tgt_all && lab_all && table && hist && q && y && (!do_u || (b1 && U && W1k_bf16)),
                "din_batch: null pointer");
  const unsigned grid = (unsigned)cdiv(B, 32);
  hipStream_t st = (hipStream_t)stream;
  const uint16_t* tb = static_cast<const uint16_t*>(table);
  uint16_t* wk = static_cast<uint16_t*>(W1k_bf16);
#define NRK_BATCH(DD)                                                                                               \
  do {                                                                                                              \
    if (do_u)                                                                                                       \
      hipLaunchKernelGGL((din_batch_kernel<DD, true>), dim3(grid), dim3(256), 0, st, idx, B, hist_all, tgt_all,     \
                         lab_all, n_rows, L, tb, n_table, W1, b1, A, hist, q, y, U, wk);                              \
    else                                                                                                            \
      hipLaunchKernelGGL((din_batch_kernel<DD, false>), dim3(grid), dim3(256), 0, st, idx, B, hist_all, tgt_all,    \
                         lab_all, n_rows, L, tb, n_table, W1, b1, A, hist, q, y, U, wk);                              \
  } while (0)
  if (d == 256) NRK_BATCH(256); else if (d == 128) NRK_BATCH(128); else NRK_BATCH(64);
#undef NRK_BATCH
  NRK_CHECK_LAUNCH("din_batch_kernel");
  return NRK_OK;
}

static int bwd_params_impl(const void* table, const int32_t* hist_ids, int64_t n_table, int32_t dtype,
                           const float* q, const float* U, const void* W1k, const float* w2, int32_t B, int32_t L,
                           int32_t d, int32_t A, const float* dpooled, const float* alpha, const float* pooled,
                           float* gW1, float* gb1, float* gw2, float* gb2, float* dU, void* ws, size_t ws_bytes,
                           void* stream, const DpSrc* dps, int64_t n_flat = 0, double* norm_part = nullptr) {
  int rc = check_common(table, dtype, B, L, d, A);
  if (rc) return rc;
  NRK_CHECK_ARG(dtype == NRK_DTYPE_BF16 && hist_ids != nullptr &&
                    (d == 64 || d == 128 || (d == 256 && dU == nullptr)),
                "din_bwd_params: needs a bf16 table, history ids and emb_dim 64 or 128 (256: no dU output)");
  NRK_CHECK_ARG(B > 0, "din_bwd_params: empty batch");
  NRK_CHECK_ARG(q && U && W1k && w2 && (dpooled || dps) && alpha && gW1 && gb1 && gw2 && gb2 && ws,
                "din_bwd_params: null pointer");
  NRK_CHECK_ARG(!dps || (dU == nullptr && (d == 64 || d == 128) && L <= 64),
                "din_bwd_params_head: d=%d L=%d (needs d 64 or 128, L <= 64)", d, L);
  const int grid = din_grid(B, true);
  size_t woff[4];
  const size_t need = bwd_ws_parts(B, d, A, woff);
  if (ws_bytes < need) return fail(NRK_EWORKSPACE, "din_bwd_params: workspace %zu < %zu", ws_bytes, need);
  float* dUp = reinterpret_cast<float*>(static_cast<char*>(ws) + woff[1]);
  float* qpart_w8 = reinterpret_cast<float*>(static_cast<char*>(ws) + woff[2]);
  float* dmy = reinterpret_cast<float*>(static_cast<char*>(ws) + woff[3]);
  const float* qpart = nullptr;
  const int Lp = (L + 31) & ~31;
  const size_t psm = (size_t)(2 * (d + 128 + Lp * d / 2) + 4 * 128) * 4;
  NRK_CHECK_ARG(psm <= 160 * 1024, "din_bwd_params: L=%d d=%d needs %zu B LDS", L, d, psm);
  hipStream_t st = (hipStream_t)stream;
  float* slabs = static_cast<float*>(ws);
  const uint16_t* tb = static_cast<const uint16_t*>(table);
  const uint16_t* wk = static_cast<const uint16_t*>(W1k);
  if (dU == nullptr && d == 256) {  // the reference's width: column-split 8-wave backward
    const int LPk = Lp <= 32 ? 32 : 64;
    constexpr int NS = 3, RING = 4;
    const size_t dsm = (size_t)(NS * (4 * 128 + LPk * d / 2) + 8 * RING * 64 + 8 * 64 + 64 + 8 * 1024) * 4;
    NRK_CHECK_ARG(dsm <= 160 * 1024, "din_bwd_params: L=%d d=%d needs %zu B LDS", L, d, dsm);
    if (L > 64) {  // two half-samples per sample; the softmax term first (into the dW1q chunk area,
                   // which din_dwq_kernel only writes after the backward)
      NRK_CHECK_ARG((size_t)B <= (size_t)DWQ_KC * A * d, "din_bwd_params: batch %d too large for L > 64", B);
      float* cd = qpart_w8;
      if (pooled)  // sum_l alpha_l (dp . k_l) = dp . pooled: 8 KB per sample instead of the key rows
        hipLaunchKernelGGL(din_cdot_pooled_kernel<256>, dim3((unsigned)cdiv(B, 4)), dim3(256), 0, st, dpooled, pooled,
                           B, cd);
      else
        hipLaunchKernelGGL(din_cdot_kernel<256>, dim3((unsigned)cdiv(B, 4)), dim3(256), 0, st, tb, hist_ids, n_table,
                           dpooled, alpha, B, L, cd);
      NRK_CHECK_LAUNCH("din_cdot_kernel");
      hipLaunchKernelGGL((din_bwd_deep8c_kernel<256, 64, NS, true>), dim3(grid), dim3(512), dsm, st, tb, hist_ids,
                         n_table, U, wk, w2, B, L, A, dpooled, alpha, slabs, dUp, dmy, cd);
    } else if (LPk == 32)
      hipLaunchKernelGGL((din_bwd_deep8c_kernel<256, 32, NS>), dim3(grid), dim3(512), dsm, st, tb, hist_ids, n_table, U,
                         wk, w2, B, L, A, dpooled, alpha, slabs, dUp, dmy);
    else
      hipLaunchKernelGGL((din_bwd_deep8c_kernel<256, 64, NS>), dim3(grid), dim3(512), dsm, st, tb, hist_ids, n_table, U,
                         wk, w2, B, L, A, dpooled, alpha, slabs, dUp, dmy);
    NRK_CHECK_LAUNCH("din_bwd_deep8c_kernel");
    const int kchunk = (int)cdiv(B, DWQ_KC);
    hipLaunchKernelGGL(din_dwq_kernel, dim3((unsigned)(A / 32 * (d / 32)), DWQ_KC), dim3(256), 0, st, dUp, q, B, A, d, d,
                       kchunk, qpart_w8);
    NRK_CHECK_LAUNCH("din_dwq_kernel");
    qpart = qpart_w8;
  } else if (dU == nullptr) {  // the fused train step: deep-prefetch kernels, dW1q formed here too
    const int LPk = Lp <= 32 ? 32 : Lp <= 64 ? 64 : 128;
    const int nslot = 4;
    const bool w8 = LPk * d >= 4096;  // >= 8 key-image pieces: one per wave
    size_t dsm = (size_t)(nslot * (4 * 128 + LPk * d / 2) + 4 * 4 * 128 + 5 * 128) * 4;
    // deep8: 3 slots (2 samples in flight; 4 and 5 measured no faster, profiles/r03_din_ab.log)
    constexpr int nslot8 = 3;
    // dW1q folded into the 8-wave kernel (16 samples' dU / q rows in LDS) while a
    // workgroup holds at most 16 samples; beyond, dU rows + din_dwq_kernel
    const bool fold_q = cdiv(B, grid) <= 16;
    if (w8) {
      const int ring8 = 4;
      dsm = (size_t)(nslot8 * (4 * 128 + LPk * d / 2) + 8 * ring8 * 128 + 9 * 128 + (fold_q ? 48 * 128 : 0) +
                     (dps ? 32 * d + 6 * d : 0)) * 4;
      const size_t xneed = ((size_t)4 * 32 * d + 257) * 4;  // pair-combine exchange area (reuses the slots)
      if (dsm < xneed) dsm = xneed;
    }
    // head-fused with dW1q folded: the two-stream form (two groups of four waves, one
    // sample each per iteration): 151.5 -> 148.1 us per train step at B = 4096 against
    // the row-group split (profiles/r03_deep8_groups_ab.log)
    const bool group8 = dps && w8 && fold_q && LPk <= 64;
    if (group8) {
      dsm = (size_t)(2 * 3 * (4 * 128 + LPk * d / 2) + 8 * 4 * 64 + 8 * 64 + 2 * 64 + 2 * 16 * 128 + 2 * d + 32 * d +
                     5 * d) * 4;
      const size_t xneed = ((size_t)4 * 32 * d + 257) * 4;
      if (dsm < xneed) dsm = xneed;
    }
    NRK_CHECK_ARG(dsm <= 160 * 1024, "din_bwd_params: L=%d d=%d needs %zu B LDS", L, d, dsm);
#define NRK_BWD_DEEP8_V(DD, LL, FQV, FDPV)                                                                         \
  hipLaunchKernelGGL((din_bwd_deep8_kernel<DD, LL, 3, FQV, FDPV>), dim3(grid), dim3(512), dsm, st, tb, hist_ids,     \
                     n_table, U, wk, w2, B, L, A, dpooled, alpha, slabs, q, d, dUp, dmy, dpv)
#define NRK_BWD_DEEP8_FDP(DD, LL)                                                                                   \
  do {                                                                                                              \
    if (group8)                                                                                                     \
      hipLaunchKernelGGL((din_bwd_deep8g_kernel<DD, LL>), dim3(grid), dim3(512), dsm, st, tb, hist_ids, n_table, U, wk, \
                         w2, B, L, A, alpha, slabs, q, d, dpv);                                                      \
    else NRK_BWD_DEEP8_V(DD, LL, false, true);                                                                      \
  } while (0)
#define NRK_BWD_DEEP(DD, LL)                                                                                          \
  do {                                                                                                              \
    if (w8) {                                                                                                       \
      if (fold_q) NRK_BWD_DEEP8_V(DD, LL, true, false); else NRK_BWD_DEEP8_V(DD, LL, false, false);                 \
    } else                                                                                                          \
      hipLaunchKernelGGL((din_bwd_deep_kernel<DD, LL, 4>), dim3(grid), dim3(256), dsm, st, tb, hist_ids, n_table, U, wk, \
                         w2, B, L, A, dpooled, alpha, slabs, q, d);                                                   \
  } while (0)
    const DpSrc dpv = dps ? *dps : DpSrc{};
    if (dps) {
      NRK_CHECK_ARG(w8, "din_bwd_params_head: needs the 8-wave backward (L * d >= 4096)");
      if (d == 128) {
        if (LPk == 32) NRK_BWD_DEEP8_FDP(128, 32); else NRK_BWD_DEEP8_FDP(128, 64);
      } else {
        NRK_BWD_DEEP8_FDP(64, 64);  // w8: L d >= 4096, so LPk = 64 here
      }
    } else
    if (d == 128) {
      if (LPk == 32) NRK_BWD_DEEP(128, 32); else if (LPk == 64) NRK_BWD_DEEP(128, 64); else NRK_BWD_DEEP(128, 128);
    } else {
      if (LPk == 32) NRK_BWD_DEEP(64, 32); else if (LPk == 64) NRK_BWD_DEEP(64, 64); else NRK_BWD_DEEP(64, 128);
    }
#undef NRK_BWD_DEEP
#undef NRK_BWD_DEEP8_FDP
#undef NRK_BWD_DEEP8_V
    NRK_CHECK_LAUNCH("din_bwd_deep_kernel");
    if (w8 && !fold_q) {
      const int kchunk = (int)cdiv(B, DWQ_KC);
      hipLaunchKernelGGL(din_dwq_kernel, dim3((unsigned)(A / 32 * (d / 32)), DWQ_KC), dim3(256), 0, st, dUp, q, B, A, d, d,
                         kchunk, qpart_w8);
      NRK_CHECK_LAUNCH("din_dwq_kernel");
      qpart = qpart_w8;
    }
  } else {
    if (d == 128)
      hipLaunchKernelGGL(din_bwd_pipe_kernel<128>, dim3(grid), dim3(256), psm, st, tb, hist_ids, n_table, U, wk, w2, B,
                         L, A, dpooled, alpha, dU, slabs, q, d);
    else
      hipLaunchKernelGGL(din_bwd_pipe_kernel<64>, dim3(grid), dim3(256), psm, st, tb, hist_ids, n_table, U, wk, w2, B, L,
                         A, dpooled, alpha, dU, slabs, q, d);
    NRK_CHECK_LAUNCH("din_bwd_pipe_kernel");
  }
  const size_t nout = 2 * (size_t)A * d + 2 * (size_t)A + 1;
  const int64_t nblk_out = cdiv(norm_part ? (n_flat > (int64_t)nout ? n_flat : (int64_t)nout) : (int64_t)nout, 64);
  if (norm_part) {
    NRK_CHECK_ARG(gb1 == gW1 + 2 * (size_t)A * d && gw2 == gb1 + A && gb2 == gw2 + A && n_flat >= (int64_t)nout,
                  "din_bwd_params: norm partials need [gW1 | gb1 | gw2 | gb2] at the start of the flat buffer");
  }
  hipLaunchKernelGGL(din_bwd_reduce_params_kernel, dim3((unsigned)nblk_out), dim3(512), 0, st, slabs,
                     grid, A, d, d, gW1, gb1, gw2, gb2, qpart, qpart ? DWQ_KC : 0, n_flat, norm_part);
  NRK_CHECK_LAUNCH("din_bwd_reduce_params_kernel");
  return NRK_OK;
}

extern "C" int nrk_din_attn_bwd_params(const void* table, const int32_t* hist_ids, int64_t n_table, int32_t dtype,
                                       const float* q, const float* U, const void* W1k, const float* w2, int32_t B,
                                       int32_t L, int32_t d, int32_t A, const float* dpooled, const float* alpha,
                                       const float* pooled, float* gW1, float* gb1, float* gw2, float* gb2, float* dU,
                                       int64_t n_flat, double* norm_part, void* ws, size_t ws_bytes, void* stream) {
  return bwd_params_impl(table, hist_ids, n_table, dtype, q, U, W1k, w2, B, L, d, A, dpooled, alpha, pooled, gW1, gb1,
                         gw2, gb2, dU, ws, ws_bytes, stream, nullptr, n_flat, norm_part);
}

extern "C" int nrk_din_attn_bwd_params_head(const void* table, const int32_t* hist_ids, int64_t n_table,
                                            int32_t dtype, const float* q, const float* U, const void* W1k,
                                            const float* w2, int32_t B, int32_t L, int32_t d, int32_t A,
                                            const float* pooled, const float* alpha, int32_t F,
                                            const nrk_din_head_params* hp, const void* head_ws, size_t head_ws_bytes,
                                            float* gW1, float* gb1, float* gw2, float* gb2, int64_t n_flat,
                                            double* norm_part, void* ws, size_t ws_bytes, void* stream) {
  NRK_CHECK_ARG(F == 32 && hp && pooled && head_ws, "din_bwd_params_head: needs F = 32, head params, pooled, head ws");
  DpSrc dps{};
  const float* da1 = nullptr;
  int rc = nrk_din_head_ws_views(B, d, F, head_ws, head_ws_bytes, &dps.stat0, &dps.sum5, &da1);
  if (rc) return rc;
  dps.pooled = pooled;
  dps.da1 = da1;
  dps.w1 = hp->fc1_w;
  dps.bn0w = hp->bn0_w;
  dps.invB = 1.f / (float)B;
  return bwd_params_impl(table, hist_ids, n_table, dtype, q, U, W1k, w2, B, L, d, A, nullptr, alpha, nullptr, gW1, gb1, gw2,
                         gb2, nullptr, ws, ws_bytes, stream, &dps, n_flat, norm_part);
}

extern "C" int nrk_din_batch_u(const float* q, int32_t B, int32_t d, const float* W1, const float* b1, int32_t A,
                               float* U, void* W1k_bf16, void* stream) {
  NRK_CHECK_ARG(d == 64 || d == 128 || d == 256, "din_batch_u: emb_dim %d unsupported (64, 128, 256)", d);
  NRK_CHECK_ARG(A >= 32 && A <= 128 && A % 32 == 0, "din_batch_u: attn_units %d unsupported (32..128 step 32)", A);
  NRK_CHECK_ARG(B >= 0, "din_batch_u: bad B=%d", B);
  if (B == 0) return NRK_OK;
  NRK_CHECK_ARG(q && W1 && b1 && U && W1k_bf16, "din_batch_u: null pointer");
  const unsigned grid = (unsigned)cdiv(B, 16);
  hipStream_t st = (hipStream_t)stream;
  uint16_t* wk = static_cast<uint16_t*>(W1k_bf16);
  if (d == 256) hipLaunchKernelGGL(din_u_kernel<256>, dim3(grid), dim3(256), 0, st, q, B, W1, b1, A, U, wk);
  else if (d == 128) hipLaunchKernelGGL(din_u_kernel<128>, dim3(grid), dim3(256), 0, st, q, B, W1, b1, A, U, wk);
  else hipLaunchKernelGGL(din_u_kernel<64>, dim3(grid), dim3(256), 0, st, q, B, W1, b1, A, U, wk);
  NRK_CHECK_LAUNCH("din_u_kernel");
  return NRK_OK;
}
