// knn_flat.hip — exact flat k-NN for gfx950 (replaces faiss IndexFlatIP /
// IndexFlatL2 .search, Retrieval.py:21,25-32).
//
// Pipeline per search (all on the caller's stream, no host sync):
//   1. query_prepare  : xq -> bf16 q^ (zero-padded to DP), per-query norms
//   2. screen         : bf16 MFMA (32x32x16) query x corpus-chunk tiles; every
//                       lane keeps its top-(M+1) screened scores in registers;
//                       writes M candidates + the (M+1)-th score (theta) per
//                       (query, chunk, lane-half)
//   3. merge_rescore  : per query: bitonic-sort the union of candidates, take
//                       the top KP, rescore them EXACTLY (fp64, sequential d —
//                       bit-identical to oracle/knn_exact.c), sort, and certify
//                       with a rigorous screening error bound that no item
//                       outside the KP candidates can enter the exact top-k;
//                       uncertified queries are appended to a fallback list
//   4. exact_topk     : fp64 brute force for the fallback list (normally empty)
// See DESIGN.md "K-GEMM-TOPK" for the bound and the roofline.
#include <float.h>
#include <math.h>

#include <type_traits>

#include "screen16.h"

namespace nrk {

// ================================================================ prepare ==
// One wave per row, grid-stride; the three corpus maxima are reduced per wave
// and published with one atomic each (per-row atomics on three addresses
// serialise at the L2).
__global__ void flat_prepare_kernel(const float* __restrict__ xb, int64_t nb, int d, int dp,
                                    uint16_t* __restrict__ xbh, float* __restrict__ meta,
                                    float* __restrict__ stats) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  float m0 = 0.f, m1 = 0.f, m2 = 0.f;
  for (int64_t row = wave0; row < nb; row += nwaves) {
    double sx2 = 0.0, sh2 = 0.0, sr2 = 0.0;
    for (int j = lane; j < dp; j += 64) {
      float x = j < d ? xb[row * d + j] : 0.f;
      uint16_t h = f32_to_bf16_rne(x);
      float hf = bf16_to_f32(h);
      double r = (double)x - (double)hf;
      sx2 += (double)x * (double)x;
      sh2 += (double)hf * (double)hf;
      sr2 += r * r;
      xbh[row * dp + j] = h;
    }
    sx2 = wave_sum(sx2);
    sh2 = wave_sum(sh2);
    sr2 = wave_sum(sr2);
    const float rn = f64_to_f32_up(sqrt(sr2) * (1.0 + 1e-9));
    if (lane == 0) {
      meta[2 * row] = (float)sx2;
      meta[2 * row + 1] = rn;
    }
    m0 = fmaxf(m0, f64_to_f32_up(sqrt(sh2) * (1.0 + 1e-9)));
    m1 = fmaxf(m1, rn);
    m2 = fmaxf(m2, f64_to_f32_up(sx2 * (1.0 + 1e-9)));
  }
  if (lane == 0 && wave0 < nb) {
    atomic_max_nonneg(&stats[0], m0);
    atomic_max_nonneg(&stats[1], m1);
    atomic_max_nonneg(&stats[2], m2);
  }
}

// qmeta[4*q] = {||q^|| (up), ||q - q^|| (up), ||q||^2, 0}
__global__ void query_prepare_kernel(const float* __restrict__ xq, int64_t nq, int64_t nq_pad, int d,
                                     int dp, uint16_t* __restrict__ qh, double* __restrict__ qmeta,
                                     int* __restrict__ zero4 = nullptr, int* __restrict__ zero2 = nullptr) {
  const int lane = threadIdx.x & 63;
  // the search's fallback counters (instead of two memset launches)
  if (blockIdx.x == 0 && threadIdx.x < 4 && zero4) zero4[threadIdx.x] = 0;
  if (blockIdx.x == 0 && threadIdx.x < 2 && zero2) zero2[threadIdx.x] = 0;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= nq_pad) return;
  double sq2 = 0.0, sh2 = 0.0, sr2 = 0.0;
  for (int j = lane; j < dp; j += 64) {
    float x = (row < nq && j < d) ? xq[row * d + j] : 0.f;
    uint16_t h = f32_to_bf16_rne(x);
    float hf = bf16_to_f32(h);
    double r = (double)x - (double)hf;
    sq2 += (double)x * (double)x;
    sh2 += (double)hf * (double)hf;
    sr2 += r * r;
    qh[row * dp + j] = h;
  }
  sq2 = wave_sum(sq2);
  sh2 = wave_sum(sh2);
  sr2 = wave_sum(sr2);
  if (lane == 0 && row < nq) {
    qmeta[4 * row + 0] = sqrt(sh2) * (1.0 + 1e-9);
    qmeta[4 * row + 1] = sqrt(sr2) * (1.0 + 1e-9);
    qmeta[4 * row + 2] = sq2;
    qmeta[4 * row + 3] = 0.0;
  }
}

// tau[q] = the R-th largest finite lane maximum of the pre-pass (or -inf if
// there are fewer than R): R distinct items score at least this much, so it
// never exceeds the query's global R-th best screened score.  One wave per
// query, values in registers.  Exact selection by bisection on the ordered
// integer keys of the floats (32 rounds of ballot counts), not R rounds of
// wave argmax (k = 200: R = 400 rounds took 0.33 ms per 4096 queries).
//
// With ids_in (IVF phase A: the position of each lane maximum), ids_out[q][i]
// receives the positions of R entries >= tau (all above it, then ties in
// (value slot, lane) order), or of every finite entry (-1 past the end).
__device__ __forceinline__ uint32_t ordered_key(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float key_value(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
__device__ __forceinline__ int lanes_below(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// VPL: values per lane (nvals <= 64 * VPL); the flat pre-pass writes 8R = 64
// values per query for k <= 8, so VPL = 1 there (16x fewer ballots per
// bisection round than the VPL = 16 form)
template <int VPL>
__global__ __launch_bounds__(256) void tau_select_kernel(const float* __restrict__ premax, int nvals, int R,
                                                         int64_t nq, float* __restrict__ tau,
                                                         const int* __restrict__ ids_in = nullptr,
                                                         int* __restrict__ ids_out = nullptr) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;
  if (ids_out)
    for (int i = lane; i < R; i += 64) ids_out[q * R + i] = -1;
  uint32_t key[VPL];       // 0: not finite (-inf, NaN: never selected)
  int nfin = 0;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int i = j * 64 + lane;
    const float v = i < nvals ? premax[q * nvals + i] : -INFINITY;
    key[j] = v > -INFINITY ? ordered_key(v) : 0u;
    nfin += __popcll(__ballot(key[j] != 0u));
  }
  uint32_t K = 0;  // the R-th largest key (0: fewer than R finite values)
  if (nfin >= R) {
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t c = K | (1u << bit);
      int n = 0;
#pragma unroll
      for (int j = 0; j < VPL; ++j) n += __popcll(__ballot(key[j] >= c));
      if (n >= R) K = c;
    }
  }
  if (lane == 0) tau[q] = K ? key_value(K) : -INFINITY;
  if (!ids_out) return;
  // every key above K, then ties at K in (j, lane) order, up to R entries
  // (K = 0: every finite entry)
  int base = 0, need = R;
#pragma unroll
  for (int j = 0; j < VPL; ++j) need -= K ? __popcll(__ballot(key[j] > K)) : 0;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const unsigned long long gt = __ballot(K ? key[j] > K : key[j] != 0u);
    const unsigned long long eq = K ? __ballot(key[j] == K) : 0ull;
    const int er = lanes_below(eq);
    const bool tie = ((eq >> lane) & 1ull) && er < need;
    const unsigned long long sel = gt | __ballot(tie);
    if ((sel >> lane) & 1ull) {
      const int pos = base + lanes_below(sel);
      if (pos < R) ids_out[q * R + pos] = ids_in[q * nvals + j * 64 + lane];
    }
    base += __popcll(sel);
    const int ne = __popcll(eq);
    need -= ne < need ? ne : need;
  }
}

// ========================================================= merge/rescore ==
// fp64 score in the oracle's serial order (bit-identical).  One lane per
// candidate row: scalar loads measured faster than float4 ones here (k = 5
// merge 0.086 vs 0.103 ms); many candidates go through the LDS-staged loop of
// merge_rescore_kernel instead.
__device__ __forceinline__ double exact_score(const float* __restrict__ qs, const float* __restrict__ x,
                                              int d, bool l2) {
  double acc = 0.0;
  if (!l2) {
    for (int j = 0; j < d; ++j) acc = fma((double)qs[j], (double)x[j], acc);
  } else {
    for (int j = 0; j < d; ++j) {
      double t = (double)qs[j] - (double)x[j];
      acc = fma(t, t, acc);
    }
  }
  return acc;
}

__device__ __forceinline__ int pow2ceil(int n) {
  int p = 1;
  while (p < n) p <<= 1;
  return p;
}

// Fallback bookkeeping shared by the merge kernels and the tiled fallback.
// An uncertified query gets a slot s (list[s] = query) and, for s < slots, the
// merge's exact k-th (goodness, id): every item of the true top-k is at least
// that good, so the fallback only has to collect those.
struct FbState {
  int* list;        // [nq] queries, in slot order
  int* count;       // [0] = entries pushed, [1] = overflow count (fallback_select)
  int slots;        // slots with candidate storage (n, the tiled fallback's candidate lists)
  int tslots;       // slots with a stored threshold (>= slots)
  double* thr_g;    // [tslots]
  int64_t* thr_i;   // [tslots]
  int* n;           // [slots] candidates seen (may exceed cap)
  int force;        // testing: certify nothing
  __device__ void push(int qi, double g, int64_t i) const {
    const int s = atomicAdd(count, 1);
    list[s] = qi;
    if (s < tslots) {
      thr_g[s] = g;
      thr_i[s] = i;
    }
    if (s < slots) n[s] = 0;
  }
};

// IVF restriction for the exact paths: only items of the query's probed lists
// are eligible (faiss IndexIVF semantics); rows are addressed by id.
struct IvfFb {
  const int64_t* pos2id;    // [n] list-major position -> id (nullptr: flat index)
  const int* pos2list;      // [n]
  const int64_t* list_off;  // [nlist + 1]
  const int64_t* probe;     // [nq][nprobe] probed lists (-1: none)
  int nprobe;
  int nlist;
  int64_t nq;               // queries of the search (0: slot queries unchecked)
  int* err;                 // the search's guard word (GuardCode bits), or nullptr
};

// Top-kp selection for merge_rescore_kernel (256 threads, EPT union entries
// per thread in registers): the kp best by (score desc, id asc) -> ids[0, kp)
// (unordered; ids[kp, P2) = INT64_MAX), by a bisection on the order-preserving
// keys of the float scores (32 block counts) instead of a bitonic sort of the
// union; ties at the cut are taken by ascending id.  Returns the best score
// left out (the old sorted g[kp]).  g / id (the union's LDS) are scratch.
__device__ __forceinline__ uint32_t score_key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_score(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k ^ 0x80000000u) : ~k);
}
// The same selection for a union of at most 64 NK entries (U <= 1024): the
// keys and ids go to LDS, then wave 0 alone runs the bisection with wave
// ballots over NK keys per lane (no block barrier per round); ties at the cut
// are taken in slot order (deterministic; any choice keeps the certificate,
// which bounds every left-out item by the best left-out score, returned).
template <int NK, int EPT>
__device__ float select_top_wave(const double* rg, const int64_t* ri, const bool* rv, int U, int kp,
                                 uint32_t* kbuf, int64_t* ibuf, int64_t* ids, int P2) {
  __shared__ float s_out;
  const int tid = threadIdx.x, lane = tid & 63;
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int i = tid + 256 * e;
    if (i < U) {
      kbuf[i] = rv[e] ? score_key((float)rg[e]) : 0u;  // valid keys are >= 1
      ibuf[i] = ri[e];
    }
  }
  __syncthreads();
  if (tid < 64) {
    uint32_t kk[NK];
#pragma unroll
    for (int j = 0; j < NK; ++j) kk[j] = lane + 64 * j < U ? kbuf[lane + 64 * j] : 0u;
    uint32_t T = 0;  // the kp-th largest key
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t c = T | (1u << bit);
      int n = 0;
#pragma unroll
      for (int j = 0; j < NK; ++j) n += __popcll(__ballot(kk[j] >= c));
      if (n >= kp) T = c;
    }
    int ngt = 0;
#pragma unroll
    for (int j = 0; j < NK; ++j) ngt += __popcll(__ballot(kk[j] > T));
    int ties = kp - ngt, off = 0;  // ties at T still to take; output offset
    const uint64_t below = (1ull << lane) - 1;
    uint32_t kout = 0;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      const uint64_t eq = __ballot(kk[j] == T);
      const int rank = __popcll(eq & below);  // ties before this slot in this group
      const bool sel = kk[j] > T || (kk[j] == T && rank < ties);
      const uint64_t sm = __ballot(sel);
      if (sel) ids[off + __popcll(sm & below)] = ibuf[lane + 64 * j];
      if (!sel && kk[j] > kout) kout = kk[j];
      off += __popcll(sm);
      const int te = __popcll(eq);
      ties -= te < ties ? te : ties;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) kout = max(kout, (uint32_t)__shfl_xor((int)kout, o, 64));
    if (lane == 0) s_out = kout ? key_score(kout) : -INFINITY;
  }
  for (int i = kp + tid; i < P2; i += 256) ids[i] = INT64_MAX;
  __syncthreads();
  return s_out;
}

template <int EPT>
__device__ float select_top(const double* rg, const int64_t* ri, const bool* rv, int kp, double* g, int64_t* id,
                            int64_t* ids, int P2) {
  __shared__ int cnt[2][4], csum[4];
  __shared__ uint32_t kmax[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t key[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) key[e] = rv[e] ? score_key((float)rg[e]) : 0u;  // valid keys are >= 1
  auto block_count = [&](uint32_t c, bool strict, int buf) {
    int n = 0;
#pragma unroll
    for (int e = 0; e < EPT; ++e) n += __popcll(__ballot(strict ? key[e] > c : key[e] >= c));
    if (lane == 0) cnt[buf][w] = n;
    __syncthreads();
    return cnt[buf][0] + cnt[buf][1] + cnt[buf][2] + cnt[buf][3];
  };
  uint32_t T = 0;  // the kp-th largest key
  for (int bit = 31; bit >= 0; --bit) {
    const uint32_t c = T | (1u << bit);
    if (block_count(c, false, bit & 1) >= kp) T = c;
  }
  const int ngt = block_count(T, true, 1);  // (buffer 1: last written two barriers ago)
  const int nge = block_count(T, false, 0);
  const int r = kp - ngt;  // ties at T to take (>= 1)
  // the id cut among the ties: all of them, or the r smallest ids
  int64_t idcut = INT64_MAX;
  if (nge - ngt > r) {
    __shared__ int nt;
    if (tid == 0) nt = 0;
    __syncthreads();
#pragma unroll
    for (int e = 0; e < EPT; ++e)
      if (key[e] == T) {
        const int o = atomicAdd(&nt, 1);
        g[o] = 0.0;
        id[o] = ri[e];
      }
    __syncthreads();
    const int n2 = nt, P = pow2ceil(n2);
    for (int i = n2 + tid; i < P; i += 256) {
      g[i] = 0.0;
      id[i] = INT64_MAX;
    }
    __syncthreads();
    block_bitonic_sort(g, id, P);  // equal scores: ascending id
    idcut = id[r - 1];
    __syncthreads();
  }
  // compaction of the selected entries into ids[0, kp); the best key left out
  int ns = 0;
  uint32_t kout = 0;
  bool sel[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    sel[e] = key[e] > T || (key[e] == T && ri[e] <= idcut);
    ns += sel[e] ? 1 : 0;
    if (!sel[e] && rv[e]) kout = max(kout, key[e]);
  }
  int incl = ns;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) kout = max(kout, (uint32_t)__shfl_xor((int)kout, o, 64));
  if (lane == 63) csum[w] = incl;
  if (lane == 0) kmax[w] = kout;
  __syncthreads();
  int off = incl - ns;
  for (int j = 0; j < w; ++j) off += csum[j];
#pragma unroll
  for (int e = 0; e < EPT; ++e)
    if (sel[e]) ids[off++] = ri[e];
  for (int i = kp + tid; i < P2; i += 256) ids[i] = INT64_MAX;
  const uint32_t km = max(max(kmax[0], kmax[1]), max(kmax[2], kmax[3]));
  __syncthreads();
  return km ? key_score(km) : -INFINITY;
}

// One 256-thread workgroup per query.  Dynamic LDS: P doubles + P int64 (the
// union; later the rescoring's row stage, at least 256 x (RS_CW + 4) floats),
// P2 doubles + P2 int64 (rescored), d floats (query), reductions.
constexpr int RS_CW = 32;       // columns per rescoring stage (one 128-B line of each candidate row)
constexpr int RS_MIN_KP = 128;  // staged rescoring from this many candidates (k = 5: lane-per-row loads)
constexpr int SEL_MIN_KP = 0;   // top-KP by selection (else bitonic sort of the union) from this KP
// bytes of the merge's union region: the union (P doubles + P ids), the
// rescoring stage, or the small selection's 256 keys + 256 ids
__host__ __device__ inline int merge_union_bytes(int P, int KP) {
  int ub = 16 * P;
  if (KP >= RS_MIN_KP && ub < 256 * (RS_CW + 4) * 4) ub = 256 * (RS_CW + 4) * 4;
  if (ub < 12 * P + 16) ub = 12 * P + 16;  // the wave selection: P keys + P ids (P >= U)
  return ub;
}
__global__ __launch_bounds__(256) void merge_rescore_kernel(
    const float* __restrict__ part_s, const int* __restrict__ part_i, const float* __restrict__ part_t,
    int nch, int M, int KP, int k, int dp, const float* __restrict__ xq, const float* __restrict__ xb,
    int64_t nb, int d, int l2, const double* __restrict__ qmeta, const float* __restrict__ stats,
    const float* __restrict__ tau_q, float* __restrict__ D, int64_t* __restrict__ I, double* __restrict__ S,
    int64_t id_offset, FbState fb, const int64_t* __restrict__ pos2id) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int qi = blockIdx.x, tid = threadIdx.x;
  const int U = nch * 2 * M, P = pow2ceil(U);
  double* g = reinterpret_cast<double*>(smem);
  int64_t* id = reinterpret_cast<int64_t*>(g + P);
  const int P2 = pow2ceil(KP);
  const int UB = merge_union_bytes(P, KP);  // union / stage / small selection
  double* g2 = reinterpret_cast<double*>(smem + UB);
  int64_t* id2 = reinterpret_cast<int64_t*>(g2 + P2);
  float* qs = reinterpret_cast<float*>(id2 + P2);
  __shared__ float red[256];

  const float* ps = part_s + (int64_t)qi * U;
  const int* pi = part_i + (int64_t)qi * U;
  // the union (U <= 2048: at most 8 entries per thread) -> registers; only the
  // valid entries (with the pre-pass bound: a few hundred at k = 200, of 2048)
  // are compacted to the front and sorted
  constexpr int EPT = 8;
  double rg[EPT];
  int64_t ri[EPT];
  bool rv[EPT];
  int nv = 0;
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int i = tid + 256 * e;
    const float v = i < U ? ps[i] : -INFINITY;
    const int64_t item = i < U ? (int64_t)pi[i] : -1;
    rv[e] = v != -INFINITY && item >= 0 && item < nb;  // never dereference an unset slot
    rg[e] = (double)v;
    ri[e] = rv[e] ? (pos2id ? pos2id[item] : item) : INT64_MAX;  // IVF: list position -> id
    nv += rv[e] ? 1 : 0;
  }
  const int lane = tid & 63, w = tid >> 6;
  int incl = nv;  // inclusive prefix of the valid counts within the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  __shared__ int wsum[4];
  if (lane == 63) wsum[w] = incl;
  float th = -INFINITY;
  for (int i = tid; i < nch * 2; i += 256) th = fmaxf(th, part_t[(int64_t)qi * nch * 2 + i]);
  red[tid] = th;
  for (int i = tid; i < d; i += 256) qs[i] = xq[(int64_t)qi * d + i];
  __syncthreads();
  const int V = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  int off = incl - nv;
  for (int j = 0; j < w; ++j) off += wsum[j];
#pragma unroll
  for (int e = 0; e < EPT; ++e)
    if (rv[e]) {
      g[off] = rg[e];
      id[off] = ri[e];
      ++off;
    }
  // staged rescoring (many candidates): the top kp are SELECTED, not sorted
  // (the exact scores are sorted afterwards anyway)
  const bool staged = (d & 3) == 0 && KP >= RS_MIN_KP;
  const bool selected = staged || KP >= SEL_MIN_KP;
  const int PS = pow2ceil(V > 1 ? V : 1);
  if (!selected)
    for (int i = V + tid; i < PS; i += 256) {
      g[i] = -INFINITY;
      id[i] = INT64_MAX;
    }
  for (int o = 128; o > 0; o >>= 1) {  // (its first barrier also publishes the compaction)
    __syncthreads();
    if (tid < o) red[tid] = fmaxf(red[tid], red[tid + o]);
  }
  __syncthreads();
  const float theta_lanes = red[0];
  const int kp = KP < V ? KP : V;
  double theta = theta_lanes;
  if (!selected) {
    block_bitonic_sort(g, id, PS);
    theta = fmax(theta, kp < V ? g[kp] : -INFINITY);
  } else if (kp < V) {
    uint32_t* kb = reinterpret_cast<uint32_t*>(smem);
    int64_t* ib = reinterpret_cast<int64_t*>(smem + 4 * P);
    const float left = U <= 256 ? select_top_wave<4, EPT>(rg, ri, rv, U, kp, kb, ib, id2, P2)
                       : U <= 512 ? select_top_wave<8, EPT>(rg, ri, rv, U, kp, kb, ib, id2, P2)
                       : U <= 1024 ? select_top_wave<16, EPT>(rg, ri, rv, U, kp, kb, ib, id2, P2)
                                   : select_top<EPT>(rg, ri, rv, kp, g, id, id2, P2);
    theta = fmax(theta, (double)left);
  } else {
    for (int i = tid; i < P2; i += 256) id2[i] = i < kp ? id[i] : INT64_MAX;
    __syncthreads();
  }
  if (tau_q) theta = fmax(theta, (double)tau_q[qi]);  // items below the bound were never kept

  // exact rescoring of the top kp screened candidates
  if (staged) {
    // lane = candidate row, fp64 in the oracle's serial order, rows staged
    // through LDS RS_CW columns at a time by coalesced loads (8 lanes per
    // 128-B row piece); the union's LDS is the stage (its ids moved to id2)
    float* stg = reinterpret_cast<float*>(smem);  // [256][RS_CW + 4]
    for (int r0 = 0; r0 < kp; r0 += 256) {
      const int nr = kp - r0 < 256 ? kp - r0 : 256;
      double acc = 0.0;
      for (int c0 = 0; c0 < d; c0 += RS_CW) {
        const int cw = d - c0 < RS_CW ? d - c0 : RS_CW;
#pragma unroll
        for (int t = 0; t < RS_CW / 4; ++t) {
          const int e = tid + 256 * t, row = e / (RS_CW / 4), c4 = e % (RS_CW / 4);
          if (row < nr && 4 * c4 < cw)
            *reinterpret_cast<float4*>(stg + row * (RS_CW + 4) + 4 * c4) =
                *reinterpret_cast<const float4*>(xb + id2[r0 + row] * d + c0 + 4 * c4);
        }
        __syncthreads();
        if (tid < nr) {
          const float* xr = stg + tid * (RS_CW + 4);
          for (int j = 0; j < cw; j += 4) {
            const float4 v = *reinterpret_cast<const float4*>(xr + j);
            const float xv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              if (l2) {
                const double t = (double)qs[c0 + j + u] - (double)xv[u];
                acc = fma(t, t, acc);
              } else {
                acc = fma((double)qs[c0 + j + u], (double)xv[u], acc);
              }
            }
          }
        }
        __syncthreads();
      }
      if (tid < nr) g2[r0 + tid] = l2 ? -acc : acc;
    }
    for (int i = kp + tid; i < P2; i += 256) g2[i] = -INFINITY;
  } else {
    for (int i = tid; i < P2; i += 256) {
      if (i < kp) {
        const int64_t item = selected ? id2[i] : id[i];
        const double s = exact_score(qs, xb + item * d, d, l2 != 0);
        g2[i] = l2 ? -s : s;
        id2[i] = item;
      } else {
        g2[i] = -INFINITY;
        id2[i] = INT64_MAX;
      }
    }
  }
  __syncthreads();
  block_bitonic_sort(g2, id2, P2);

  if (tid == 0) {
    bool ok = kp >= k;
    if (ok && theta != -INFINITY) {
      const double nqh = qmeta[4 * qi + 0], nrq = qmeta[4 * qi + 1], qn2 = qmeta[4 * qi + 2];
      const double Xh = stats[0], R = stats[1], NX = stats[2];
      const double gam = (double)dp * 0x1p-22;
      const double bip = gam * nqh * Xh + nqh * R + nrq * Xh + nrq * R;
      const double kth = g2[k - 1];
      if (!l2) {
        const double lim = theta + bip;
        ok = kth - lim > 1e-12 * (fabs(lim) + fabs(kth));
      } else {
        const double B = 2.0 * bip + 0x1p-21 * (NX + nqh * Xh);
        const double lo = qn2 - theta - B;  // lower bound on any outsider's distance
        ok = lo - (-kth) > 1e-12 * (fabs(lo) + fabs(kth) + qn2);
      }
    }
    if (fb.force) ok = false;
    if (!ok) fb.push(qi, kp >= k ? g2[k - 1] : -INFINITY, kp >= k ? id2[k - 1] : (int64_t)-1);
  }
  for (int j = tid; j < k; j += 256) {
    const int64_t o = (int64_t)qi * k + j;
    const bool valid = j < kp;
    const double s = valid ? (l2 ? -g2[j] : g2[j]) : (l2 ? DBL_MAX : -DBL_MAX);
    D[o] = valid ? (float)s : (l2 ? FLT_MAX : -FLT_MAX);
    I[o] = valid ? id2[j] + id_offset : -1;
    if (S) S[o] = s;
  }
}

// ============================================================ exact top-k ==
// Workgroups loop over a query list (fallback) or over all queries (direct
// exact mode).  Block top-k kept in LDS: list [0,k), staged candidates
// [k, k+256), bitonic-merged whenever something was staged.
__global__ __launch_bounds__(256) void exact_topk_kernel(
    const float* __restrict__ xq, int64_t nq, const float* __restrict__ xb, int64_t nb, int d, int k,
    int l2, const int* __restrict__ qlist, const int* __restrict__ qcount, float* __restrict__ D,
    int64_t* __restrict__ I, double* __restrict__ S, int64_t id_offset, IvfFb iv,
    int* __restrict__ cnt_out = nullptr, const int* __restrict__ cnt_a = nullptr,
    const int* __restrict__ cnt_b = nullptr) {
  // the search's fallback counts (final: written by earlier launches) -> the
  // caller's n_fallback (instead of two copy launches)
  if (cnt_out && blockIdx.x == 0 && threadIdx.x == 0) {
    cnt_out[0] = *cnt_a;
    cnt_out[1] = *cnt_b;
  }
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int P = pow2ceil(k + 256);
  double* g = reinterpret_cast<double*>(smem);
  int64_t* id = reinterpret_cast<int64_t*>(g + P);
  float* qs = reinterpret_cast<float*>(id + P);
  __shared__ int s_nst, s_cnt;
  const int tid = threadIdx.x;
  const int64_t nwork = qcount ? (int64_t)*qcount : nq;
  for (int64_t wi = blockIdx.x; wi < nwork; wi += gridDim.x) {
    const int64_t qi = qlist ? (int64_t)qlist[wi] : wi;
    if (!guard_ok((uint64_t)qi < (uint64_t)nq, iv.err, GUARD_FB_QUERY)) continue;  // (block-uniform)
    for (int i = tid; i < P; i += 256) {
      g[i] = -INFINITY;
      id[i] = INT64_MAX;
    }
    for (int i = tid; i < d; i += 256) qs[i] = xq[qi * d + i];
    if (tid == 0) {
      s_nst = 0;
      s_cnt = 0;
    }
    __syncthreads();
    const int nrange = iv.pos2id ? iv.nprobe : 1;
    for (int pr = 0; pr < nrange; ++pr) {
    int64_t lo = 0, hi = nb;
    if (iv.pos2id) {
      const int64_t l = iv.probe[qi * iv.nprobe + pr];
      const bool ok = l >= 0 && guard_ok(l < iv.nlist, iv.err, GUARD_PROBE_LIST);
      lo = ok ? iv.list_off[l] : 0;
      hi = ok ? iv.list_off[l + 1] : 0;
    }
    for (int64_t base = lo; base < hi; base += 256) {
      const int64_t pp = base + tid;  // position (== id for a flat index)
      const int64_t i = pp < hi ? (iv.pos2id ? iv.pos2id[pp] : pp) : nb;
      const int cnt = s_cnt;
      const double tg = g[k - 1];
      const int64_t tidx = id[k - 1];
      if (pp < hi) {
        const double s = exact_score(qs, xb + i * d, d, l2 != 0);
        const double gv = l2 ? -s : s;
        if (cnt < k || better(gv, i, tg, tidx)) {
          const int pos = atomicAdd(&s_nst, 1);
          g[k + pos] = gv;
          id[k + pos] = i;
        }
      }
      __syncthreads();
      const int nst = s_nst;
      if (nst > 0) {
        block_bitonic_sort(g, id, P);
        for (int j = k + tid; j < P; j += 256) {
          g[j] = -INFINITY;
          id[j] = INT64_MAX;
        }
        __syncthreads();
        if (tid == 0) {
          s_cnt = cnt + nst < k ? cnt + nst : k;
          s_nst = 0;
        }
      }
      __syncthreads();
    }
    }
    for (int j = tid; j < k; j += 256) {
      const int64_t o = qi * k + j;
      const bool valid = id[j] != INT64_MAX;
      const double s = valid ? (l2 ? -g[j] : g[j]) : (l2 ? DBL_MAX : -DBL_MAX);
      D[o] = valid ? (float)s : (l2 ? FLT_MAX : -FLT_MAX);
      I[o] = valid ? id[j] + id_offset : -1;
      if (S) S[o] = s;
    }
    __syncthreads();
  }
}

// ============================================================ small corpus ==
// Exact search over a SMALL corpus (nb <= SMALL_NB: the coarse quantizer's
// centroids, k-means assignment, IndexIVFFlat.add): the (query, item) scores
// are computed EXACTLY in fp64 with the oracle's operation order (sequential d,
// fma) as a 64 x 64 tile GEMM on the VALU — one tile per workgroup, a 4 x 4
// register micro-tile per thread, f32 operands staged d-major through LDS —
// so no certificate is needed.  k = 1 fuses the arg-best into the tile loop
// (a workgroup walks all items for its 64 queries); larger k writes the
// goodness matrix of a query chunk and selects per query with a block bitonic
// sort (P = pow2ceil(nb) <= SMALL_NB entries in LDS).
constexpr int SM_T = 64;          // queries and items per tile
constexpr int SM_DC = 32;         // dimensions staged per LDS step
constexpr int SM_LD = SM_T + 4;   // LDS row stride (floats): conflict-light transposed stores
constexpr int SMALL_NB = 4096;
constexpr int64_t EXACT_BELOW = 16384;  // nb in (SMALL_NB, EXACT_BELOW): block-per-query fp64 scan

template <bool L2>
__device__ __forceinline__ void small_tile(const float* __restrict__ xq, int64_t q0, int64_t nq,
                                           const float* __restrict__ xb, int64_t j0, int64_t nb, int d,
                                           float* __restrict__ Qs, float* __restrict__ Xs, double (&acc)[4][4]) {
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = 0.0;
  for (int dc = 0; dc < d; dc += SM_DC) {
    const int w = d - dc < SM_DC ? d - dc : SM_DC;
    __syncthreads();  // previous step's readers are done
#pragma unroll
    for (int u = 0; u < (SM_T * SM_DC) / 256; ++u) {
      const int e = tid + u * 256;
      const int r = e / SM_DC, c = e % SM_DC;  // consecutive threads: consecutive dims of one row
      const int64_t qi = q0 + r, xi = j0 + r;
      Qs[c * SM_LD + r] = (c < w && qi < nq) ? xq[qi * d + dc + c] : 0.f;
      Xs[c * SM_LD + r] = (c < w && xi < nb) ? xb[xi * d + dc + c] : 0.f;
    }
    __syncthreads();
    for (int j = 0; j < w; ++j) {
      const float4 qv = *reinterpret_cast<const float4*>(Qs + j * SM_LD + ty * 4);
      const float4 xv = *reinterpret_cast<const float4*>(Xs + j * SM_LD + tx * 4);
      const double qd[4] = {(double)qv.x, (double)qv.y, (double)qv.z, (double)qv.w};
      const double xd[4] = {(double)xv.x, (double)xv.y, (double)xv.z, (double)xv.w};
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (L2) {
            const double t = qd[r] - xd[c];
            acc[r][c] = fma(t, t, acc[r][c]);
          } else {
            acc[r][c] = fma(qd[r], xd[c], acc[r][c]);
          }
        }
    }
  }
}

// k = 1: grid = query tiles; each workgroup walks every item tile.
template <bool L2>
__global__ __launch_bounds__(256) void small_best_kernel(const float* __restrict__ xq, int64_t nq,
                                                         const float* __restrict__ xb, int64_t nb, int d,
                                                         float* __restrict__ D, int64_t* __restrict__ I,
                                                         double* __restrict__ S, int64_t id_offset,
                                                         int32_t* __restrict__ nfb) {
  __shared__ __attribute__((aligned(16))) float Qs[SM_DC * SM_LD];
  __shared__ __attribute__((aligned(16))) float Xs[SM_DC * SM_LD];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  if (nfb && blockIdx.x == 0 && tid < 2) nfb[tid] = 0;  // n_fallback: the exact path answers every query
  const int64_t q0 = (int64_t)blockIdx.x * SM_T;
  double bg[4];
  int64_t bi[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    bg[r] = -INFINITY;
    bi[r] = INT64_MAX;
  }
  for (int64_t j0 = 0; j0 < nb; j0 += SM_T) {
    double acc[4][4];
    small_tile<L2>(xq, q0, nq, xb, j0, nb, d, Qs, Xs, acc);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t j = j0 + tx * 4 + c;
      if (j < nb) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double g = L2 ? -acc[r][c] : acc[r][c];
          if (better(g, j, bg[r], bi[r])) {
            bg[r] = g;
            bi[r] = j;
          }
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {  // arg-best over the 16 lanes sharing these rows
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      const double og = __shfl_xor(bg[r], o, 64);
      const int64_t oi = __shfl_xor(bi[r], o, 64);
      if (better(og, oi, bg[r], bi[r])) {
        bg[r] = og;
        bi[r] = oi;
      }
    }
    const int64_t qi = q0 + ty * 4 + r;
    if (tx == 0 && qi < nq) {
      const bool valid = bi[r] != INT64_MAX;
      const double sc = valid ? (L2 ? -bg[r] : bg[r]) : (L2 ? DBL_MAX : -DBL_MAX);
      D[qi] = valid ? (float)sc : (L2 ? FLT_MAX : -FLT_MAX);
      I[qi] = valid ? bi[r] + id_offset : -1;
      if (S) S[qi] = sc;
    }
  }
}

// k > 1, pass 1: goodness G[q - q0][j] for one query chunk; grid = (item tiles, query tiles).
template <bool L2>
__global__ __launch_bounds__(256) void small_scores_kernel(const float* __restrict__ xq, int64_t q0, int64_t nq,
                                                           const float* __restrict__ xb, int64_t nb, int d,
                                                           double* __restrict__ G, int64_t ldg) {
  __shared__ __attribute__((aligned(16))) float Qs[SM_DC * SM_LD];
  __shared__ __attribute__((aligned(16))) float Xs[SM_DC * SM_LD];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int64_t j0 = (int64_t)blockIdx.x * SM_T;
  const int64_t qt = q0 + (int64_t)blockIdx.y * SM_T;
  double acc[4][4];
  small_tile<L2>(xq, qt, nq, xb, j0, nb, d, Qs, Xs, acc);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t qi = qt + ty * 4 + r;
    if (qi >= nq) continue;
    double* row = G + (qi - q0) * ldg + j0 + tx * 4;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (j0 + tx * 4 + c < nb) row[c] = L2 ? -acc[r][c] : acc[r][c];
  }
}

// Few queries (nq < SM_T: the reference's one-profile-at-a-time loop,
// Retrieval.py:28-34): one thread per (query, item) instead of 64 x 64 tiles,
// so nb items spread over nb threads rather than over nb / 64 tile workgroups
// (small_best_kernel spent 188 us on one query over 300 centroids in one
// workgroup).  The arithmetic is small_tile's: fp64 over the dims in order,
// (q - x)^2 or q x fma'd into one accumulator, so the goodness is bit-identical.
template <bool L2>
__global__ __launch_bounds__(256) void small_rows_kernel(const float* __restrict__ xq, int64_t q0, int64_t nc,
                                                         const float* __restrict__ xb, int64_t nb, int d,
                                                         double* __restrict__ G, int64_t ldg) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= nc * nb) return;
  const int64_t ql = e / nb, j = e - ql * nb;
  const float* q = xq + (q0 + ql) * d;
  const float* x = xb + j * d;
  double acc = 0.0;
  int c = 0;
  if ((d & 3) == 0) {
    for (; c < d; c += 4) {
      const float4 qv = *reinterpret_cast<const float4*>(q + c);
      const float4 xv = *reinterpret_cast<const float4*>(x + c);
      const double qd[4] = {(double)qv.x, (double)qv.y, (double)qv.z, (double)qv.w};
      const double xd[4] = {(double)xv.x, (double)xv.y, (double)xv.z, (double)xv.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (L2) {
          const double t = qd[u] - xd[u];
          acc = fma(t, t, acc);
        } else {
          acc = fma(qd[u], xd[u], acc);
        }
      }
    }
  }
  for (; c < d; ++c) {
    const double qd = q[c], xd = x[c];
    if (L2) {
      const double t = qd - xd;
      acc = fma(t, t, acc);
    } else {
      acc = fma(qd, xd, acc);
    }
  }
  G[ql * ldg + j] = L2 ? -acc : acc;
}

// k > 1, pass 1 on 32 x 32 tiles (2 x 2 outputs per thread) where 64 x 64 tiles
// give the chip too few workgroups (the coarse quantizer: 4096 queries x 300
// centroids is 320 of them); the same fp64 arithmetic per output.
constexpr int S2_T = 32, S2_LD = S2_T + 2;
template <bool L2>
__global__ __launch_bounds__(256) void small_scores32_kernel(const float* __restrict__ xq, int64_t q0, int64_t nq,
                                                             const float* __restrict__ xb, int64_t nb, int d,
                                                             double* __restrict__ G, int64_t ldg) {
  __shared__ __attribute__((aligned(16))) float Qs[SM_DC * S2_LD];
  __shared__ __attribute__((aligned(16))) float Xs[SM_DC * S2_LD];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int64_t j0 = (int64_t)blockIdx.x * S2_T;
  const int64_t qt = q0 + (int64_t)blockIdx.y * S2_T;
  double acc[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
  for (int dc = 0; dc < d; dc += SM_DC) {
    const int w = d - dc < SM_DC ? d - dc : SM_DC;
    __syncthreads();  // previous step's readers are done
#pragma unroll
    for (int u = 0; u < (S2_T * SM_DC) / 256; ++u) {
      const int e = tid + u * 256;
      const int r = e / SM_DC, c = e % SM_DC;
      const int64_t qi = qt + r, xi = j0 + r;
      Qs[c * S2_LD + r] = (c < w && qi < nq) ? xq[qi * d + dc + c] : 0.f;
      Xs[c * S2_LD + r] = (c < w && xi < nb) ? xb[xi * d + dc + c] : 0.f;
    }
    __syncthreads();
    for (int j = 0; j < w; ++j) {
      const float2 qv = *reinterpret_cast<const float2*>(Qs + j * S2_LD + ty * 2);
      const float2 xv = *reinterpret_cast<const float2*>(Xs + j * S2_LD + tx * 2);
      const double qd[2] = {(double)qv.x, (double)qv.y};
      const double xd[2] = {(double)xv.x, (double)xv.y};
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          if (L2) {
            const double t = qd[r] - xd[c];
            acc[r][c] = fma(t, t, acc[r][c]);
          } else {
            acc[r][c] = fma(qd[r], xd[c], acc[r][c]);
          }
        }
    }
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int64_t qi = qt + ty * 2 + r;
    if (qi >= nq) continue;
    double* row = G + (qi - q0) * ldg + j0 + tx * 2;
#pragma unroll
    for (int c = 0; c < 2; ++c)
      if (j0 + tx * 2 + c < nb) row[c] = L2 ? -acc[r][c] : acc[r][c];
  }
}

// k > 1, pass 2: one workgroup per query of the chunk sorts its nb goodness values.
__global__ __launch_bounds__(256) void small_select_kernel(const double* __restrict__ G, int64_t ldg, int64_t q0,
                                                           int64_t nq, int64_t nb, int k, int l2, int P,
                                                           float* __restrict__ D, int64_t* __restrict__ I,
                                                           double* __restrict__ S, int64_t id_offset,
                                                           int32_t* __restrict__ nfb) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* g = reinterpret_cast<double*>(smem);
  int64_t* id = reinterpret_cast<int64_t*>(g + P);
  if (nfb && blockIdx.x == 0 && threadIdx.x < 2) nfb[threadIdx.x] = 0;
  const int64_t qi = q0 + blockIdx.x;
  if (qi >= nq) return;
  const double* row = G + (int64_t)blockIdx.x * ldg;
  for (int i = threadIdx.x; i < P; i += 256) {
    const bool ok = i < nb;
    g[i] = ok ? row[i] : -INFINITY;
    id[i] = ok ? (int64_t)i : INT64_MAX;
  }
  __syncthreads();
  block_bitonic_sort(g, id, P);
  for (int j = threadIdx.x; j < k; j += 256) {
    const int64_t o = qi * k + j;
    const bool valid = j < P && id[j] != INT64_MAX;
    const double sc = valid ? (l2 ? -g[j] : g[j]) : (l2 ? DBL_MAX : -DBL_MAX);
    D[o] = valid ? (float)sc : (l2 ? FLT_MAX : -FLT_MAX);
    I[o] = valid ? id[j] + id_offset : -1;
    if (S) S[o] = sc;
  }
}

// k <= SW_K and nb <= 64 * VPL (the coarse quantizer: nlist centroids, k =
// nprobe): one wave per query, VPL goodness values per lane in registers, k
// rounds of wave argmax in the bitonic sort's order (goodness descending, id
// ascending).  A block sort per query spends most of its time in barriers.
constexpr int SW_K = 64;
// (value, index) argmax over the wave, every lane receiving the winner: larger
// value first, ties -> lower index (a total order, so any combining tree picks
// the same winner).  DPP row ops and the CDNA4 permlane swaps instead of
// __shfl_xor, which moves each 32-bit half through a ds_bpermute round trip (18
// dependent LDS trips per selection round: 46 us for 4096 queries at k = 32).
__device__ __forceinline__ void am_take(double& v, int& i, double ov, int oi) {
  // bitwise | and & (no short circuit): the compiler otherwise branches on exec
  // masks at every step (two s_cbranch per step, ~39 us for 4096 queries at k = 32)
  const bool t = (ov > v) | ((ov == v) & (oi < i));
  v = t ? ov : v;
  i = t ? oi : i;
}
template <int CTRL>
__device__ __forceinline__ void am_dpp(double& v, int& i) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, true);
  const int oi = __builtin_amdgcn_mov_dpp(i, CTRL, 0xf, 0xf, true);
  am_take(v, i, __hiloint2double(hi, lo), oi);
}
__device__ __forceinline__ void am_swap(double& v, int& i, bool half32) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const auto rl = half32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                         : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto rh = half32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                         : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const auto ri = half32 ? __builtin_amdgcn_permlane32_swap(i, i, false, false)
                         : __builtin_amdgcn_permlane16_swap(i, i, false, false);
  double a = __hiloint2double((int)rh[0], (int)rl[0]);
  int ia = (int)ri[0];
  am_take(a, ia, __hiloint2double((int)rh[1], (int)rl[1]), (int)ri[1]);
  v = a;
  i = ia;
}
__device__ __forceinline__ void wave_argmax(double& v, int& i) {
  am_dpp<0xB1>(v, i);   // quad_perm [1,0,3,2]
  am_dpp<0x4E>(v, i);   // quad_perm [2,3,0,1]
  am_dpp<0x141>(v, i);  // row_half_mirror
  am_dpp<0x140>(v, i);  // row_mirror
  am_swap(v, i, false); // rows 2k <-> 2k+1
  am_swap(v, i, true);  // halves
}
template <int VPL>
__global__ __launch_bounds__(256) void small_select_wave_kernel(const double* __restrict__ G, int64_t ldg, int64_t q0,
                                                                int64_t nc, int64_t nq, int64_t nb, int k, int l2,
                                                                float* __restrict__ D, int64_t* __restrict__ I,
                                                                double* __restrict__ S, int64_t id_offset,
                                                                int32_t* __restrict__ nfb) {
  const int lane = threadIdx.x & 63;
  if (nfb && blockIdx.x == 0 && threadIdx.x < 2) nfb[threadIdx.x] = 0;
  const int64_t ql = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t qi = q0 + ql;
  if (ql >= nc || qi >= nq) return;
  const double* row = G + ql * ldg;
  double v[VPL];
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int64_t i = (int64_t)j * 64 + lane;
    v[j] = i < nb ? row[i] : -INFINITY;
  }
  for (int r = 0; r < k; ++r) {
    // the lane's best (an extracted entry reads -inf; it can only win once no
    // real item is left, i.e. r >= nb): first item, then strictly greater, so
    // the lowest index wins ties
    double bv = -INFINITY;
    int bj = VPL;
#pragma unroll
    for (int j = 0; j < VPL; ++j)
      if (((int64_t)j * 64 + lane < nb) & ((bj == VPL) | (v[j] > bv))) {
        bv = v[j];
        bj = j;
      }
    int bi = bj < VPL ? bj * 64 + lane : INT_MAX;
    wave_argmax(bv, bi);
    const bool valid = r < nb && bi != INT_MAX;
    if (valid && lane == (bi & 63)) {
#pragma unroll
      for (int j = 0; j < VPL; ++j)
        if (j == (bi >> 6)) v[j] = -INFINITY;
    }
    if (lane == 0) {
      const int64_t o = qi * k + r;
      const double sc = valid ? (l2 ? -bv : bv) : (l2 ? DBL_MAX : -DBL_MAX);
      D[o] = valid ? (float)sc : (l2 ? FLT_MAX : -FLT_MAX);
      I[o] = valid ? (int64_t)bi + id_offset : -1;
      if (S) S[o] = sc;
    }
  }
}

// ========================================================= tiled fallback ==
// Chip-wide fp64 scan for the fallback slots: 64-row fp32 tiles staged in LDS
// (row stride d+1, so lane = row reads are bank-conflict free), each wave
// scores its tile against slots w, w+4, ... (the query pointer is wave-uniform)
// with exact_score, and keeps the items at least as good as the slot's
// threshold.  Cost = slots x nb x d fp64 FMA, spread over every CU.
constexpr int FB_TR = 64;
constexpr int FB_SLOTS_MAX = 16384;  // collect slots per round / tiled-fallback slots per search

__global__ __launch_bounds__(256) void fallback_scan_kernel(const float* __restrict__ xq,
                                                            const float* __restrict__ xb, int64_t nb, int d,
                                                            int l2, FbState fb, double* __restrict__ cand_g,
                                                            int64_t* __restrict__ cand_i, int cap, IvfFb iv) {
  extern __shared__ float tile[];
  const int c0 = *fb.count;
  const int cnt = c0 < fb.slots ? c0 : fb.slots;
  if (cnt == 0) return;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int ds = d + 1;
  const int64_t ntiles = cdiv(nb, (int64_t)FB_TR);
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t r0 = t * FB_TR;
    const int rows = nb - r0 < FB_TR ? (int)(nb - r0) : FB_TR;
    __syncthreads();
    if (iv.pos2id) {  // IVF: gather rows by id
      for (int e = threadIdx.x; e < rows * d; e += 256) {
        const int r = e / d;
        tile[r * ds + (e - r * d)] = xb[iv.pos2id[r0 + r] * d + (e - r * d)];
      }
    } else if ((d & 3) == 0) {  // 16 float4 loads in flight per thread (one latency per tile)
      const float4* src = reinterpret_cast<const float4*>(xb + r0 * d);
      const int n4 = (rows * d) >> 2;
      for (int e0 = threadIdx.x; e0 < n4; e0 += 256 * 16) {
        float4 v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int e = e0 + u * 256;
          if (e < n4) v[u] = src[e];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int e = e0 + u * 256;
          if (e < n4) {
            const int f = 4 * e, r = f / d;
            float* o = tile + r * ds + (f - r * d);
            o[0] = v[u].x;
            o[1] = v[u].y;
            o[2] = v[u].z;
            o[3] = v[u].w;
          }
        }
      }
    } else {
      for (int e = threadIdx.x; e < rows * d; e += 256) {
        const int r = e / d;
        tile[r * ds + (e - r * d)] = xb[r0 * d + e];
      }
    }
    __syncthreads();
    if (lane >= rows) continue;
    const float* row = tile + lane * ds;
    const int64_t item = iv.pos2id ? iv.pos2id[r0 + lane] : r0 + lane;
    const int mylist = iv.pos2id ? iv.pos2list[r0 + lane] : 0;
    for (int s = wv; s < cnt; s += 4) {
      const int qi = fb.list[s];
      if (iv.nq > 0 && !guard_ok((uint64_t)qi < (uint64_t)iv.nq, iv.err, GUARD_FB_QUERY)) continue;
      if (iv.pos2id) {
        bool member = false;
        for (int pr = 0; pr < iv.nprobe; ++pr) member |= iv.probe[(int64_t)qi * iv.nprobe + pr] == mylist;
        if (!member) continue;
      }
      const double acc = exact_score(xq + (int64_t)qi * d, row, d, l2 != 0);
      const double gv = l2 ? -acc : acc;
      const int64_t ti = fb.thr_i[s];
      if (item == ti || better(gv, item, fb.thr_g[s], ti)) {
        const int pos = atomicAdd(&fb.n[s], 1);
        if (pos < cap) {
          cand_g[(int64_t)s * cap + pos] = gv;
          cand_i[(int64_t)s * cap + pos] = item;
        }
      }
    }
  }
}

// Per slot: sort the collected candidates and write the top k.  Slots whose
// list overflowed (or that have no storage) go to the overflow list, which the
// block-per-query exact kernel finishes.
__global__ __launch_bounds__(256) void fallback_select_kernel(FbState fb, const double* __restrict__ cand_g,
                                                              const int64_t* __restrict__ cand_i, int cap, int k,
                                                              int l2, float* __restrict__ D, int64_t* __restrict__ I,
                                                              double* __restrict__ S, int64_t id_offset,
                                                              int* __restrict__ ov_list, int64_t nq,
                                                              int* __restrict__ err = nullptr) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* g = reinterpret_cast<double*>(smem);
  int64_t* id = reinterpret_cast<int64_t*>(g + pow2ceil(cap));  // the sort pads n up to a power of two
  const int cnt = *fb.count;
  const int tid = threadIdx.x;
  for (int s = blockIdx.x; s < cnt; s += gridDim.x) {
    const int qi = fb.list[s];
    if (!guard_ok((uint64_t)qi < (uint64_t)nq, err, GUARD_FB_QUERY)) continue;  // (block-uniform)
    const int n = s < fb.slots ? fb.n[s] : cap + 1;
    if (n > cap || n < k) {
      if (tid == 0) ov_list[atomicAdd(&fb.count[1], 1)] = qi;
      continue;
    }
    const int P = pow2ceil(n);
    for (int i = tid; i < P; i += 256) {
      g[i] = i < n ? cand_g[(int64_t)s * cap + i] : -INFINITY;
      id[i] = i < n ? cand_i[(int64_t)s * cap + i] : INT64_MAX;
    }
    __syncthreads();
    block_bitonic_sort(g, id, P);
    for (int j = tid; j < k; j += 256) {
      const int64_t o = (int64_t)qi * k + j;
      const double sc = l2 ? -g[j] : g[j];
      D[o] = (float)sc;
      I[o] = id[j] + id_offset;
      if (S) S[o] = sc;
    }
    __syncthreads();
  }
}

// ============================================================ shard merge ==
__global__ void topk_merge_kernel(const double* __restrict__ Sp, const int64_t* __restrict__ Ip, int nparts,
                                  int64_t nq, int k, int l2, float* __restrict__ D, int64_t* __restrict__ I,
                                  double* __restrict__ S) {
  const int64_t qi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (qi >= nq) return;
  int pos[16];
  for (int p = 0; p < nparts; ++p) pos[p] = 0;
  for (int j = 0; j < k; ++j) {
    int best = -1;
    double bg = 0.0;
    int64_t bi = 0;
    for (int p = 0; p < nparts; ++p) {
      if (pos[p] >= k) continue;
      const int64_t o = ((int64_t)p * nq + qi) * k + pos[p];
      const int64_t ii = Ip[o];
      if (ii < 0) continue;
      const double gv = l2 ? -Sp[o] : Sp[o];
      if (best < 0 || better(gv, ii, bg, bi)) {
        best = p;
        bg = gv;
        bi = ii;
      }
    }
    const int64_t oo = qi * k + j;
    if (best < 0) {
      D[oo] = l2 ? FLT_MAX : -FLT_MAX;
      I[oo] = -1;
      if (S) S[oo] = l2 ? DBL_MAX : -DBL_MAX;
    } else {
      const double s = l2 ? -bg : bg;
      D[oo] = (float)s;
      I[oo] = bi;
      if (S) S[oo] = s;
      pos[best]++;
    }
  }
}

// ============================================================== IVF-Flat ==
// faiss IndexIVFFlat.search (BASELINE configs[3]; the inverted lists of
// Retrieval.py:21-23).  The caller supplies the probed lists (the coarse
// quantizer's top-nprobe, a flat search over the centroids).  List-major
// batching: every (query, probe) pair is grouped under its list, each list's
// probing queries are gathered into a padded bf16 segment, and the screen
// kernel (MODE 2) runs (list, query tile, list chunk) work items, so each list
// chunk is streamed once per 32*QT*WAVES queries.  Merge, certificate and the
// exact fallback are the flat path's, restricted to the probed lists.

__global__ void ivf_count_kernel(const int64_t* __restrict__ probe, int64_t npairs, int nlist, int* __restrict__ cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npairs) return;
  const int64_t l = probe[i];
  if (l >= 0 && l < nlist) atomicAdd(&cnt[l], 1);
}

// Contention-free grouping (nlist <= GROUP_LDS_LISTS): GROUP_BLOCKS blocks
// each count their slice of the (query, probe) pairs per list in LDS and write
// one histogram row; the plan kernel turns the rows into per-block offsets; the
// placing blocks re-read their slice and rank inside the block with LDS
// atomics.  (One global atomic per pair on a few hundred list counters cost
// ~50 us per grouping at 131K pairs.)  The order of a list's queries inside its
// segment is arbitrary: every consumer is order-independent.
constexpr int GROUP_BLOCKS = 64;
constexpr int GROUP_LDS_LISTS = 16384;

__global__ __launch_bounds__(1024) void ivf_hist_kernel(const int64_t* __restrict__ probe, int64_t npairs, int nlist,
                                                        int* __restrict__ H) {
  extern __shared__ int hist[];
  for (int l = threadIdx.x; l < nlist; l += blockDim.x) hist[l] = 0;
  __syncthreads();
  const int64_t per = cdiv(npairs, (int64_t)gridDim.x);
  const int64_t i0 = (int64_t)blockIdx.x * per, i1 = i0 + per < npairs ? i0 + per : npairs;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const int64_t l = probe[i];
    if (l >= 0 && l < nlist) atomicAdd(&hist[l], 1);
  }
  __syncthreads();
  for (int l = threadIdx.x; l < nlist; l += blockDim.x) H[(int64_t)blockIdx.x * nlist + l] = hist[l];
}

__global__ __launch_bounds__(1024) void ivf_place_kernel(const int64_t* __restrict__ probe, int64_t npairs, int nlist,
                                                         const int* __restrict__ seg_off, const int* __restrict__ H,
                                                         int* __restrict__ slot_pair) {
  extern __shared__ int base[];
  for (int l = threadIdx.x; l < nlist; l += blockDim.x) base[l] = seg_off[l] + H[(int64_t)blockIdx.x * nlist + l];
  __syncthreads();
  const int64_t per = cdiv(npairs, (int64_t)gridDim.x);
  const int64_t i0 = (int64_t)blockIdx.x * per, i1 = i0 + per < npairs ? i0 + per : npairs;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const int64_t l = probe[i];
    if (l >= 0 && l < nlist) slot_pair[atomicAdd(&base[l], 1)] = (int)i;
  }
}

// One block: per-list query segments (padded to wq rows) and work-item prefix.
// With H (the histogram rows of ivf_hist_kernel), the per-list counts are
// first summed over the GB rows, which become exclusive per-block offsets.
__global__ __launch_bounds__(1024) void ivf_plan_kernel(int* __restrict__ cnt,
                                                        const int64_t* __restrict__ list_off, int nlist, int wq,
                                                        int ch, int* __restrict__ seg_off, int* __restrict__ work_off,
                                                        int* __restrict__ fill, int* __restrict__ H = nullptr,
                                                        int GB = 0) {
  __shared__ int s_seg[1024], s_work[1024];
  const int t = threadIdx.x;
  const int per = (nlist + 1023) / 1024;
  const int lo = t * per < nlist ? t * per : nlist, hi = lo + per < nlist ? lo + per : nlist;
  if (H) {
    for (int l = lo; l < hi; ++l) {
      int run = 0;
      for (int b0 = 0; b0 < GB; b0 += 16) {  // 16 loads in flight
        int v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = b0 + u < GB ? H[(int64_t)(b0 + u) * nlist + l] : 0;
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (b0 + u < GB) {
            H[(int64_t)(b0 + u) * nlist + l] = run;
            run += v[u];
          }
      }
      cnt[l] = run;  // read back below by this same thread
    }
  }
  int ss = 0, sw = 0;
  for (int l = lo; l < hi; ++l) {
    const int rows = (cnt[l] + wq - 1) / wq * wq;
    const int nchl = (int)cdiv(list_off[l + 1] - list_off[l], (int64_t)ch);
    ss += rows;
    sw += rows / wq * nchl;
  }
  s_seg[t] = ss;
  s_work[t] = sw;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int a = t >= o ? s_seg[t - o] : 0, b = t >= o ? s_work[t - o] : 0;
    __syncthreads();
    s_seg[t] += a;
    s_work[t] += b;
    __syncthreads();
  }
  int es = s_seg[t] - ss, ew = s_work[t] - sw;
  for (int l = lo; l < hi; ++l) {
    const int rows = (cnt[l] + wq - 1) / wq * wq;
    const int nchl = (int)cdiv(list_off[l + 1] - list_off[l], (int64_t)ch);
    seg_off[l] = es;
    work_off[l] = ew;
    fill[l] = 0;
    es += rows;
    ew += rows / wq * nchl;
  }
  if (t == 1023) {
    seg_off[nlist] = s_seg[1023];
    work_off[nlist] = s_work[1023];
  }
}

__global__ void ivf_scatter_kernel(const int64_t* __restrict__ probe, int64_t npairs, int nlist,
                                   const int* __restrict__ seg_off, int* __restrict__ fill,
                                   int* __restrict__ slot_pair) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npairs) return;
  const int64_t l = probe[i];
  if (l < 0 || l >= nlist) return;
  slot_pair[seg_off[l] + atomicAdd(&fill[l], 1)] = (int)i;
}

// gathered query rows: one wave per slot row (padding rows are zeroed), a
// grid-stride loop over the rows the grouping produced (seg_off[nlist]; a grid
// sized for the upper bound launched ~50K blocks of which most exited: 25 us)
constexpr int GATHER_BLOCKS = 2048;
__global__ void ivf_gather_kernel(const uint16_t* __restrict__ qh, int dp, int nprobe,
                                  const int* __restrict__ slot_pair, const int* __restrict__ seg_off, int nlist,
                                  int64_t max_rows, uint16_t* __restrict__ qh_ivf, int64_t npairs,
                                  int* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int64_t nrows = seg_off[nlist] < max_rows ? seg_off[nlist] : max_rows;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); row < nrows; row += nw) {
    int pair = slot_pair[row];
    if (pair >= 0 && !guard_ok(pair < npairs, err, GUARD_GATHER_PAIR)) pair = -1;
    const int64_t q = pair >= 0 ? pair / nprobe : 0;
    for (int j = lane * 4; j < dp; j += 256) {
      uint2 v = make_uint2(0u, 0u);
      if (pair >= 0) v = *reinterpret_cast<const uint2*>(qh + q * dp + j);
      *reinterpret_cast<uint2*>(qh_ivf + row * dp + j) = v;
    }
  }
}

// Collect threshold in screened units.  e_k is the exact goodness of a real
// item ranked k-th among exactly scored real items, so the true k-th best is at
// least e_k; every true top-k item x then has screened(x) >= exact(x) - B_q >=
// e_k - B_q (IP), resp. screened = 2 q^.x^ - |x|^2 >= e_k + |q|^2 - B_q (L2,
// goodness = -|q - x|^2), with the flat certificate's error bound B_q.  Rounded
// down to f32 with slack for the fp64 evaluation of the bound itself.
__device__ __forceinline__ float collect_threshold(double ek, const double* __restrict__ qm,
                                                   const float* __restrict__ stats, int dp, int l2) {
  const double nqh = qm[0], nrq = qm[1], qn2 = qm[2];
  const double Xh = stats[0], Rr = stats[1], NX = stats[2];
  const double gam = (double)dp * 0x1p-22;
  const double bip = gam * nqh * Xh + nqh * Rr + nrq * Xh + nrq * Rr;
  // L2: + dp 2^-23 NX for screens whose accumulators start at -|x|^2 / 2
  // (screen16_collect_kernel): up to dp fp32 roundings of a running value that
  // holds half the row norm, doubled with the score
  const double B = l2 ? 2.0 * bip + 0x1p-21 * (NX + nqh * Xh) + (double)dp * 0x1p-23 * NX : bip;
  double t = (l2 ? qn2 + ek : ek) - B;
  t -= 1e-9 * (fabs(t) + fabs(ek) + qn2 + B);
  float f = (float)t;
  if ((double)f > t) f = nextafterf(f, -INFINITY);
  return f < -FLT_MAX ? -FLT_MAX : f;
}

// IVF phase A seed: exact rescoring of the R best lane maxima of the nearest
// list (distinct real items) -> e_k = their k-th best exact (goodness, id),
// a lower bound on the true k-th best s_k.  Every true top-k item x then has
// screened(x) >= exact(x) - B >= e_k - B =: T (screened units, rounded down;
// same error bound B_q as the flat certificate), and (e_k, id) is the
// fallback threshold.  Fewer than k seeds: the query goes to the fallback.
__global__ __launch_bounds__(64) void ivf_seed_kernel(const int* __restrict__ seed_pos, int R, int k,
                                                       const int64_t* __restrict__ pos2id,
                                                       const float* __restrict__ xq, const float* __restrict__ xb,
                                                       int d, int l2, const double* __restrict__ qmeta,
                                                       const float* __restrict__ stats, int dp,
                                                       float* __restrict__ thr, double* __restrict__ lb_g,
                                                       int64_t* __restrict__ lb_i, int* __restrict__ cand_cnt,
                                                       int cap, int64_t n, int* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int q = blockIdx.x, tid = threadIdx.x;
  const int P = pow2ceil(R);
  double* g = reinterpret_cast<double*>(smem);
  int64_t* id = reinterpret_cast<int64_t*>(g + P);
  float* qs = reinterpret_cast<float*>(id + P);
  __shared__ int s_valid;
  if (tid == 0) s_valid = 0;
  // one wave per query (a 256-thread block idled 7/8 of its lanes and paid the
  // sort's barriers across four waves)
  for (int i = tid; i < d; i += blockDim.x) qs[i] = xq[(int64_t)q * d + i];
  __syncthreads();
  for (int i = tid; i < P; i += blockDim.x) {
    const int pos = i < R ? seed_pos[(int64_t)q * R + i] : -1;
    if (pos >= 0 && guard_ok(pos < n, err, GUARD_SEED_POS)) {
      const int64_t item = pos2id[pos];
      const double sc = exact_score(qs, xb + item * d, d, l2 != 0);
      g[i] = l2 ? -sc : sc;
      id[i] = item;
      atomicAdd(&s_valid, 1);
    } else {
      g[i] = -INFINITY;
      id[i] = INT64_MAX;
    }
  }
  __syncthreads();
  block_bitonic_sort(g, id, P);
  if (tid != 0) return;
  if (s_valid < k) {  // too few seeds for a bound: no collection, straight to the fallback
    thr[q] = INFINITY;
    lb_g[q] = -INFINITY;
    lb_i[q] = -1;
    cand_cnt[q] = cap + 1;
    return;
  }
  const double ek = g[k - 1];
  thr[q] = collect_threshold(ek, qmeta + 4 * q, stats, dp, l2);
  lb_g[q] = ek;
  lb_i[q] = id[k - 1];
}

// IVF phase B: exact rescoring of every collected candidate, top-k.  Queries
// whose buffer overflowed go to the fallback with threshold (e_k, id).
constexpr int CR_CW = 16;   // collect_rescore: columns per staging step
constexpr int CR_MIN = 64;  // ... staged from this many candidates
// dynamic LDS of collect_rescore_kernel for a candidate capacity and dimension
static size_t collect_rescore_smem(int cap, int d) {
  size_t p = 1;
  while (p < (size_t)cap) p <<= 1;
  return p * 16 + (size_t)((d + 3) & ~3) * 4 + (size_t)256 * (CR_CW + 4) * 4;
}

__global__ __launch_bounds__(256) void collect_rescore_kernel(
    const int* __restrict__ cand_cnt, const int* __restrict__ cand_pos, int cap, const int64_t* __restrict__ pos2id,
    const float* __restrict__ xq, const float* __restrict__ xb, int d, int k, int l2,
    const double* __restrict__ lb_g, const int64_t* __restrict__ lb_i, float* __restrict__ D,
    int64_t* __restrict__ I, double* __restrict__ S, int64_t id_offset, FbState fb, int64_t nq, int64_t n,
    int* __restrict__ err, const int* __restrict__ qlist = nullptr, const int* __restrict__ qcount = nullptr) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  // IVF: slot = query.  Flat collect pass: slot b holds query qlist[b], if any.
  const int sl = blockIdx.x;
  if (qlist && sl >= *qcount) return;
  const int qi = qlist ? qlist[sl] : sl;
  if (!guard_ok((uint64_t)qi < (uint64_t)nq, err, GUARD_FB_QUERY)) return;
  int c = cand_cnt[sl];
  if (!guard_ok(c >= 0, err, GUARD_CAND_COUNT)) c = 0;
  if (c > cap) {
    if (tid == 0) fb.push(qi, lb_g[sl], lb_i[sl]);
    return;
  }
  const int P = pow2ceil(c > 0 ? c : 1);
  double* g = reinterpret_cast<double*>(smem);
  int64_t* id = reinterpret_cast<int64_t*>(g + P);
  float* qs = reinterpret_cast<float*>(id + P);
  for (int i = tid; i < d; i += 256) qs[i] = xq[(int64_t)qi * d + i];
  const bool staged = (d & 3) == 0 && c >= CR_MIN;
  for (int i = tid; i < P; i += 256) {
    if (i < c) {
      const int pos = cand_pos[(int64_t)sl * cap + i];
      // an out-of-range position (a broken invariant) is flagged and read as row 0
      const int64_t p = guard_ok((uint64_t)pos < (uint64_t)n, err, GUARD_CAND_POS) ? pos : 0;
      id[i] = pos2id ? pos2id[p] : p;
    } else {
      g[i] = -INFINITY;
      id[i] = INT64_MAX;
    }
  }
  __syncthreads();
  if (staged) {
    // lane = candidate row, fp64 in the oracle's serial order; the rows are
    // staged through LDS CR_CW columns at a time by coalesced float4 loads
    // (one lane per candidate row reading it 4 B at a time left every load
    // instruction touching 256 different rows)
    float* stg = qs + ((d + 3) & ~3);  // [256][CR_CW + 4]
    for (int r0 = 0; r0 < c; r0 += 256) {
      const int nr = c - r0 < 256 ? c - r0 : 256;
      double acc = 0.0;
      for (int c0 = 0; c0 < d; c0 += CR_CW) {
        const int cw = d - c0 < CR_CW ? d - c0 : CR_CW;
#pragma unroll
        for (int t = 0; t < CR_CW / 4; ++t) {
          const int e = tid + 256 * t, row = e / (CR_CW / 4), c4 = e % (CR_CW / 4);
          if (row < nr && 4 * c4 < cw)
            *reinterpret_cast<float4*>(stg + row * (CR_CW + 4) + 4 * c4) =
                *reinterpret_cast<const float4*>(xb + id[r0 + row] * d + c0 + 4 * c4);
        }
        __syncthreads();
        if (tid < nr) {
          const float* xr = stg + tid * (CR_CW + 4);
          for (int j = 0; j < cw; j += 4) {
            const float4 v = *reinterpret_cast<const float4*>(xr + j);
            const float xv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              if (l2) {
                const double t = (double)qs[c0 + j + u] - (double)xv[u];
                acc = fma(t, t, acc);
              } else {
                acc = fma((double)qs[c0 + j + u], (double)xv[u], acc);
              }
            }
          }
        }
        __syncthreads();
      }
      if (tid < nr) g[r0 + tid] = l2 ? -acc : acc;
    }
  } else {
    for (int i = tid; i < c; i += 256) {
      const double sc = exact_score(qs, xb + id[i] * d, d, l2 != 0);
      g[i] = l2 ? -sc : sc;
    }
  }
  __syncthreads();
  block_bitonic_sort(g, id, P);
  for (int j = tid; j < k; j += 256) {
    const int64_t o = (int64_t)qi * k + j;
    const bool valid = j < c;
    const double sc = valid ? (l2 ? -g[j] : g[j]) : (l2 ? DBL_MAX : -DBL_MAX);
    D[o] = valid ? (float)sc : (l2 ? FLT_MAX : -FLT_MAX);
    I[o] = valid ? id[j] + id_offset : -1;
    if (S) S[o] = sc;
  }
}

// ====================================================== flat collect pass ==
// Queries the flat merge could not certify (dense neighbourhoods: the exact
// k-th best lies within the screening error bound of theta) get a second,
// exact-by-construction pass instead of an fp64 corpus scan: the IVF collect
// screen (MODE 3) over the whole corpus as ONE list, probed only by these
// queries, appends every item whose screened score reaches the query's collect
// threshold (from the merge's exact k-th e_k, collect_threshold), and
// collect_rescore ranks the candidates exactly.  Only a buffer overflow (more
// than `cap` items within the bound) goes on to the tiled fp64 fallback.
//
// Collect storage is indexed by slot s: round r of the pass takes the merge's
// fallback entries [r S, r S + S) (S = FB_SLOTS_MAX; every entry carries the
// merge's e_k), so any number of uncertified queries is collected in
// ceil(nq / S) rounds over the same fixed storage (a search of N x 4096
// queries against one corpus shard leaves more than S uncertified at L2).
// One block: turns this round's entries into the one-list work table
// (list_off, seg_off, work_off, slot_pair = s), the per-slot thresholds and
// the gathered bf16 query rows, and saves the slot -> query map for
// collect_rescore.  Queries whose candidates overflow the collect buffer go to
// the tiled fallback's own list (collect_rescore pushes them there).
__global__ __launch_bounds__(1024) void flat_collect_plan_kernel(
    FbState fb, int64_t nq, int64_t nb, int wq, int ch, const double* __restrict__ qmeta,
    const float* __restrict__ stats, int dp, int l2, int cap, int force_overflow, int round, int S,
    int64_t* __restrict__ list_off, int* __restrict__ seg_off, int* __restrict__ work_off, int* __restrict__ slot_pair,
    float* __restrict__ thr, double* __restrict__ lb_g, int64_t* __restrict__ lb_i, int* __restrict__ cand_cnt,
    int* __restrict__ clist, int* __restrict__ ccount, const uint16_t* __restrict__ qh, uint16_t* __restrict__ qc) {
  const int t = threadIdx.x, nt = blockDim.x;
  const int n = (int)min((int64_t)fb.count[0], nq);
  const int lo = round * S;
  const int nc = n - lo <= 0 ? 0 : (n - lo < S ? n - lo : S);  // this round's slots
  const int rows = (nc + wq - 1) / wq * wq;
  for (int s = t; s < rows; s += nt) slot_pair[s] = s < nc ? s : -1;
  for (int s = t; s < nc; s += nt) {
    const int q = fb.list[lo + s];
    clist[s] = q;
    const bool has = fb.thr_i[lo + s] >= 0;  // the merge rescored >= k candidates
    thr[s] = has ? collect_threshold(fb.thr_g[lo + s], qmeta + 4 * q, stats, dp, l2) : INFINITY;
    lb_g[s] = has ? fb.thr_g[lo + s] : -INFINITY;
    lb_i[s] = has ? fb.thr_i[lo + s] : -1;
    cand_cnt[s] = (has && !force_overflow) ? 0 : cap + 1;
  }
  if (t == 0) {
    list_off[0] = 0;
    list_off[1] = nb;
    seg_off[0] = 0;
    seg_off[1] = rows;
    work_off[0] = 0;
    work_off[1] = rows / wq * (int)cdiv(nb, (int64_t)ch);
    ccount[0] = nc;
    ccount[1] = n;  // queries the certificate did not cover (reported as n_fallback[0])
  }
  // the collected slots' bf16 query rows (padding rows zero): one wave per row
  for (int row = t >> 6; row < rows; row += nt >> 6) {
    const int64_t q = row < nc ? fb.list[lo + row] : -1;
    for (int j = (t & 63) * 4; j < dp; j += 256) {
      uint2 v = make_uint2(0u, 0u);
      if (q >= 0) v = *reinterpret_cast<const uint2*>(qh + q * dp + j);
      *reinterpret_cast<uint2*>(qc + (int64_t)row * dp + j) = v;
    }
  }
}

// ================================================================== plan ==
struct FlatPlan {
  bool exact_only, tau;
  bool cliff;  // exact_only forced by a shape the screen cannot plan (reported as nq fallbacks)
  bool small;  // nb <= SMALL_NB: exact fp64 tile GEMM (small_best / small_scores + small_select)
  int small_P;
  int64_t small_ld, small_chunk;
  int dp, qt, M, waves, wq, nqt, nch, U, KP;
  int R, nch_pre, tstride;  // threshold pre-pass: bound rank, chunks, tile stride
  int fb_slots, fb_cap;     // tiled fallback: slots with candidate storage, candidates per slot
  int64_t nq_pad, chunk, chunk_pre;
  size_t off_qh, off_qmeta, off_ps, off_pi, off_pt, off_fbl, off_fbc, off_tau, off_pre, total;
  size_t off_fbt, off_fbi, off_fbn, off_fcg, off_fci, off_ovl, off_tfl, off_tft, off_tfi;
  // collect pass for uncertified queries (flat_collect_plan_kernel)
  int cwq, cch, ccap, cgrid;
  int64_t crows;
  size_t off_clo, off_cseg, off_cwork, off_csp, off_cqi, off_cthr, off_clbg, off_clbi, off_ccnt, off_cpos, off_clist,
      off_ccount;
};

static int padded_dim(int d) {
  if (d <= 32) return 32;
  if (d <= 64) return 64;
  if (d <= 128) return 128;
  if (d <= 256) return 256;
  return (int)align_up((size_t)d, 32);
}

static int host_pow2ceil(int n) {
  int p = 1;
  while (p < n) p <<= 1;
  return p;
}

// Test hooks (tests/test_knn_gpu.py, tests/test_ivf_gpu.py) that drive the
// rare exact paths on ordinary data; nothing else reads the environment.
//   NRK_FORCE_FALLBACK=1  certify nothing (flat: the collect pass answers)
//   NRK_FORCE_FALLBACK=2  certify nothing and overflow every collect buffer
//                         (the tiled fp64 fallback answers)
//   NRK_FB_CAP=n          tiled-fallback candidates per slot (tiny: the
//                         block-per-query exact kernel answers)
//   NRK_SCREEN16=0        the 32x32x16 kernels for the flat inner-product main
//                         pass and the IVF collect (test_knn_gpu.py
//                         ::test_screen_main_pass_forms, test_ivf_gpu.py
//                         ::test_ivf_collect_forms)
static int test_hook(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}

static FlatPlan make_plan(int64_t nq, int64_t nb, int d, int k) {
  FlatPlan p;
  memset(&p, 0, sizeof(p));
  p.dp = padded_dim(d);
  if (nb <= SMALL_NB && k <= SMALL_NB && nq > 0) {  // exact fp64 tile GEMM, no screening
    p.small = true;
    p.exact_only = true;
    const int64_t P = host_pow2ceil(nb > 0 ? (int)nb : 1);
    p.small_ld = align_up((size_t)(nb > 0 ? nb : 1), SM_T);
    const int64_t want = ((int64_t)64 << 20) / (p.small_ld * 8);  // <= 64 MB of goodness per chunk
    p.small_chunk = want < SM_T ? SM_T : want / SM_T * SM_T;
    if (p.small_chunk > (int64_t)align_up((size_t)nq, SM_T)) p.small_chunk = align_up((size_t)nq, SM_T);
    p.small_P = (int)P;
    // (k = 1 with a full query tile: small_best_kernel, no goodness buffer)
    p.total = k == 1 && nq >= SM_T ? 256 : align_up((size_t)p.small_chunk * p.small_ld * 8, 256);
    return p;
  }
  p.exact_only = nb < EXACT_BELOW || d > 256 || k > 256 || nb >= (1ll << 31) || nq == 0;
  if (p.exact_only) {
    p.off_fbc = 0;
    p.total = 256;
    return p;
  }
  p.waves = 4;
  // M: per-lane list length.  tau: sampled pre-pass bound on the R-th best
  // screened score (R > k with margin), used while R stays small.
  if (k <= 8) { p.M = 4; p.qt = 2; }
  else if (k <= 24) { p.M = 8; p.qt = 1; }
  else { p.M = 16; p.qt = 1; }
  // DP = 256 with M = 4 or 16: 8-wave workgroups (256 queries per corpus pass):
  // half the LDS-DMA pieces per MFMA of the 4-wave form (10M x 256, k = 5:
  // screen 17.4 -> 15.0 ms) and, at k = 200, a chunk far larger than L2
  // re-read by half as many query tiles
  if (p.dp == 256 && (p.M == 4 || p.M == 16)) p.waves = 8;
  // R: tau bounds the R-th best screened score from the pre-pass's lane maxima
  // (every stride-th tile), so it sits near global rank ~stride * R; the main
  // pass then admits ~stride * R items per query (list insertions, the VALU
  // cost of the k = 200 screen).  k > 8: R = k / 4 and stride * R >= 4k (below
  // that a few queries per thousand are uncertified: 1M x 128 k = 100 at 2k:
  // 36 of 4096).  Measured at 10M x 256 k = 200 (stride 16): screen 19.05 ms at
  // R = 2k -> 16.83; 1.25M x 256, 32768 queries: total 38.4 -> 29.2 ms.
  // k <= 8: R = max(8, k + 3) (was 16; with the stride rule below it halves the
  // pre-pass and leaves stride * R, the admitted items, unchanged: 1M x 128
  // k = 5 total 1.055 -> 1.001 ms, L2 1.41 -> 1.27 ms, 10M x 256 16.66 -> 16.41
  // ms, 125K x 128 x 32768 queries 1.78 -> 1.64 ms; same results).
  p.R = k <= 8 ? (k + 3 > 8 ? k + 3 : 8) : (k / 4 > 16 ? k / 4 : 16);
  p.tau = true;  // k = 200 at 10M x 256: -5% retrieve time
  if (p.dp == 256) p.qt = 1;
  p.wq = p.waves * 32 * p.qt;
  p.nqt = (int)cdiv(nq, p.wq);
  p.nq_pad = (int64_t)p.nqt * p.wq;
  // k > 24 (M = 16): twice the lane streams, so that dense neighbourhoods do
  // not overflow a lane's list (10M x 256, k = 200: 2 uncertified queries per
  // 4096 -> 0, and the 4.5 ms fp64 fallback scan with them)
  // pre-pass stride: the pre-pass costs ~nb / stride per query, the main pass
  // admits ~stride * R items above tau per query (list insertions); the best
  // stride grows like sqrt(nb / R): the power of two >= 8 sqrt(nb/1M * 16/R),
  // in [2, 64] (and stride * R >= 4k, above).  Measured at R = 16 (IP, per
  // GPU): 1M x 128 k = 5 -> 8; 10M x 256 k = 5 -> 32 (total 17.0 -> 15.8 ms vs
  // 8); 125K x 128 k = 5, 32768 queries -> 4 (-7 %).  At R = 8 the same rule
  // gives 16, 64 and 8 (1M x 128: stride 16 1.001 ms, 32 1.026 ms)
  {
    const double want = 8.0 * sqrt((double)nb / 1e6 * 16.0 / p.R);
    int st = 2;
    while (st < 64 && st < want) st *= 2;
    if (k > 8)
      while (st < 64 && (int64_t)st * p.R < 4 * (int64_t)k) st *= 2;
    p.tstride = st;
  }
  int target = p.M >= 16 ? 2048 : 1024;
  int64_t nch = target / (p.nqt > 0 ? p.nqt : 1);
  // ... but at least enough chunks (2 lane streams each) that the ~stride * R
  // items above tau spread to <= M per stream: with many query tiles (a
  // corpus shard searched by N x 4096 queries) the workgroup target alone
  // left 16 streams per query and ~1/6 of the queries uncertified at k = 200
  const int64_t min_streams = cdiv((int64_t)p.tstride * p.R, (int64_t)2 * p.M);
  if (nch < min_streams) nch = min_streams;
  if (nch < 1) nch = 1;
  int64_t max_by_u = 2048 / (2 * p.M);
  if (nch > max_by_u) nch = max_by_u;
  int64_t max_by_len = cdiv(nb, 1024);
  if (nch > max_by_len) nch = max_by_len;
  if (nch < 1) nch = 1;
  // buffer descriptors address a chunk with 32-bit offsets: keep chunks < 1 GiB
  const int64_t min_nch = cdiv(nb * (int64_t)p.dp * 2, (int64_t)1 << 30);
  if (nch < min_nch) nch = min_nch;
  p.chunk = (int64_t)align_up((size_t)cdiv(nb, nch), 64);
  p.nch = (int)cdiv(nb, p.chunk);
  p.U = p.nch * 2 * p.M;
  if (p.U > 2048) {  // the merge holds the union in registers (8 entries per thread)
    p.exact_only = true;
    p.cliff = true;
    p.off_fbc = 0;
    p.total = 256;
    return p;
  }
  int kp = 2 * k > 32 ? 2 * k : 32;
  if (kp < k + 16) kp = k + 16;
  if (kp > p.U) kp = p.U;
  if (kp > 1024) kp = 1024;
  p.KP = kp;
  if (p.KP < k) {
    p.exact_only = true;
    p.cliff = true;
    p.off_fbc = 0;
    p.total = 256;
    return p;
  }
  // pre-pass: every tstride-th 64-item tile, chunks small enough that each
  // query gets >= 8R short lane streams (their maxima are distinct items), but
  // >= 8 visited tiles per workgroup (a small shard searched by many query
  // tiles otherwise launched thousands of 2-tile workgroups)
  {
    const int TI = 64;  // must equal screen_kernel TI
    int64_t tiles = cdiv(nb, TI);
    int64_t want = 4 * p.R;  // 2 lanes per chunk -> 8R streams
    const int64_t min_pre = cdiv(nb * (int64_t)p.dp * 2, (int64_t)1 << 30);
    if (want < min_pre) want = min_pre;
    if (want > 512) want = 512;
    int64_t maxc = cdiv(tiles, (int64_t)p.tstride * 8);
    if (want > maxc) want = maxc;
    if (want < 1) want = 1;
    p.chunk_pre = cdiv(cdiv(tiles, want), p.tstride) * p.tstride * TI;
    p.nch_pre = (int)cdiv(nb, p.chunk_pre);
    if (2 * p.nch_pre < p.R) p.tau = false;
  }
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off = align_up(off + bytes, 256);
    return o;
  };
  p.off_fbc = take(16);
  p.off_tau = take((size_t)nq * 4);
  p.off_pre = take((size_t)nq * p.nch_pre * 2 * 4);
  p.off_qh = take((size_t)p.nq_pad * p.dp * 2);
  p.off_qmeta = take((size_t)nq * 4 * 8);
  p.off_ps = take((size_t)nq * p.U * 4);
  p.off_pi = take((size_t)nq * p.U * 4);
  p.off_pt = take((size_t)nq * p.nch * 2 * 4);
  p.off_fbl = take((size_t)nq * 4);
  // Uncertified queries are collected in rounds of FB_SLOTS_MAX (16 K) slots,
  // as many rounds as nq needs (a corpus shard searched by N x 4096 queries
  // leaves more than 4096 of them uncertified at L2; queries beyond a fixed
  // slot budget used to take the block-per-query exact scan: 2.3 s for 574
  // queries over a 2.5M-row shard at world 4).  The tiled fp64 fallback then
  // takes the (rare) queries whose collect buffer overflowed, with storage for
  // candidates at least as good as the merge's k-th; its cap leaves room for
  // 2k + 64 (ties and near-ties), overflow goes to exact_topk.  Each slot holds
  // fb_cap x 16 B of fallback candidates and ccap x 4 B of collect positions
  // (16 KB at k <= 224), so the cap bounds this part of the workspace at 256 MB
  p.fb_slots = (int)(nq < FB_SLOTS_MAX ? nq : FB_SLOTS_MAX);
  p.fb_cap = host_pow2ceil(2 * k + 64);
  if (p.fb_cap < 512) p.fb_cap = 512;
  p.fb_cap = test_hook("NRK_FB_CAP", p.fb_cap);
  if (p.fb_cap < 1) p.fb_cap = 1;
  if (p.fb_cap > 8192) p.fb_cap = 8192;  // select kernel sorts cap x 16 B in LDS
  p.off_fbt = take((size_t)nq * 8);  // the merge's e_k of every uncertified query
  p.off_fbi = take((size_t)nq * 8);
  p.off_fbn = take((size_t)p.fb_slots * 4);
  p.off_fcg = take((size_t)p.fb_slots * p.fb_cap * 8);
  p.off_fci = take((size_t)p.fb_slots * p.fb_cap * 8);
  p.off_ovl = take((size_t)nq * 4);
  // the tiled fallback's own list (queries whose collect buffer overflowed)
  p.off_tfl = take((size_t)nq * 4);
  p.off_tft = take((size_t)p.fb_slots * 8);
  p.off_tfi = take((size_t)p.fb_slots * 8);
  // collect pass: one query tile per wave (128 queries per work item), 4096-row
  // chunks (each chunk's query tiles run back to back on one XCD), storage for
  // the fb_slots uncertified queries that carry an e_k
  p.cwq = 4 * 32;
  p.cch = 4096;
  p.ccap = 2048;
  p.crows = cdiv(p.fb_slots, p.cwq) * p.cwq;
  {
    const int64_t items = (p.crows / p.cwq) * cdiv(nb, (int64_t)p.cch);
    p.cgrid = (int)(items < 512 ? items : 512);  // two 4-wave blocks per CU fill the chip
  }
  p.off_clo = take(16);
  p.off_cseg = take(8);
  p.off_cwork = take(8);
  p.off_csp = take((size_t)p.crows * 4);
  p.off_cqi = take((size_t)p.crows * p.dp * 2);
  p.off_cthr = take((size_t)p.fb_slots * 4);
  p.off_clbg = take((size_t)p.fb_slots * 8);
  p.off_clbi = take((size_t)p.fb_slots * 8);
  p.off_ccnt = take((size_t)p.fb_slots * 4);
  p.off_cpos = take((size_t)p.fb_slots * p.ccap * 4);
  p.off_clist = take((size_t)p.fb_slots * 4);
  p.off_ccount = take(16);
  p.total = off;
  return p;
}

}  // namespace nrk

using namespace nrk;


static int small_launch(const FlatPlan& p, const float* xq, int64_t nq, const float* xb, int64_t nb, int d, int k,
                        int l2, float* D, int64_t* I, double* S, int64_t id_offset, void* ws, hipStream_t st,
                        int32_t* nfb) {
  if (k == 1 && nq >= SM_T) {
    const unsigned grid = (unsigned)cdiv(nq, SM_T);
    if (l2)
      hipLaunchKernelGGL(small_best_kernel<true>, dim3(grid), dim3(256), 0, st, xq, nq, xb, nb, d, D, I, S, id_offset,
                         nfb);
    else
      hipLaunchKernelGGL(small_best_kernel<false>, dim3(grid), dim3(256), 0, st, xq, nq, xb, nb, d, D, I, S,
                         id_offset, nfb);
    NRK_CHECK_LAUNCH("small_best_kernel");
    return NRK_OK;
  }
  double* G = static_cast<double*>(ws);
  const size_t smem = (size_t)p.small_P * 16;
  for (int64_t q0 = 0; q0 < nq; q0 += p.small_chunk) {
    const int64_t nc = nq - q0 < p.small_chunk ? nq - q0 : p.small_chunk;
    if (nb > 0 && nc < SM_T) {  // few queries: a thread per (query, item)
      const unsigned grid = (unsigned)cdiv(nc * nb, (int64_t)256);
      if (l2)
        hipLaunchKernelGGL(small_rows_kernel<true>, dim3(grid), dim3(256), 0, st, xq, q0, nc, xb, nb, d, G, p.small_ld);
      else
        hipLaunchKernelGGL(small_rows_kernel<false>, dim3(grid), dim3(256), 0, st, xq, q0, nc, xb, nb, d, G, p.small_ld);
      NRK_CHECK_LAUNCH("small_rows_kernel");
    } else if (nb > 0 && cdiv(nb, SM_T) * cdiv(nc, SM_T) < 1024) {  // few tiles: 32 x 32 ones
      const dim3 grid((unsigned)cdiv(nb, S2_T), (unsigned)cdiv(nc, S2_T));
      if (l2)
        hipLaunchKernelGGL(small_scores32_kernel<true>, grid, dim3(256), 0, st, xq, q0, nq, xb, nb, d, G, p.small_ld);
      else
        hipLaunchKernelGGL(small_scores32_kernel<false>, grid, dim3(256), 0, st, xq, q0, nq, xb, nb, d, G, p.small_ld);
      NRK_CHECK_LAUNCH("small_scores32_kernel");
    } else if (nb > 0) {
      const dim3 grid((unsigned)cdiv(nb, SM_T), (unsigned)cdiv(nc, SM_T));
      if (l2)
        hipLaunchKernelGGL(small_scores_kernel<true>, grid, dim3(256), 0, st, xq, q0, nq, xb, nb, d, G, p.small_ld);
      else
        hipLaunchKernelGGL(small_scores_kernel<false>, grid, dim3(256), 0, st, xq, q0, nq, xb, nb, d, G, p.small_ld);
      NRK_CHECK_LAUNCH("small_scores_kernel");
    }
    if (k <= SW_K && nb <= 1024) {
      const dim3 g4((unsigned)cdiv(nc, (int64_t)4));
      if (nb <= 256)
        hipLaunchKernelGGL(small_select_wave_kernel<4>, g4, dim3(256), 0, st, G, p.small_ld, q0, nc, nq, nb, k, l2, D,
                           I, S, id_offset, nfb);
      else if (nb <= 512)
        hipLaunchKernelGGL(small_select_wave_kernel<8>, g4, dim3(256), 0, st, G, p.small_ld, q0, nc, nq, nb, k, l2, D,
                           I, S, id_offset, nfb);
      else
        hipLaunchKernelGGL(small_select_wave_kernel<16>, g4, dim3(256), 0, st, G, p.small_ld, q0, nc, nq, nb, k, l2, D,
                           I, S, id_offset, nfb);
      NRK_CHECK_LAUNCH("small_select_wave_kernel");
    } else {
      hipLaunchKernelGGL(small_select_kernel, dim3((unsigned)nc), dim3(256), smem, st, G, p.small_ld, q0, nq, nb, k,
                         l2, p.small_P, D, I, S, id_offset, nfb);
      NRK_CHECK_LAUNCH("small_select_kernel");
    }
  }
  return NRK_OK;
}

static int exact_launch(const float* xq, int64_t nq, const float* xb, int64_t nb, int d, int k, int l2,
                        const int* qlist, const int* qcount, int64_t max_work, float* D, int64_t* I,
                        double* S, int64_t id_offset, hipStream_t st, IvfFb iv = IvfFb{},
                        int* cnt_out = nullptr, const int* cnt_a = nullptr, const int* cnt_b = nullptr) {
  const int P = host_pow2ceil(k + 256);
  const size_t smem = (size_t)P * 16 + (size_t)d * 4;
  if (smem > 160 * 1024) return fail(NRK_EUNSUPPORTED, "exact search: k=%d d=%d needs %zu B of LDS", k, d, smem);
  int grid = (int)(max_work < 2048 ? max_work : 2048);
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(exact_topk_kernel, dim3(grid), dim3(256), smem, st, xq, nq, xb, nb, d, k, l2, qlist, qcount,
                     D, I, S, id_offset, iv, cnt_out, cnt_a, cnt_b);
  NRK_CHECK_LAUNCH("exact_topk_kernel");
  return NRK_OK;
}

extern "C" int nrk_padded_dim(int32_t d) { return padded_dim(d); }

// The flat search's main-pass screen kernel for a plan.  Inner product: the
// 16x16x32 form where built (NRK_SCREEN16=0: the 32x32x16 kernel, which every
// other form runs; a test hook).
static screen_fn main_pass(const FlatPlan& p, bool l2, bool* s16) {
  *s16 = false;
  screen_fn fn = p.waves == 8 ? pick_screen_dp256_w8(p.M, l2, 0) : pick_screen(p.dp, p.qt, p.M, l2, 0);
  if (!l2 && test_hook("NRK_SCREEN16", 1)) {
    screen_fn f16 = p.waves == 8 ? (p.dp == 256 ? pick_screen16_dp256_w8(p.M) : nullptr)
                                 : (p.dp == 128 ? pick_screen16_dp128(p.qt, p.M) : nullptr);
    if (f16) {
      fn = f16;
      *s16 = true;
    }
  }
  return fn;
}

extern "C" int nrk_knn_flat_main_pass(int64_t nq, int64_t nb, int32_t d, int32_t k, int32_t metric, char* name,
                                      size_t len) {
  NRK_CHECK_ARG(name && len > 0 && nq >= 0 && nb >= 0 && d > 0 && k > 0, "knn_flat_main_pass: bad arguments");
  const FlatPlan p = make_plan(nq, nb, d, k);
  const bool l2 = metric == NRK_METRIC_L2;
  if (p.small) snprintf(name, len, "small_exact (fp64 tile GEMM, no screen)");
  else if (p.exact_only) snprintf(name, len, "exact_topk_kernel (fp64 brute force, no screen)");
  else {
    bool s16 = false;
    (void)main_pass(p, l2, &s16);
    snprintf(name, len, "%s<dp %d, qt %d, M %d, %d waves, %s> (bf16 v_mfma_f32_%s)", s16 ? "screen16_kernel" : "screen_kernel",
             p.dp, p.qt, p.M, p.waves, l2 ? "L2" : "IP", s16 ? "16x16x32" : "32x32x16");
  }
  return NRK_OK;
}

extern "C" int nrk_flat_prepare(const float* xb, int64_t nb, int32_t d, uint16_t* xb_bf16, float* xb_meta,
                                float* stats, void* stream) {
  NRK_CHECK_ARG(d > 0 && nb >= 0, "flat_prepare: bad shape nb=%lld d=%d", (long long)nb, d);
  if (nb == 0) return NRK_OK;
  NRK_CHECK_ARG(xb && xb_bf16 && xb_meta && stats, "flat_prepare: null pointer");
  const int dp = padded_dim(d);
  const int rows_per_block = 4;
  const int64_t blocks = cdiv(nb, rows_per_block) < 8192 ? cdiv(nb, rows_per_block) : 8192;
  hipLaunchKernelGGL(flat_prepare_kernel, dim3((unsigned)blocks), dim3(64 * rows_per_block), 0,
                     (hipStream_t)stream, xb, nb, d, dp, xb_bf16, xb_meta, stats);
  NRK_CHECK_LAUNCH("flat_prepare_kernel");
  return NRK_OK;
}

extern "C" int nrk_knn_flat_workspace(int64_t nq, int64_t nb, int32_t d, int32_t k, size_t* ws_bytes) {
  NRK_CHECK_ARG(ws_bytes && nq >= 0 && nb >= 0 && d > 0 && k > 0, "knn_flat_workspace: bad arguments");
  *ws_bytes = make_plan(nq, nb, d, k).total;
  return NRK_OK;
}

extern "C" int nrk_knn_exact(const float* xq, int64_t nq, const float* xb, int64_t nb, int32_t d, int32_t k,
                             int32_t metric, float* D, int64_t* I, double* S, int64_t id_offset, void* stream) {
  NRK_CHECK_ARG(d > 0 && k > 0 && k <= 1024 && nq >= 0 && nb >= 0, "knn_exact: bad shape nq=%lld nb=%lld d=%d k=%d",
                (long long)nq, (long long)nb, d, k);
  NRK_CHECK_ARG(metric == NRK_METRIC_INNER_PRODUCT || metric == NRK_METRIC_L2, "knn_exact: bad metric %d", metric);
  if (nq == 0) return NRK_OK;
  NRK_CHECK_ARG(xq && D && I && (xb || nb == 0), "knn_exact: null pointer");
  return exact_launch(xq, nq, xb, nb, d, k, metric == NRK_METRIC_L2, nullptr, nullptr, nq, D, I, S, id_offset,
                      (hipStream_t)stream);
}

extern "C" int nrk_knn_flat(const float* xq, int64_t nq, const float* xb, const uint16_t* xb_bf16,
                            const float* xb_meta, const float* stats, int64_t nb, int32_t d, int32_t k,
                            int32_t metric, float* D, int64_t* I, double* S, int64_t id_offset,
                            int32_t* n_fallback, void* ws, size_t ws_bytes, void* const* stage_events,
                            void* stream) {
  NRK_CHECK_ARG(d > 0 && k > 0 && k <= 1024 && nq >= 0 && nb >= 0, "knn_flat: bad shape nq=%lld nb=%lld d=%d k=%d",
                (long long)nq, (long long)nb, d, k);
  NRK_CHECK_ARG(metric == NRK_METRIC_INNER_PRODUCT || metric == NRK_METRIC_L2, "knn_flat: bad metric %d", metric);
  hipStream_t st = (hipStream_t)stream;
  FlatPlan p = make_plan(nq, nb, d, k);
  // L2: rescore at least the top 128 screened candidates.  The certificate
  // needs the k-th exact score to clear theta (>= the best candidate NOT
  // rescored) by the screening-error bound, which for squared L2 on clustered
  // data often exceeds the gap between the 5th and the 33rd neighbour: 10M x 128
  // k = 5 at KP = 32 left 1125 of 4096 queries to the collect pass (12.9 ms),
  // at KP = 128 4 (10.4 ms); 1M x 128: 74 -> 0, 1.33 -> 1.23 ms.  The workspace
  // does not depend on KP.
  if (metric == NRK_METRIC_L2 && !p.exact_only && p.KP < 128) p.KP = p.U < 128 ? p.U : 128;
  if (ws_bytes < p.total) return fail(NRK_EWORKSPACE, "knn_flat: workspace %zu < %zu bytes", ws_bytes, p.total);
  NRK_CHECK_ARG(ws != nullptr, "knn_flat: null workspace");
  char* w = static_cast<char*>(ws);
  int* fbc = reinterpret_cast<int*>(w + p.off_fbc);
  // the screened path zeroes its counters in query_prepare_kernel and publishes
  // them from exact_topk_kernel; the other paths use memsets
  // (the small path zeroes n_fallback in its kernels and uses no counters: no memsets)
  const bool fused_counts = nq > 0 && !p.small && !p.exact_only;
  if (!fused_counts && !p.small) {
    if (hipMemsetAsync(fbc, 0, 16, st) != hipSuccess) return fail(NRK_ELAUNCH, "knn_flat: memset failed");
    if (n_fallback && hipMemsetAsync(n_fallback, 0, 8, st) != hipSuccess)
      return fail(NRK_ELAUNCH, "knn_flat: memset failed");
  }
  if (nq == 0) return NRK_OK;
  NRK_CHECK_ARG(xq && D && I && (xb || nb == 0), "knn_flat: null pointer");
  const int l2 = metric == NRK_METRIC_L2;
  if (p.small) return small_launch(p, xq, nq, xb, nb, d, k, l2, D, I, S, id_offset, ws, st, n_fallback);
  if (p.exact_only) {
    // a shape the screen cannot plan (merge union > 2048, d or k > 256) runs the
    // fp64 brute force for every query: say so through the fallback count
    if (n_fallback && (p.cliff || d > 256 || k > 256) &&
        hipMemsetD32Async(n_fallback, (int)nq, 2, st) != hipSuccess)
      return fail(NRK_ELAUNCH, "knn_flat: memset failed");
    return exact_launch(xq, nq, xb, nb, d, k, l2, nullptr, nullptr, nq, D, I, S, id_offset, st);
  }
  NRK_CHECK_ARG(xb_bf16 && xb_meta && stats, "knn_flat: index not prepared (null bf16/meta/stats)");
  auto mark = [&](int i) {
    if (stage_events) (void)hipEventRecord((hipEvent_t)stage_events[i], st);
  };
  uint16_t* qh = reinterpret_cast<uint16_t*>(w + p.off_qh);
  double* qmeta = reinterpret_cast<double*>(w + p.off_qmeta);
  float* ps = reinterpret_cast<float*>(w + p.off_ps);
  int* pi = reinterpret_cast<int*>(w + p.off_pi);
  float* pt = reinterpret_cast<float*>(w + p.off_pt);
  int* fbl = reinterpret_cast<int*>(w + p.off_fbl);
  FbState fb;  // the merge's uncertified queries (collect pass, in rounds)
  fb.list = fbl;
  fb.count = fbc;
  fb.slots = 0;
  fb.tslots = (int)nq;
  fb.thr_g = reinterpret_cast<double*>(w + p.off_fbt);
  fb.thr_i = reinterpret_cast<int64_t*>(w + p.off_fbi);
  fb.n = nullptr;
  fb.force = test_hook("NRK_FORCE_FALLBACK", 0);
  FbState fbt;  // the tiled fp64 fallback (collect buffer overflow)
  fbt.list = reinterpret_cast<int*>(w + p.off_tfl);
  fbt.count = fbc + 2;
  fbt.slots = p.fb_slots;
  fbt.tslots = p.fb_slots;
  fbt.thr_g = reinterpret_cast<double*>(w + p.off_tft);
  fbt.thr_i = reinterpret_cast<int64_t*>(w + p.off_tfi);
  fbt.n = reinterpret_cast<int*>(w + p.off_fbn);
  fbt.force = 0;
  double* fcg = reinterpret_cast<double*>(w + p.off_fcg);
  int64_t* fci = reinterpret_cast<int64_t*>(w + p.off_fci);
  int* ovl = reinterpret_cast<int*>(w + p.off_ovl);
  float* tau = reinterpret_cast<float*>(w + p.off_tau);
  float* pre = reinterpret_cast<float*>(w + p.off_pre);

  mark(0);
  hipLaunchKernelGGL(query_prepare_kernel, dim3((unsigned)cdiv(p.nq_pad, 4)), dim3(256), 0, st, xq, nq, p.nq_pad, d,
                     p.dp, qh, qmeta, fbc, n_fallback);
  NRK_CHECK_LAUNCH("query_prepare_kernel");
  if (p.tau) {
    screen_fn pf = p.waves == 8 ? pick_screen_dp256_w8(p.M, l2 != 0, 1) : pick_screen(p.dp, p.qt, p.M, l2 != 0, 1);
    if (!pf) return fail(NRK_EUNSUPPORTED, "knn_flat: no pre-pass kernel for dp=%d", p.dp);
    hipLaunchKernelGGL(pf, dim3(p.nqt * p.nch_pre), dim3(p.waves * 64), 0, st, qh, xb_bf16, xb_meta, nq, nb,
                       p.chunk_pre, p.nch_pre, p.nqt, p.tstride, nullptr, nullptr, pre, nullptr, IvfScreen{});
    NRK_CHECK_LAUNCH("screen_kernel (pre-pass)");
    const int nv = 2 * p.nch_pre;
    auto tsel = nv <= 64 ? tau_select_kernel<1> : nv <= 256 ? tau_select_kernel<4> : tau_select_kernel<16>;
    hipLaunchKernelGGL(tsel, dim3((unsigned)cdiv(nq, 4)), dim3(256), 0, st, pre, nv, p.R, nq, tau, nullptr, nullptr);
    NRK_CHECK_LAUNCH("tau_select_kernel");
  }

  bool s16 = false;
  screen_fn fn = main_pass(p, l2 != 0, &s16);
  if (!fn) return fail(NRK_EUNSUPPORTED, "knn_flat: no screen kernel for dp=%d", p.dp);
  const int nblk = p.nqt * p.nch;
  mark(1);
  hipLaunchKernelGGL(fn, dim3(nblk), dim3(p.waves * 64), 0, st, qh, xb_bf16, xb_meta, nq, nb, p.chunk, p.nch, p.nqt, 1,
                     ps, pi, pt, p.tau ? tau : nullptr, IvfScreen{});
  NRK_CHECK_LAUNCH("screen_kernel");

  mark(2);
  {
    const int P = host_pow2ceil(p.U), P2 = host_pow2ceil(p.KP);
    const size_t ub = (size_t)merge_union_bytes(P, p.KP);
    const size_t smem = ub + (size_t)P2 * 16 + (size_t)d * 4;
    if (smem > 150 * 1024) return fail(NRK_EUNSUPPORTED, "knn_flat: merge needs %zu B LDS", smem);
    hipLaunchKernelGGL(merge_rescore_kernel, dim3((unsigned)nq), dim3(256), smem, st, ps, pi, pt, p.nch, p.M, p.KP, k,
                       p.dp, xq, xb, nb, d, l2, qmeta, stats, p.tau ? tau : nullptr, D, I, S, id_offset, fb, nullptr);
    NRK_CHECK_LAUNCH("merge_rescore_kernel");
  }

  mark(3);
  {  // collect pass for the uncertified queries (normally none: every launch exits at once)
    int64_t* clo = reinterpret_cast<int64_t*>(w + p.off_clo);
    int* cseg = reinterpret_cast<int*>(w + p.off_cseg);
    int* cwork = reinterpret_cast<int*>(w + p.off_cwork);
    int* csp = reinterpret_cast<int*>(w + p.off_csp);
    uint16_t* cqi = reinterpret_cast<uint16_t*>(w + p.off_cqi);
    float* cthr = reinterpret_cast<float*>(w + p.off_cthr);
    double* clbg = reinterpret_cast<double*>(w + p.off_clbg);
    int64_t* clbi = reinterpret_cast<int64_t*>(w + p.off_clbi);
    int* ccnt = reinterpret_cast<int*>(w + p.off_ccnt);
    int* cpos = reinterpret_cast<int*>(w + p.off_cpos);
    int* clist = reinterpret_cast<int*>(w + p.off_clist);
    int* ccount = reinterpret_cast<int*>(w + p.off_ccount);
    screen_fn fc = pick_screen(p.dp, 1, p.M, l2 != 0, 3);
    if (!fc) return fail(NRK_EUNSUPPORTED, "knn_flat: no collect kernel for dp=%d", p.dp);
    IvfScreen isc{cwork, clo, cseg, csp, 1, p.cch, (int)cdiv(nb, (int64_t)p.cch), cthr, ccnt, cpos, p.ccap, 1};
    const size_t smem = collect_rescore_smem(p.ccap, d);
    const int rounds = (int)cdiv(nq, (int64_t)FB_SLOTS_MAX);
    for (int r = 0; r < rounds; ++r) {  // each round exits at once when it has no queries
      hipLaunchKernelGGL(flat_collect_plan_kernel, dim3(1), dim3(1024), 0, st, fb, nq, nb, p.cwq, p.cch, qmeta, stats,
                         p.dp, l2, p.ccap, fb.force >= 2 ? 1 : 0, r, FB_SLOTS_MAX, clo, cseg, cwork, csp, cthr, clbg,
                         clbi, ccnt, clist, ccount, qh, cqi);
      NRK_CHECK_LAUNCH("flat_collect_plan_kernel");
      hipLaunchKernelGGL(fc, dim3((unsigned)p.cgrid), dim3(4 * 64), 0, st, cqi, xb_bf16, xb_meta, (int64_t)p.fb_slots,
                         nb, 0, 0, 0, 1, nullptr, nullptr, nullptr, nullptr, isc);
      NRK_CHECK_LAUNCH("screen_kernel (flat collect)");
      hipLaunchKernelGGL(collect_rescore_kernel, dim3((unsigned)p.fb_slots), dim3(256), smem, st, ccnt, cpos, p.ccap,
                         nullptr, xq, xb, d, k, l2, clbg, clbi, D, I, S, id_offset, fbt, nq, nb, nullptr, clist,
                         ccount);
      NRK_CHECK_LAUNCH("collect_rescore_kernel (flat)");
    }
  }
  {
    const int64_t ntiles = cdiv(nb, (int64_t)FB_TR);
    const int grid = (int)(ntiles < 2048 ? ntiles : 2048);
    hipLaunchKernelGGL(fallback_scan_kernel, dim3(grid), dim3(256), (size_t)FB_TR * (d + 1) * 4, st, xq, xb, nb, d,
                       l2, fbt, fcg, fci, p.fb_cap, IvfFb{});
    NRK_CHECK_LAUNCH("fallback_scan_kernel");
    hipLaunchKernelGGL(fallback_select_kernel, dim3(256), dim3(256), (size_t)host_pow2ceil(p.fb_cap) * 16, st, fbt, fcg,
                       fci, p.fb_cap, k, l2, D, I, S, id_offset, ovl, nq);
    NRK_CHECK_LAUNCH("fallback_select_kernel");
  }
  int rc = exact_launch(xq, nq, xb, nb, d, k, l2, ovl, fbt.count + 1, 256, D, I, S, id_offset, st, IvfFb{}, n_fallback,
                        reinterpret_cast<const int*>(w + p.off_ccount + 4), fbt.count);
  if (rc != NRK_OK) return rc;
  mark(4);
  return NRK_OK;
}

extern "C" int nrk_topk_merge(const double* S_parts, const int64_t* I_parts, int32_t nparts, int64_t nq, int32_t k,
                              int32_t metric, float* D, int64_t* I, double* S, void* stream) {
  NRK_CHECK_ARG(nparts >= 1 && nparts <= 16 && k > 0 && nq >= 0, "topk_merge: bad arguments nparts=%d k=%d", nparts,
                k);
  NRK_CHECK_ARG(metric == NRK_METRIC_INNER_PRODUCT || metric == NRK_METRIC_L2, "topk_merge: bad metric %d", metric);
  if (nq == 0) return NRK_OK;
  NRK_CHECK_ARG(S_parts && I_parts && D && I, "topk_merge: null pointer");
  hipLaunchKernelGGL(topk_merge_kernel, dim3((unsigned)cdiv(nq, 256)), dim3(256), 0, (hipStream_t)stream, S_parts,
                     I_parts, nparts, nq, k, metric == NRK_METRIC_L2, D, I, S);
  NRK_CHECK_LAUNCH("topk_merge_kernel");
  return NRK_OK;
}

namespace nrk {
struct IvfPlan {
  int dp, qt, M, waves, wq, nqt;
  int wavesB;               // phase B (collect) waves per workgroup: wq = wavesB x 32 x qt
  int qtA, wqA;             // phase A query tiles per wave / queries per work item
  int nA, chA, cmaxA, R;    // phase A: lane maxima (+positions) over the nA nearest lists, R seeds
  int chB, cmaxB, cap;      // phase B: all probed lists, collect above e_k - B
  int fb_slots, fb_cap;
  int64_t nq_pad, max_rows, ubA, ubB;
  size_t off_fbc, off_cnt, off_fill, off_hist, off_seg, off_work, off_sp, off_qh, off_qmeta, off_qi, off_p0, off_ps, off_pi,
      off_pt, off_pa, off_tau, off_seed, off_lbg, off_lbi, off_thr, off_ccnt, off_cpos, off_fbl, off_fbt, off_fbi, off_fbn, off_fcg, off_fci,
      off_ovl, total;
};

static IvfPlan make_ivf_plan(int64_t nq, int nprobe, int nlist, int64_t max_list, int d, int k) {
  IvfPlan p;
  memset(&p, 0, sizeof(p));
  p.dp = padded_dim(d);
  p.waves = 4;
  p.M = 1;  // neither phase keeps lane lists (mode 4: lane maxima, mode 3: collect)
  // phase B: two query tiles per wave at k <= 8 (one at DP = 256 or k > 8), 4 waves
  // (256 probing queries per work item at configs[3]).  8 waves (512 per item) cut
  // the configs[3] fetch 6.0 -> 4.0 GB per launch but padded the list segments more
  // (3.66 -> 4.11 padded TF) and ran 3.36 -> 3.79 ms (profiles/r03_ivf_collect_ab.log):
  // the screen is MFMA-bound, not HBM-bound
  p.qt = (k <= 8 && p.dp != 256) ? 2 : 1;
  p.wavesB = 4;
  p.wq = p.wavesB * 32 * p.qt;
  // phase A (lane maxima over the nA nearest lists) runs one query tile per
  // wave: half the work-item padding of the grouped queries and a lighter
  // epilogue.  Phase B keeps p.qt (two tiles share each A fragment).
  p.qtA = 1;
  p.wqA = p.waves * 32 * p.qtA;
  p.nqt = (int)cdiv(nq, p.wq);
  p.nq_pad = (int64_t)p.nqt * p.wq;
  const int64_t ml = max_list > 0 ? max_list : 1;
  const int64_t ch_gib = ((int64_t)1 << 30) / (p.dp * 2) / 64 * 64;  // buffer descriptor range
  // phase A: the nA nearest lists per query in chunks of max_list / 128 items (2 lane
  // streams per chunk and query; more streams -> tighter seeds); tau_select
  // takes <= 1024 values per query
  // (one list per query left too few seeds for some queries: fp64 scans, 3.4 -> 248 ms
  // per search; profiles/r06_ivf_phaseA_ab.log)
  p.nA = nprobe < 2 ? nprobe : 2;
  // chunks scale with the lists (max_list / 128, in [64, 4096] rows): a
  // corpus shard's short lists (the 8-GPU configs[3]: ~4K rows) otherwise
  // gave ~20 lane maxima per query, weak seeds, a low collect threshold and
  // ~3 % of the queries overflowing into the fp64 scan
  // (capped at 4096 rows: at configs[3] (max list 213K) 1024-row chunks made ~5-tile
  // items whose prologues dominated phase A; 0.49 -> 0.41 ms, the exact rescore +0.01
  // ms; ml / 32 starved the seeds: profiles/r04_ivf_phaseA_chunks_ab.log)
  int64_t chA = (int64_t)align_up((size_t)(ml / 128 > 64 ? ml / 128 : 64), 64);
  if (chA > 4096) chA = 4096;
  const int64_t cmax_a = 512 / p.nA;
  if (cdiv(ml, chA) > cmax_a) chA = (int64_t)align_up((size_t)cdiv(ml, cmax_a), 64);
  if (chA > ch_gib) chA = ch_gib;
  p.chA = (int)chA;
  p.cmaxA = (int)cdiv(ml, chA);
  p.R = 2 * k > 32 ? 2 * k : 32;  // seeds rescored exactly
  if (p.R > 2 * p.nA * p.cmaxA) p.R = 2 * p.nA * p.cmaxA;
  if (p.R < 1) p.R = 1;
  // phase B: chunk size only sets the work-item granularity
  int64_t chB = 4096;
  if (chB > ch_gib) chB = ch_gib;
  p.chB = (int)chB;
  p.cmaxB = (int)cdiv(ml, chB);
  p.cap = k > 2048 ? k : 2048;
  const int64_t npairs = nq * nprobe;
  p.max_rows = npairs + (int64_t)nlist * (p.wq - 1);
  p.max_rows = (p.max_rows + p.wq - 1) / p.wq * p.wq;
  // persistent grids over the device work tables (upper bound on the items)
  const int64_t gcap = 2048;
  p.ubA = (cdiv(nq * p.nA, (int64_t)p.wqA) + nlist) * p.cmaxA;
  p.ubB = (cdiv(npairs, (int64_t)p.wq) + nlist) * p.cmaxB;
  if (p.ubA > gcap) p.ubA = gcap;
  if (p.ubB > gcap) p.ubB = gcap;
  p.fb_slots = (int)(nq < FB_SLOTS_MAX ? nq : FB_SLOTS_MAX);  // as the flat plan
  p.fb_cap = host_pow2ceil(2 * k + 64);
  if (p.fb_cap < 512) p.fb_cap = 512;
  p.fb_cap = test_hook("NRK_FB_CAP", p.fb_cap);
  if (p.fb_cap < 1) p.fb_cap = 1;
  if (p.fb_cap > 8192) p.fb_cap = 8192;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off = align_up(off + bytes, 256);
    return o;
  };
  // fallback counters [0, 16), guard word [16, 20) (nrk_ivf_search_status reads it
  // at this fixed offset: keep this the first region), collect work tickets [32, 64)
  p.off_fbc = take(64);
  p.off_cnt = take((size_t)nlist * 4);
  p.off_fill = take((size_t)nlist * 4);
  p.off_hist = take((size_t)GROUP_BLOCKS * nlist * 4);
  p.off_seg = take((size_t)(nlist + 1) * 4);
  p.off_work = take((size_t)(nlist + 1) * 4);
  p.off_sp = take((size_t)p.max_rows * 4);
  p.off_qh = take((size_t)p.nq_pad * p.dp * 2);
  p.off_qmeta = take((size_t)nq * 4 * 8);
  p.off_qi = take((size_t)p.max_rows * p.dp * 2);
  p.off_p0 = take((size_t)nq * p.nA * 8);
  p.off_pt = take((size_t)nq * p.nA * p.cmaxA * 2 * 4);
  p.off_pa = take((size_t)nq * p.nA * p.cmaxA * 2 * 4);
  p.off_tau = take((size_t)nq * 4);
  p.off_seed = take((size_t)nq * p.R * 4);
  p.off_lbg = take((size_t)nq * 8);
  p.off_lbi = take((size_t)nq * 8);
  p.off_thr = take((size_t)nq * 4);
  p.off_ccnt = take((size_t)nq * 4);
  p.off_cpos = take((size_t)nq * p.cap * 4);
  p.off_fbl = take((size_t)nq * 4);
  p.off_fbt = take((size_t)p.fb_slots * 8);
  p.off_fbi = take((size_t)p.fb_slots * 8);
  p.off_fbn = take((size_t)p.fb_slots * 4);
  p.off_fcg = take((size_t)p.fb_slots * p.fb_cap * 8);
  p.off_fci = take((size_t)p.fb_slots * p.fb_cap * 8);
  p.off_ovl = take((size_t)nq * 4);
  p.total = off;
  return p;
}

// The search's start-of-call state in ONE launch instead of five blits (each a
// ~4.5 us fill kernel on the stream): the counters and guard word (fbc[0..16)),
// n_fallback, the phase-A probe copy p0 (the nA nearest lists of each query),
// the phase-A lane maxima (all bits set: NaN, never selected), the candidate
// counts and phase A's slot -> pair table (all -1).
__global__ __launch_bounds__(256) void ivf_init_kernel(int* __restrict__ fbc, int32_t* __restrict__ nfb,
                                                       int64_t* __restrict__ p0, const int64_t* __restrict__ probe,
                                                       int64_t nq, int64_t nq_p0, int nprobe, int nA,
                                                       uint32_t* __restrict__ pt, int64_t npt, int* __restrict__ ccnt,
                                                       int* __restrict__ sp, int64_t nsp) {
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x, stride = (int64_t)gridDim.x * 256;
  if (t0 < 16) fbc[t0] = 0;
  if (nfb && t0 < 2) nfb[t0] = 0;
  for (int64_t i = t0; i < nq_p0 * nA; i += stride) p0[i] = probe[(i / nA) * nprobe + i % nA];
  for (int64_t i = t0; i < npt; i += stride) pt[i] = 0xffffffffu;
  for (int64_t i = t0; i < nq; i += stride) ccnt[i] = 0;
  for (int64_t i = t0; i < nsp; i += stride) sp[i] = -1;
}

// group (query, probe) pairs by list and gather the probing queries list-major
// (fill_sp: set the slot -> pair table to -1 first; the first grouping's was set
// by ivf_init_kernel)
static int ivf_group(const int64_t* probe, int64_t nq, int nprobe, int nlist, const int64_t* list_off, int wq, int ch,
                     int dp, int64_t max_rows, const uint16_t* qh, int* cnt, int* fill, int* seg, int* work, int* sp,
                     uint16_t* qi, int* H, int* err, hipStream_t st, bool fill_sp = true) {
  const int64_t npairs = nq * nprobe;
  if (fill_sp && hipMemsetAsync(sp, 0xff, (size_t)max_rows * 4, st) != hipSuccess)
    return fail(NRK_ELAUNCH, "ivf_search: memset failed");
  if (nlist <= GROUP_LDS_LISTS) {
    const size_t lds = (size_t)nlist * 4;
    hipLaunchKernelGGL(ivf_hist_kernel, dim3(GROUP_BLOCKS), dim3(1024), lds, st, probe, npairs, nlist, H);
    NRK_CHECK_LAUNCH("ivf_hist_kernel");
    hipLaunchKernelGGL(ivf_plan_kernel, dim3(1), dim3(1024), 0, st, cnt, list_off, nlist, wq, ch, seg, work, fill, H,
                       GROUP_BLOCKS);
    NRK_CHECK_LAUNCH("ivf_plan_kernel");
    hipLaunchKernelGGL(ivf_place_kernel, dim3(GROUP_BLOCKS), dim3(1024), lds, st, probe, npairs, nlist, seg, H, sp);
    NRK_CHECK_LAUNCH("ivf_place_kernel");
  } else {
    if (hipMemsetAsync(cnt, 0, (size_t)nlist * 4, st) != hipSuccess)
      return fail(NRK_ELAUNCH, "ivf_search: memset failed");
    hipLaunchKernelGGL(ivf_count_kernel, dim3((unsigned)cdiv(npairs, 256)), dim3(256), 0, st, probe, npairs, nlist,
                       cnt);
    NRK_CHECK_LAUNCH("ivf_count_kernel");
    hipLaunchKernelGGL(ivf_plan_kernel, dim3(1), dim3(1024), 0, st, cnt, list_off, nlist, wq, ch, seg, work, fill,
                       nullptr, 0);
    NRK_CHECK_LAUNCH("ivf_plan_kernel");
    hipLaunchKernelGGL(ivf_scatter_kernel, dim3((unsigned)cdiv(npairs, 256)), dim3(256), 0, st, probe, npairs, nlist,
                       seg, fill, sp);
    NRK_CHECK_LAUNCH("ivf_scatter_kernel");
  }
  const int64_t gblk = cdiv(max_rows, 4) < GATHER_BLOCKS ? cdiv(max_rows, 4) : GATHER_BLOCKS;
  hipLaunchKernelGGL(ivf_gather_kernel, dim3((unsigned)gblk), dim3(256), 0, st, qh, dp, nprobe, sp, seg,
                     nlist, max_rows, qi, npairs, err);
  NRK_CHECK_LAUNCH("ivf_gather_kernel");
  return NRK_OK;
}

}  // namespace nrk

extern "C" int nrk_ivf_search_workspace(int64_t nq, int32_t nprobe, int32_t nlist, int64_t max_list, int32_t d,
                                        int32_t k, size_t* ws_bytes) {
  NRK_CHECK_ARG(ws_bytes && nq >= 0 && nprobe > 0 && nlist > 0 && max_list >= 0 && d > 0 && d <= 256 && k > 0 &&
                    k <= 256,
                "ivf_search_workspace: bad arguments");
  *ws_bytes = make_ivf_plan(nq, nprobe, nlist, max_list, d, k).total;
  return NRK_OK;
}

extern "C" int nrk_ivf_search(const float* xq, int64_t nq, const int64_t* probe, int32_t nprobe, const float* xb,
                              const uint16_t* xbh_ivf, const float* meta_ivf, const float* stats,
                              const int64_t* list_off, const int64_t* pos2id, const int32_t* pos2list, int32_t nlist,
                              int64_t n, int64_t max_list, int32_t d, int32_t k, int32_t metric, float* D, int64_t* I,
                              double* S, int64_t id_offset, int32_t* n_fallback, void* ws, size_t ws_bytes,
                              void* const* stage_events, void* stream) {
  NRK_CHECK_ARG(nq >= 0 && nprobe > 0 && nlist > 0 && n >= 0 && max_list >= 0 && d > 0 && d <= 256 && k > 0 &&
                    k <= 256,
                "ivf_search: bad shape nq=%lld nprobe=%d nlist=%d d=%d k=%d", (long long)nq, nprobe, nlist, d, k);
  NRK_CHECK_ARG(metric == NRK_METRIC_INNER_PRODUCT || metric == NRK_METRIC_L2, "ivf_search: bad metric %d", metric);
  NRK_CHECK_ARG(n < ((int64_t)1 << 31), "ivf_search: %lld rows exceed int32 positions", (long long)n);
  hipStream_t st = (hipStream_t)stream;
  const IvfPlan p = make_ivf_plan(nq, nprobe, nlist, max_list, d, k);
  if (ws_bytes < p.total) return fail(NRK_EWORKSPACE, "ivf_search: workspace %zu < %zu bytes", ws_bytes, p.total);
  NRK_CHECK_ARG(ws != nullptr, "ivf_search: null workspace");
  char* w = static_cast<char*>(ws);
  int* fbc = reinterpret_cast<int*>(w + p.off_fbc);
  NRK_CHECK_ARG(nq == 0 || (xq && probe && D && I && list_off), "ivf_search: null pointer");
  NRK_CHECK_ARG(n == 0 || (xb && xbh_ivf && meta_ivf && stats && pos2id && pos2list), "ivf_search: null index data");
  const int l2 = metric == NRK_METRIC_L2;
  auto mark = [&](int i) {
    if (stage_events) (void)hipEventRecord((hipEvent_t)stage_events[i], st);
  };
  int* cnt = reinterpret_cast<int*>(w + p.off_cnt);
  int* fill = reinterpret_cast<int*>(w + p.off_fill);
  int* hist = reinterpret_cast<int*>(w + p.off_hist);
  int* seg = reinterpret_cast<int*>(w + p.off_seg);
  int* work = reinterpret_cast<int*>(w + p.off_work);
  int* sp = reinterpret_cast<int*>(w + p.off_sp);
  uint16_t* qh = reinterpret_cast<uint16_t*>(w + p.off_qh);
  double* qmeta = reinterpret_cast<double*>(w + p.off_qmeta);
  uint16_t* qi = reinterpret_cast<uint16_t*>(w + p.off_qi);
  int64_t* p0 = reinterpret_cast<int64_t*>(w + p.off_p0);
  float* pt = reinterpret_cast<float*>(w + p.off_pt);
  int* pa = reinterpret_cast<int*>(w + p.off_pa);
  float* tau = reinterpret_cast<float*>(w + p.off_tau);
  int* seed = reinterpret_cast<int*>(w + p.off_seed);
  double* lbg = reinterpret_cast<double*>(w + p.off_lbg);
  int64_t* lbi = reinterpret_cast<int64_t*>(w + p.off_lbi);
  float* thr = reinterpret_cast<float*>(w + p.off_thr);
  int* ccnt = reinterpret_cast<int*>(w + p.off_ccnt);
  int* cpos = reinterpret_cast<int*>(w + p.off_cpos);
  FbState fb;
  fb.list = reinterpret_cast<int*>(w + p.off_fbl);
  fb.count = fbc;
  fb.slots = p.fb_slots;
  fb.tslots = p.fb_slots;
  fb.thr_g = reinterpret_cast<double*>(w + p.off_fbt);
  fb.thr_i = reinterpret_cast<int64_t*>(w + p.off_fbi);
  fb.n = reinterpret_cast<int*>(w + p.off_fbn);
  fb.force = 0;
  double* fcg = reinterpret_cast<double*>(w + p.off_fcg);
  int64_t* fci = reinterpret_cast<int64_t*>(w + p.off_fci);
  int* ovl = reinterpret_cast<int*>(w + p.off_ovl);
  int* gerr = fbc + 4;  // the guard word (zeroed with the counters; nrk_ivf_search_status)
  IvfFb ivf{pos2id, pos2list, list_off, probe, nprobe, nlist, nq, gerr};
  const bool force_fb = test_hook("NRK_FORCE_FALLBACK", 0) != 0;
  mark(0);
  {  // counters, guard word, n_fallback, candidate counts; with rows: phase A's p0 / pt / sp
    const bool rows = n > 0 && nq > 0;
    const int64_t npt = rows ? nq * p.nA * p.cmaxA * 2 : 0, nsp = rows ? p.max_rows : 0;
    int64_t big = npt > nsp ? npt : nsp;
    if (nq * p.nA > big) big = nq * p.nA;
    const unsigned gi = (unsigned)(big > 16 ? (cdiv(big, 256) < 2048 ? cdiv(big, 256) : 2048) : 1);
    hipLaunchKernelGGL(ivf_init_kernel, dim3(gi), dim3(256), 0, st, fbc, n_fallback, p0, probe, nq, rows ? nq : 0,
                       nprobe, p.nA, reinterpret_cast<uint32_t*>(pt), npt, ccnt, sp, nsp);
    NRK_CHECK_LAUNCH("ivf_init_kernel");
  }
  if (nq == 0) return NRK_OK;

  hipLaunchKernelGGL(query_prepare_kernel, dim3((unsigned)cdiv(p.nq_pad, 4)), dim3(256), 0, st, xq, nq, p.nq_pad, d,
                     p.dp, qh, qmeta);
  NRK_CHECK_LAUNCH("query_prepare_kernel");
  if (n > 0) {
    // ---- phase A: lane maxima over the nearest list of every query -> tau
    // (p0, pt (NaN: never selected), ccnt and sp were set by ivf_init_kernel)
    int rc =
        ivf_group(p0, nq, p.nA, nlist, list_off, p.wqA, p.chA, p.dp, p.max_rows, qh, cnt, fill, seg, work, sp, qi, hist, gerr,
                  st, false);
    if (rc != NRK_OK) return rc;
    screen_fn fa = pick_screen(p.dp, p.qtA, p.M, l2 != 0, 4);
    if (!fa) return fail(NRK_EUNSUPPORTED, "ivf_search: no screen kernel for dp=%d", p.dp);
    IvfScreen isa{work, list_off, seg, sp, nlist, p.chA, p.cmaxA, nullptr, nullptr, nullptr, 0, p.nA, nullptr, gerr};
    hipLaunchKernelGGL(fa, dim3((unsigned)p.ubA), dim3(p.waves * 64), 0, st, qi, xbh_ivf, meta_ivf, nq, n, 0, 0, 0,
                       3, nullptr, pa, pt, nullptr, isa);  // every third tile: seeds from a third of the rows
    // (tile strides 2 / 3 / 4 / 6: search 3.49 / 3.46 / 3.48 / 3.50 ms, phase A falling and the
    // exact rescore of the wider collect rising; profiles/r04_ivf_phaseA_stride_ab.log)
    NRK_CHECK_LAUNCH("screen_kernel (ivf phase A)");
    const int nva = 2 * p.nA * p.cmaxA;
    auto tsel = nva <= 64 ? tau_select_kernel<1> : nva <= 256 ? tau_select_kernel<4>
              : nva <= 512 ? tau_select_kernel<8> : tau_select_kernel<16>;
    hipLaunchKernelGGL(tsel, dim3((unsigned)cdiv(nq, 4)), dim3(256), 0, st, pt, nva, p.R, nq, tau, pa, seed);
    NRK_CHECK_LAUNCH("tau_select_kernel (ivf)");
    hipLaunchKernelGGL(ivf_seed_kernel, dim3((unsigned)nq), dim3(64), (size_t)host_pow2ceil(p.R) * 16 + (size_t)d * 4,
                       st, seed, p.R, k, pos2id, xq, xb, d, l2, qmeta, stats, p.dp, thr, lbg, lbi, ccnt, p.cap, n, gerr);
    NRK_CHECK_LAUNCH("ivf_seed_kernel");
    NRK_CHECK_LAUNCH("ivf_thr_kernel");
    // ---- phase B grouping: every probed list
    rc = ivf_group(probe, nq, nprobe, nlist, list_off, p.wq, p.chB, p.dp, p.max_rows, qh, cnt, fill, seg, work, sp, qi,
                   hist, gerr, st);
    if (rc != NRK_OK) return rc;
  }  // (empty index: ccnt zeroed by ivf_init_kernel, so every query reads all -1)

  mark(1);
  if (n > 0) {
    // ---- phase B: collect every probed item at or above e_k - B_q
    screen_fn fbk = pick_screen(p.dp, p.qt, p.M, l2 != 0, 3);
    // the 16x16x32 collect where built (NRK_SCREEN16=0: the 32x32x16 one; a test hook)
    if (p.dp == 128 && p.qt == 2 && p.wavesB == 4 && test_hook("NRK_SCREEN16", 1)) fbk = pick_collect16_dp128(l2 != 0);
    if (!fbk) return fail(NRK_EUNSUPPORTED, "ivf_search: no collect kernel for dp=%d", p.dp);
    IvfScreen isb{work, list_off, seg, sp, nlist, p.chB, p.cmaxB, thr, ccnt, cpos, p.cap, nprobe, fbc + 8, gerr};
    hipLaunchKernelGGL(fbk, dim3((unsigned)p.ubB), dim3(p.wavesB * 64), 0, st, qi, xbh_ivf, meta_ivf, nq, n, 0, 0, 0, 1,
                       nullptr, nullptr, nullptr, nullptr, isb);
    NRK_CHECK_LAUNCH("screen_kernel (ivf collect)");
  }

  mark(2);
  {
    if (force_fb && n > 0 && hipMemsetAsync(ccnt, 0x7f, (size_t)nq * 4, st) != hipSuccess)  // testing: overflow all
      return fail(NRK_ELAUNCH, "ivf_search: memset failed");
    const size_t smem = collect_rescore_smem(p.cap, d);
    hipLaunchKernelGGL(collect_rescore_kernel, dim3((unsigned)nq), dim3(256), smem, st, ccnt, cpos, p.cap, pos2id, xq,
                       xb, d, k, l2, lbg, lbi, D, I, S, id_offset, fb, nq, n, gerr);
    NRK_CHECK_LAUNCH("collect_rescore_kernel");
  }

  mark(3);
  if (n > 0) {
    const int64_t ntiles = cdiv(n, (int64_t)FB_TR);
    const int grid = (int)(ntiles < 2048 ? ntiles : 2048);
    hipLaunchKernelGGL(fallback_scan_kernel, dim3(grid), dim3(256), (size_t)FB_TR * (d + 1) * 4, st, xq, xb, n, d, l2,
                       fb, fcg, fci, p.fb_cap, ivf);
    NRK_CHECK_LAUNCH("fallback_scan_kernel (ivf)");
  }
  hipLaunchKernelGGL(fallback_select_kernel, dim3(256), dim3(256), (size_t)host_pow2ceil(p.fb_cap) * 16, st, fb, fcg,
                     fci, p.fb_cap, k, l2, D, I, S, id_offset, ovl, nq, gerr);
  NRK_CHECK_LAUNCH("fallback_select_kernel (ivf)");
  int rc = exact_launch(xq, nq, xb, n, d, k, l2, ovl, fbc + 1, 256, D, I, S, id_offset, st, ivf);
  if (rc != NRK_OK) return rc;
  mark(4);
  // [0] the tiled fp64 scan's queries (collect overflow / too few seeds), [1] of
  // those, the ones its buffer could not hold either (the block-per-query scan)
  if (n_fallback && hipMemcpyAsync(n_fallback, fbc, 8, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return fail(NRK_ELAUNCH, "ivf_search: copy of fallback counts failed");
  return NRK_OK;
}

// The guard word of the last nrk_ivf_search on this workspace (GuardCode bits,
// 0 = every workspace-derived index was in range) -> device int32 (async).
extern "C" int nrk_ivf_search_status(const void* ws, size_t ws_bytes, int32_t* guard, void* stream) {
  NRK_CHECK_ARG(ws != nullptr && guard != nullptr && ws_bytes >= 64, "ivf_search_status: bad arguments");
  // make_ivf_plan: off_fbc == 0, guard word = fbc[4]
  if (hipMemcpyAsync(guard, static_cast<const char*>(ws) + 16, 4, hipMemcpyDeviceToDevice, (hipStream_t)stream) !=
      hipSuccess)
    return fail(NRK_ELAUNCH, "ivf_search_status: copy failed");
  return NRK_OK;
}
