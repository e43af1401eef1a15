// din_rerank.hip — DIN evaluate() for re-ranking, fused: every candidate of a
// user attends over the same history (DIN.py:166-173, `his.expand(C, -1, -1)`)
// and goes through the eval-mode head (DIN.py:113-133), one launch for all
// users, nothing but the logits written to HBM.
//
// Per candidate c of user u (q = its table row, K = u's history rows):
//   U[c]  = W1q q + b1                    (attention query half, DIN.py:104-106)
//   P[r]  = W1k K[r]                      (once per USER)
//   s[c][r] = b2 + sum_n w2[n] relu(U[c][n] + P[r][n])
//   alpha[c] = softmax_r s[c][.] over all L slots (padding included, DIN.py:108)
//   pooled[c] = sum_r alpha[c][r] K[r]
//   logit[c] = h3 . relu(H2 relu(H1q q + H1p pooled + c1) + c2) + c3
// with the three BatchNorms folded into the Linears after them (eval mode,
// pipeline._fold_eval_head).  Reassociated so that per candidate only the
// scoring stays:
//   * H1p pooled[c] = (sum_r e[c][r] R[r]) / sum_r e[c][r] with R = K H1p^T
//     (once per user): pooled itself is never formed;
//   * w2[n] relu(x) = (y + sgn_n |y|) / 2 with y = w2[n] x, sgn_n = sign(w2[n]),
//     so s = (SU[c] + SP[r] + sum_n sgn_n |U'[c][n] + P'[r][n]|) / 2 with
//     U' = w2 . U, P' = w2 . P, SU = sum U', SP = sum P': per (candidate, row,
//     unit) one add and one fma with |.| as a source modifier (2 VALU);
//   * padding slots (ids < 0 or >= n_table) hold zero keys: they all share one
//     row (P = R = 0) that enters the softmax denominator L - nv times, so a
//     user has nr = nv + [nv < L] rows.
// Precision: the table is bf16 (exact in the MFMA); every f32 weight enters the
// bf16 MFMAs as hi + lo bf16 (16 mantissa bits), the softmax weights e and the
// per-user R and the head's h1 as hi + lo too (three products: hi.hi, lo.hi,
// hi.lo); f32 accumulation throughout.  Measured against the reference's own
// evaluate() in tests/test_din_bf16_oracle.py / test_rerank_cluster.py.
//
// One 512-thread workgroup per CU (LDS), persistent over a work queue of users
// (one atomic per user, fetched a user ahead).  Per user: its compacted
// history rows -> LDS, [P | R] on MFMA (16x16x32) with W1k / H1p fragments
// read from L2.  Then per chunk of 64 candidates (five barriers):
//   1. the chunk's candidate rows (loaded into registers during the previous
//      chunk) -> LDS image;  U' = w2 (W1q q + b1) on MFMA, W1q^T fragments of
//      the wave's 16-unit tile resident in registers; Q1 = H1q q tiles kept in
//      the registers of the wave that later finishes them;
//   2. scoring on the VALU: lane = (2 candidates, A/8 units), 8 lanes per
//      candidate pair (sums by DPP), waves 0-3 take the even history rows and
//      waves 4-7 the odd ones (each SIMD hosts waves w and w + 4);
//      e = exp(s - m_g) per row group g, written back in place;
//   3. h1 = relu(Q1 + (e R) / sum e + c1) on MFMA (e, R hi + lo);
//   4. h2 on MFMA, logit = h3 . relu(h2 + c2) + c3 by 16-lane DPP sums;
//   5. logits -> HBM (-inf for padded candidates).
#include <math.h>

#include "din_rerank.h"

namespace nrk {
namespace rr {

constexpr int NT = 512;  // 8 waves
constexpr int CH = 64;   // candidates per chunk
constexpr int SST = 68;  // S row stride (floats): per-candidate scores / softmax weights


// LDS image of 64 rows of D bf16: 16-B chunks XOR-swizzled by row, so the
// 16x16x32 A-fragment reads (16 rows x one chunk per lane group) are
// conflict-free.
template <int D>
__device__ __forceinline__ int img_off(int row, int chunk) {  // byte offset of 16-B chunk `chunk` of `row`
  constexpr int CPR = D / 8;
  constexpr int SW = CPR >= 16 ? 15 : CPR - 1;
  return row * 2 * D + 16 * (chunk ^ (row & SW));
}

template <int D, int A>
struct Geo {
  static constexpr int SL = A / 8;                 // units per scoring lane
  static constexpr int PRS = A;                    // P' / U' row stride (floats): 8 slices of SL units
  // physical float4 of the i4-th float4 of slice sj: at SL = 16 the slices sj and
  // sj + 4 (256 B apart, same banks) store their float4s rotated by two, so the
  // eight slices' b128 reads of a row stay conflict-free without padding
  __device__ static int pos4(int sj, int i4) { return SL == 16 ? (i4 + 2 * (sj >> 2)) & 3 : i4; }
  // float offset of attention unit n within a P' / U' row
  __device__ static int col(int n) {
    const int sj = n / SL, w = n % SL;
    return sj * SL + 4 * pos4(sj, w >> 2) + (w & 3);
  }
  static constexpr int NE = LP * (D / 8) / NT;     // staged 16-B chunks per thread
  static constexpr int KSD = D / 32;               // k-steps over d
  static constexpr int NUT = A / 16;               // 16-unit tiles of U / P
};

template <int D, int A, int F, bool PROJ>
struct Lds {  // byte offsets
  int p, hsp, rt, q, us, ms, lgp, cst, h2, sx, h1q, total;
  bool h2l;   // H2 hi / lo resident in LDS (when it fits)
  bool ssep;  // S in a region of its own (when it fits), not over the image
  bool h1l;   // H1q hi / lo resident in LDS (when it fits; else read from L2 per chunk)
  __host__ __device__ constexpr Lds()
      : p(0), hsp(0), rt(0), q(0), us(0), ms(0), lgp(0), cst(0), h2(0), sx(0), h1q(0), total(0), h2l(false),
        ssep(false), h1l(false) {
    using G = Geo<D, A>;
    p = 0;                                     // P' [LP][A] f32
    hsp = p + LP * G::PRS * 4;                 // SP / 2 [LP] f32
    rt = hsp + LP * 4;                         // R^T hi, lo [F][LP] bf16
    q = rt + 2 * F * LP * 2;                   // candidate / history image [64][D] bf16;  S [CH][SST] f32 later
                                               // (PROJ: the chunk's Q1 [CH][F] f32; there is no row image)
    const int qb = PROJ ? CH * F * 4 : (CH * D * 2 > CH * SST * 4 ? CH * D * 2 : CH * SST * 4);
    us = q + qb;                               // U' [CH][A] f32;  h1 [CH][F + 4] f32 later
    const int ub = CH * G::PRS * 4 > CH * (F + 4) * 4 ? CH * G::PRS * 4 : CH * (F + 4) * 4;
    ms = us + ub;                              // {m, sum} of the two row groups [2][2][CH] f32
    lgp = ms + 4 * CH * 4;                     // partial logits [F/32][CH] f32 (F/2 units in 16-unit tiles)
    cst = lgp + (F / 32 > 0 ? F / 32 : 1) * CH * 4;  // c1 [F], c2 [F/2], h3 [F/2] f32; candidate valid [2][CH] i32
    h2 = cst + 2 * F * 4 + 2 * CH * 4 + A * 4;  // (+ w2 [A] f32);  H2 hi, lo [F/2][F] bf16 (if it fits)
    const int h2b = 2 * (F / 2) * F * 2;
    h2l = h2 + h2b + 16 <= 160 * 1024;
    if (PROJ && h2 + h2b + CH * SST * 4 + 16 > 160 * 1024) h2l = false;  // PROJ needs S apart: H2 from L2
    int end = h2l ? h2 + h2b : h2;
    ssep = end + CH * SST * 4 + 16 <= 160 * 1024;
    sx = ssep ? end : q;                       // S [CH][SST] f32
    if (ssep) end += CH * SST * 4;
    h1q = end;                                 // H1q hi, lo [F][D] bf16 (image swizzle), if it fits
    h1l = !PROJ && end + 2 * F * D * 2 + 16 <= 160 * 1024;
    total = (h1l ? end + 2 * F * D * 2 : end) + 16;
  }
};

// A pointer offset by an opaque zero: loads from it stay where they are written
// instead of being hoisted out of the user / chunk loops (loop-invariant fragment
// loads would otherwise pin their registers kernel-wide).  The base keeps its
// global address space (hiding the pointer itself would turn them into flat loads).
template <class T>
__device__ __forceinline__ const T* pinned(const T* p) {
  int z = 0;
  asm volatile("" : "+s"(z));
  return p + z;
}


template <int D, int A, int F, bool PROJ>
__global__ __launch_bounds__(NT, 1) void din_rerank_kernel(RerankArgs a) {
  using G = Geo<D, A>;
  constexpr int SL = G::SL, PRS = G::PRS, NE = G::NE, KSD = G::KSD, NUT = G::NUT;
  constexpr int CPR = D / 8, F2 = F / 2, NFT = F / 16, NQT = F / 32;  // Q1 tiles per wave
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr Lds<D, A, F, PROJ> lo_{};
  static_assert(!PROJ || lo_.ssep, "din_rerank: the projected form keeps S apart from the image");
  float* Pp = reinterpret_cast<float*>(smem + lo_.p);
  float* hSP = reinterpret_cast<float*>(smem + lo_.hsp);
  uint16_t* Rth = reinterpret_cast<uint16_t*>(smem + lo_.rt);
  uint16_t* Rtl = Rth + F * LP;
  unsigned char* img = smem + lo_.q;
  float* S = reinterpret_cast<float*>(smem + lo_.sx);
  float* Us = reinterpret_cast<float*>(smem + lo_.us);
  float* H1s = reinterpret_cast<float*>(smem + lo_.us);
  float* MS = reinterpret_cast<float*>(smem + lo_.ms);  // [g][{m, sum}][CH]
  float* LGP = reinterpret_cast<float*>(smem + lo_.lgp);
  float* c1s = reinterpret_cast<float*>(smem + lo_.cst);
  float* c2s = c1s + F;
  float* h3s = c2s + F2;
  int* cval = reinterpret_cast<int*>(h3s + F2);
  float* w2s = reinterpret_cast<float*>(cval + 2 * CH);
  uint16_t* H2h = reinterpret_cast<uint16_t*>(smem + lo_.h2);
  uint16_t* H2l = H2h + F2 * F;
  unsigned char* H1qh = smem + lo_.h1q;  // H1q hi rows, then lo rows (img_off layout, row stride 2 D bytes)
  unsigned char* H1ql = H1qh + F * D * 2;
  int* qslot = reinterpret_cast<int*>(smem + lo_.total - 16);

  // Lane-dependent indices are re-derived at the top of every user and chunk
  // from a thread id the compiler cannot see through (refresh): otherwise it
  // hoists dozens of per-thread LDS / global addresses to the kernel entry and
  // spills them, and every reload then waits behind the in-flight row gathers
  // (vmcnt counts in order).  Wave-uniform indices live in SGPRs.
  int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int lane, l15, l4, sj, pl;
  auto refresh = [&]() __attribute__((always_inline)) {
    asm volatile("" : "+v"(tid));
    lane = tid & 63;
    l15 = lane & 15;
    l4 = lane >> 4;
    // scoring lane: pair slot pl (two candidates), unit slice sj = lane & 7
    // (units sj SL .. sj SL + SL - 1)
    sj = lane & 7;
    pl = lane >> 3;
  };
  refresh();

  // ---- the head's constants -> LDS (published by the first barrier) ---------
  for (int i = tid; i < F; i += NT) c1s[i] = a.c1[i];
  for (int i = tid; i < A; i += NT) w2s[i] = a.w2[i];
  for (int i = tid; i < F2; i += NT) {
    c2s[i] = a.c2[i];
    h3s[i] = a.h3[i];
  }
  if constexpr (lo_.h1l) {
    for (int i = tid; i < F * CPR; i += NT) {
      const int f = i / CPR, c = i % CPR;
      *reinterpret_cast<bf16x8*>(H1qh + img_off<D>(f, c)) = *reinterpret_cast<const bf16x8*>(a.H1q_hi + (int64_t)f * D + 8 * c);
      *reinterpret_cast<bf16x8*>(H1ql + img_off<D>(f, c)) = *reinterpret_cast<const bf16x8*>(a.H1q_lo + (int64_t)f * D + 8 * c);
    }
  }
  if constexpr (lo_.h2l) {
    for (int i = tid; i < F2 * F / 8; i += NT) {
      reinterpret_cast<uint4*>(H2h)[i] = reinterpret_cast<const uint4*>(a.H2_hi)[i];
      reinterpret_cast<uint4*>(H2l)[i] = reinterpret_cast<const uint4*>(a.H2_lo)[i];
    }
  }

  // ---- resident: this wave's 16-unit tile of W1q^T (B operand, hi + lo) --
  // projection tiles: unit tile ut, candidate tiles [ct0, ct0 + nct)
  constexpr int GP = 8 / NUT > 0 ? 8 / NUT : 1;  // waves per unit tile
  const int ut = w % NUT, pg = w / NUT;
  const bool proj_on = pg < GP;
  const int nct = 4 / GP, ct0 = pg * nct;
  bf16x8 wqh[KSD], wql[KSD];
  float b1u = 0.f, w2u = 0.f;
  if constexpr (!PROJ) {
    const int u = 16 * ut + l15;
#pragma unroll
    for (int s = 0; s < KSD; ++s) {
      wqh[s] = *reinterpret_cast<const bf16x8*>(a.W1q_hi + (int64_t)u * D + 32 * s + 8 * l4);
      wql[s] = *reinterpret_cast<const bf16x8*>(a.W1q_lo + (int64_t)u * D + 32 * s + 8 * l4);
    }
    b1u = a.b1[u];
    w2u = a.w2[u];
  }
  float sgn[SL];
#pragma unroll
  for (int i = 0; i < SL; ++i) sgn[i] = a.w2[sj * SL + i] >= 0.f ? 1.f : -1.f;

  // ---- staging: the next work item's 64 rows (history or candidates) go
  // through registers.  Ids are read well before the rows they name (a
  // dependent load pair would otherwise expose two memory latencies per
  // chunk): sidn = the row ids this thread stages next.
  // (non-temporal gathers: the rows are used once, and keeping them out of L2
  // keeps the H1q / W1k / H1p fragments every chunk and user re-reads there)
  bf16x8 stg[NE];
  const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
  int sidn[NE];
  unsigned svalid = 0;  // bit k: stg[k] holds a valid candidate row
  // the stored id of candidate ci of user u_ (the appended extra at ci == len;
  // -1 past the list): a load whose value is only tested where it is used
  // (valid_id), so issuing it never waits for it
  auto cand_raw = [&](int u_, int64_t off, int len, int ci) -> int {
    int id = -1;
    if (ci < len) id = a.cand[off + ci];
    else if (ci == len && a.extra) id = a.extra[u_];
    return id;
  };
  auto valid_id = [&](int id) -> bool { return id >= 0 && id < a.n_table; };
  [[maybe_unused]] auto cand_id = [&](int u_, int64_t off, int len, int ci) -> int {
    const int id = cand_raw(u_, off, len, ci);
    return valid_id(id) ? id : -1;
  };
  auto load_cids = [&](int u_, int64_t off, int len, int c0_) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < NE; ++k) sidn[k] = cand_raw(u_, off, len, c0_ + (tid + NT * k) / CPR);
  };
  auto issue_rows = [&]() __attribute__((always_inline)) {
    svalid = 0;
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      const int cc = (tid + NT * k) % CPR;
      stg[k] = z8;
      if (valid_id(sidn[k])) {
        stg[k] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(a.table + (int64_t)sidn[k] * D + cc * 8));
        svalid |= 1u << k;
      }
    }
  };
  auto store_rows = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      const int e = tid + NT * k, row = e / CPR, cc = e % CPR;
      *reinterpret_cast<bf16x8*>(img + img_off<D>(row, cc)) = stg[k];
    }
  };
  auto store_valid = [&](int* cv) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      const int e = tid + NT * k;
      if (e % CPR == 0) cv[e / CPR] = (svalid >> k) & 1;
    }
  };
  // history of a user (hid: lane's slot id): valid mask of the first L slots
  // (wave-uniform), rows compacted to the front
  auto load_hid = [&](int u_) -> int { return lane < a.L ? a.hist[(int64_t)u_ * a.L + lane] : -1; };
  auto issue_hist = [&](int hid, uint64_t& vm_) __attribute__((always_inline)) {
    vm_ = __ballot(lane < a.L && hid >= 0 && hid < a.n_table);
    const int nv_ = __popcll(vm_);
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      const int e = tid + NT * k, row = e / CPR, cc = e % CPR;
      const int src = __shfl(hid, row < nv_ ? nth_set_bit(vm_, row) : 0, 64);
      stg[k] = z8;
      if (row < nv_) stg[k] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(a.table + (int64_t)src * D + cc * 8));
    }
  };
  // PROJ: a chunk's projected candidates, CPX float4s each ([U' | Q1]: to the
  // U' rows and the Q1 rows of LDS), and the validity of candidate tid (< CH)
  constexpr int CPX = (A + F) / 4, NEP = (CH * CPX + NT - 1) / NT;
  float4 stp[PROJ ? NEP : 1];
  int vid = -1;
  float* Q1s = reinterpret_cast<float*>(smem + lo_.q);  // [CH][F] (PROJ)
  auto load_proj = [&](int u_, int64_t off, int len, int c0_) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < NEP; ++k) {
      const int e = tid + NT * k, cand = e / CPX, part = e % CPX, ci = c0_ + cand;
      const float* src = nullptr;
      if (e < CH * CPX) {
        if (ci < len) src = a.cproj + (off + ci) * (A + F);
        else if (ci == len && a.xproj) src = a.xproj + (int64_t)u_ * (A + F);
      }
      stp[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (src) stp[k] = *reinterpret_cast<const float4*>(src + 4 * part);
    }
    vid = tid < CH ? cand_raw(u_, off, len, c0_ + tid) : -1;
  };
  auto store_proj = [&](int* cv) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < NEP; ++k) {
      const int e = tid + NT * k, cand = e / CPX, part = e % CPX;
      if (e < CH * CPX) {
        if (part < A / 4) *reinterpret_cast<float4*>(Us + cand * PRS + 4 * part) = stp[k];
        else *reinterpret_cast<float4*>(Q1s + cand * F + 4 * (part - A / 4)) = stp[k];
      }
    }
    if (tid < CH) cv[tid] = valid_id(vid);
  };
  // PROJ: a user's history arrives projected ([P' | R] per slot, from hproj):
  // the compacted valid slots' projections go through the same registers as a
  // chunk's (the next user is staged only after the last chunk's were stored),
  // rows from nv on are zero (the shared padding row and the MFMA's K padding)
  static_assert(CH == LP, "din_rerank: a chunk and a history hold the same row count");
  auto issue_hist_proj = [&](int u_, int hid, uint64_t& vm_) __attribute__((always_inline)) {
    vm_ = __ballot(lane < a.L && hid >= 0 && hid < a.n_table);
    const int nv_ = __popcll(vm_);
#pragma unroll
    for (int k = 0; k < NEP; ++k) {
      const int e = tid + NT * k, row = e / CPX, part = e % CPX;
      stp[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < LP * CPX && row < nv_)
        stp[k] = *reinterpret_cast<const float4*>(a.hproj + ((int64_t)u_ * a.L + nth_set_bit(vm_, row)) * (A + F) +
                                                  4 * part);
    }
  };
  auto store_hist_proj = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < NEP; ++k) {
      const int e = tid + NT * k, row = e / CPX, part = e % CPX;
      if (e < LP * CPX) {
        if (part < A / 4) {
          *reinterpret_cast<float4*>(Pp + row * PRS + 4 * part) = stp[k];  // (already in the slice order)
        } else {
          const int f0 = 4 * (part - A / 4);
          const float v[4] = {stp[k].x, stp[k].y, stp[k].z, stp[k].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            short h, l;
            split_bf16(v[j], h, l);
            Rth[(f0 + j) * LP + row] = (uint16_t)h;
            Rtl[(f0 + j) * LP + row] = (uint16_t)l;
          }
        }
      }
    }
  };

  if (tid == 0) qslot[0] = atomicAdd(a.queue, 1);
  __syncthreads();
  int u = qslot[0];
  uint64_t vm = 0;
  if (u < a.nU) {
    if constexpr (PROJ) issue_hist_proj(u, load_hid(u), vm);
    else issue_hist(load_hid(u), vm);
  }

  while (u < a.nU) {
    refresh();
    const int nv = __popcll(vm), npad = a.L - nv, nr = nv + (npad > 0 ? 1 : 0);
    const int nrp = (nr + 31) & ~31;  // rows of the softmax-weight MFMA (K multiple of 32)
    const int64_t coff = a.cand_off[u];
    const int clen = a.cand_len[u];
    const int ctot = clen + (a.extra ? 1 : 0);
    const int nchunk = (ctot + CH - 1) / CH;
    const int64_t ooff = a.out_off[u];
    __syncthreads();  // the previous user's last chunk is done with the image region (PROJ: with P', R)
    if constexpr (PROJ) store_hist_proj();  // [P' | R] -> LDS
    else store_rows();                      // history rows -> image
    if (tid == 0) qslot[1] = atomicAdd(a.queue, 1);  // the next user (read after chunk 0's first barrier)
    __syncthreads();
    if (nchunk > 0) {
      if constexpr (PROJ) load_proj(u, coff, clen, 0);  // chunk 0's projections (in flight during [P | R])
      else load_cids(u, coff, clen, 0);  // chunk 0's ids (its rows are issued after [P | R])
    }

    // ---- [P | R] = K [W1k ; H1p]^T for the 16-row tiles below nrp ----------
    // Tile t = (unit tile t / nrt, row tile t % nrt); wave w takes the
    // contiguous range [w ntile / 8, (w + 1) ntile / 8), so it reads the B
    // fragments (hi + lo, from L2) of at most two or three unit tiles.
    // (PROJ: staged above, with this MFMA sequence, by nrk_din_rerank_project_hist)
    if constexpr (!PROJ) {
      const int nrt = nrp / 16, ntile = (NUT + NFT) * nrt;
      const int t0 = (w * ntile) >> 3, t1 = ((w + 1) * ntile) >> 3;
      auto load_frags = [&](int uti, bf16x8(&fh)[KSD], bf16x8(&fl)[KSD]) __attribute__((always_inline)) {
        const bool isP = uti < NUT;
        const int urow = isP ? 16 * uti + l15 : 16 * (uti - NUT) + l15;
        const uint16_t* bh = (isP ? pinned(a.W1k_hi) : pinned(a.H1p_hi)) + (int64_t)urow * D + 8 * l4;
        const uint16_t* bl = (isP ? pinned(a.W1k_lo) : pinned(a.H1p_lo)) + (int64_t)urow * D + 8 * l4;
#pragma unroll
        for (int s = 0; s < KSD; ++s) {
          fh[s] = *reinterpret_cast<const bf16x8*>(bh + 32 * s);
          fl[s] = *reinterpret_cast<const bf16x8*>(bl + 32 * s);
        }
      };
      for (int uti = t0 / nrt; uti * nrt < t1; ++uti) {
        const bool isP = uti < NUT;
        const int urow = isP ? 16 * uti + l15 : 16 * (uti - NUT) + l15;
        bf16x8 fh[KSD], fl[KSD];
        load_frags(uti, fh, fl);
        const int rb = t0 > uti * nrt ? t0 - uti * nrt : 0;
        const int re = t1 < (uti + 1) * nrt ? t1 - uti * nrt : nrt;
        for (int rt = rb; rt < re; ++rt) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KSD; ++s) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(img + img_off<D>(16 * rt + l15, 4 * s + l4));
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, fl[s], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, fh[s], acc, 0, 0, 0);
        }
        const int r0 = 16 * rt + 4 * l4;
        if (isP) {
          const float wv = w2s[urow];
          const int col = G::col(urow);
#pragma unroll
          for (int i = 0; i < 4; ++i) Pp[(r0 + i) * PRS + col] = wv * acc[i];
        } else {
          short h[4], l[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) split_bf16(acc[i], h[i], l[i]);
          const int f = urow;
          *reinterpret_cast<uint2*>(Rth + f * LP + r0) =
              make_uint2((uint16_t)h[0] | ((uint32_t)(uint16_t)h[1] << 16), (uint16_t)h[2] | ((uint32_t)(uint16_t)h[3] << 16));
          *reinterpret_cast<uint2*>(Rtl + f * LP + r0) =
              make_uint2((uint16_t)l[0] | ((uint32_t)(uint16_t)l[1] << 16), (uint16_t)l[2] | ((uint32_t)(uint16_t)l[3] << 16));
        }
        }
      }
    }
    if constexpr (!PROJ) {
      if (nchunk > 0) issue_rows();  // chunk 0's rows
    }
    __syncthreads();
    {  // SP / 2 per row: thread = (row, slice)
      const int r = tid >> 3, j = tid & 7;
      float sp = 0.f;
      if (r < nr) {
#pragma unroll
        for (int i = 0; i < SL; ++i) sp += Pp[r * PRS + j * SL + i];
      }
      sp = oct_sum(sp);
      if (j == 0) hSP[r] = 0.5f * sp;
    }
    // (published by the chunk's first barrier)

    int un = a.nU;
    for (int ch = 0; ch < nchunk; ++ch) {
      const int c0 = ch * CH, nc = ctot - c0 < CH ? ctot - c0 : CH;
      int* cvb = cval + (ch & 1) * CH;  // validity of this chunk's candidates (double-buffered)
      // With S apart from the image, the previous chunk's head (which reads S,
      // h1 and the other validity buffer) may still run while the rows land.
      // (PROJ: the store below writes U' over the previous chunk's h1)
      if (!lo_.ssep || ch == 0 || PROJ) __syncthreads();  // (ch == 0: SP published)
      refresh();
      if constexpr (PROJ) {
        store_proj(cvb);  // projected candidates -> U' rows, Q1 rows
      } else {
        store_rows();     // candidate rows -> image
        store_valid(cvb);
      }
      __syncthreads();
      if (ch == 0) un = qslot[1];
      // the next work item: the next chunk, or the next user's history.  Its
      // ids are read now, its rows once Q1 is issued (registers, kept in flight
      // across the scoring; PROJ: the projections are read now)
      const bool nxt_c = ch + 1 < nchunk, nxt_h = !nxt_c && un < a.nU;
      int hid = -1;
      if constexpr (PROJ) {
        if (nxt_c) load_proj(u, coff, clen, c0 + CH);
      } else {
        if (nxt_c) load_cids(u, coff, clen, c0 + CH);
      }
      if (nxt_h) hid = load_hid(un);
      // Q1 tiles of this wave: candidate tile qct = w & 3, F tiles ft = (w >> 2) + 2 i;
      // H1q fragments from LDS, or (when it does not fit) from L2, the first
      // tile's read before the projection
      const int qct = w & 3;
      bf16x8 q1h[KSD], q1l[KSD];
      if constexpr (!lo_.h1l && !PROJ) {
        const int64_t fo = (int64_t)(16 * (w >> 2) + l15) * D + 8 * l4;
        const uint16_t *qh = pinned(a.H1q_hi), *ql = pinned(a.H1q_lo);
#pragma unroll
        for (int s = 0; s < KSD; ++s) {
          q1h[s] = *reinterpret_cast<const bf16x8*>(qh + fo + 32 * s);
          q1l[s] = *reinterpret_cast<const bf16x8*>(ql + fo + 32 * s);
        }
      }
      // ---- 1. U' = w2 (W1q q + b1) -> Us;  Q1 = H1q q tiles -> registers ----
      // (PROJ: both were staged)
      if (proj_on && !PROJ) {
        for (int ct = ct0; ct < ct0 + nct && 16 * ct < nc; ++ct) {  // (empty tiles of a short chunk skipped)
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < KSD; ++s) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(img + img_off<D>(16 * ct + l15, 4 * s + l4));
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wql[s], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wqh[s], acc, 0, 0, 0);
          }
          const int col = G::col(16 * ut + l15);
#pragma unroll
          for (int i = 0; i < 4; ++i) Us[(16 * ct + 4 * l4 + i) * PRS + col] = w2u * (acc[i] + b1u);
        }
      }
      f32x4 q1[NQT];
#pragma unroll
      for (int i = 0; i < NQT; ++i) {
        q1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (PROJ) continue;  // (Q1 staged)
        if constexpr (lo_.h1l) {
          const int f = 16 * ((w >> 2) + 2 * i) + l15;
#pragma unroll
          for (int s = 0; s < KSD; ++s) {
            q1h[s] = *reinterpret_cast<const bf16x8*>(H1qh + img_off<D>(f, 4 * s + l4));
            q1l[s] = *reinterpret_cast<const bf16x8*>(H1ql + img_off<D>(f, 4 * s + l4));
          }
        } else if (i > 0) {  // F > 32: later tiles' fragments are read here
          const int64_t fo = (int64_t)(16 * ((w >> 2) + 2 * i) + l15) * D + 8 * l4;
          const uint16_t *qh = pinned(a.H1q_hi), *ql = pinned(a.H1q_lo);
#pragma unroll
          for (int s = 0; s < KSD; ++s) {
            q1h[s] = *reinterpret_cast<const bf16x8*>(qh + fo + 32 * s);
            q1l[s] = *reinterpret_cast<const bf16x8*>(ql + fo + 32 * s);
          }
        }
        if (16 * qct < nc) {
#pragma unroll
          for (int s = 0; s < KSD; ++s) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(img + img_off<D>(16 * qct + l15, 4 * s + l4));
            q1[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, q1l[s], q1[i], 0, 0, 0);
            q1[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, q1h[s], q1[i], 0, 0, 0);
          }
        }
      }
      if constexpr (PROJ) {
        if (nxt_h) issue_hist_proj(un, hid, vm);  // (U', Q1 were published by the barrier above)
      } else {
        if (nxt_c) issue_rows();
        else if (nxt_h) issue_hist(hid, vm);
        __syncthreads();  // U' published; the image is dead (S takes its place)
      }

      // ---- 2. scoring.  Softmax groups: rows grp, grp + 2, ... (grp = w >> 2); in
      // the exp phase below, lane (pl, sj) of wave w takes the candidate pair cq
      // and the rows grp + 2 sj + 16 k.  A full chunk scores the same way (each
      // wave writes the S rows its own exp phase reads).  A chunk of at most 32
      // candidates spreads its rows over 4 or 8 stripes of waves instead and
      // combines the stripes' maxima through LDS; the max is exact and the
      // scores and the exp / sum order are those of the full layout, so the
      // padded and ragged forms of a list still agree bit for bit.
      constexpr int G = 2;
      const int grp = w >> 2;  // wave-uniform
      const int cq = 2 * (4 * pl + (w & 3));
      const bool spread = nc <= 32;  // uniform
      float m0 = -INFINITY, m1 = -INFINITY;
      // this lane's candidate pair (cx, cx + 1) over rows r0, r0 + rs, ...
      auto score_rows = [&](int cx, int r0, int rs) __attribute__((always_inline)) {
        float u0[SL], u1[SL];
#pragma unroll
        for (int i = 0; i < SL; i += 4) {
          const int o = sj * SL + 4 * G::pos4(sj, i >> 2);
          const float4 x0 = *reinterpret_cast<const float4*>(Us + cx * PRS + o);
          const float4 x1 = *reinterpret_cast<const float4*>(Us + (cx + 1) * PRS + o);
          u0[i] = x0.x; u0[i + 1] = x0.y; u0[i + 2] = x0.z; u0[i + 3] = x0.w;
          u1[i] = x1.x; u1[i + 1] = x1.y; u1[i + 2] = x1.z; u1[i + 3] = x1.w;
        }
        float hsu0 = 0.f, hsu1 = 0.f;
#pragma unroll
        for (int i = 0; i < SL; ++i) {
          hsu0 += u0[i];
          hsu1 += u1[i];
        }
        hsu0 = 0.5f * oct_sum(hsu0);
        hsu1 = 0.5f * oct_sum(hsu1);
        if (__ballot(cx < nc) == 0 || r0 >= nr) return;  // whole waves skip empty pairs
        // a row's P' slice and SP / 2, read one row ahead (two register sets)
        float pa[SL], pb[SL], ha, hb;
        auto load_p = [&](float(&p)[SL], float& h, int r) __attribute__((always_inline)) {
          h = hSP[r];
          const float* pr = Pp + r * PRS + sj * SL;
#pragma unroll
          for (int i = 0; i < SL; i += 4) {
            const float4 x = *reinterpret_cast<const float4*>(pr + 4 * G::pos4(sj, i >> 2));
            p[i] = x.x; p[i + 1] = x.y; p[i + 2] = x.z; p[i + 3] = x.w;
          }
        };
        auto score = [&](const float(&p)[SL], float h, int r) __attribute__((always_inline)) {
          float a0 = 0.f, a1 = 0.f;
#pragma unroll
          for (int i = 0; i < SL; i += 2) {  // two units per packed add
            const f32x2 pv = {p[i], p[i + 1]};
            const f32x2 y0 = f32x2{u0[i], u0[i + 1]} + pv, y1 = f32x2{u1[i], u1[i + 1]} + pv;
            a0 = fmaf(fabsf(y0.x), sgn[i], a0);
            a1 = fmaf(fabsf(y1.x), sgn[i], a1);
            a0 = fmaf(fabsf(y0.y), sgn[i + 1], a0);
            a1 = fmaf(fabsf(y1.y), sgn[i + 1], a1);
          }
          a0 = oct_sum(a0);
          a1 = oct_sum(a1);
          const float s0 = fmaf(0.5f, a0, hsu0 + h), s1 = fmaf(0.5f, a1, hsu1 + h);
          m0 = fmaxf(m0, s0);
          m1 = fmaxf(m1, s1);
          if (sj == 0) {
            S[cx * SST + r] = s0;
            S[(cx + 1) * SST + r] = s1;
          }
        };
        load_p(pa, ha, r0);
        for (int r = r0; r < nr; r += 2 * rs) {
          const bool more = r + rs < nr;
          if (more) load_p(pb, hb, r + rs);
          score(pa, ha, r);
          if (!more) break;
          if (r + 2 * rs < nr) load_p(pa, ha, r + 2 * rs);
          score(pb, hb, r + rs);
        }
      };
      if (!spread) {
        score_rows(cq, grp, G);
      } else {
        // stripes of rows: 8 (one wave each, 8 pairs = 16 candidates) or 4 (wave
        // pairs, two sets of 8 pairs); their maxima in the S rows of candidates
        // 32.. (beyond any spread chunk's candidates)
        const int nst = nc <= 16 ? 8 : 4;
        const int stripe = nc <= 16 ? w : (w >> 1);
        const int cs = 2 * (8 * (nc <= 16 ? 0 : (w & 1)) + pl);
        float* MX = S + 32 * SST;  // [stripe][CH]
        score_rows(cs, stripe, nst);
        if (sj == 0) {
          MX[stripe * CH + cs] = m0;
          MX[stripe * CH + cs + 1] = m1;
        }
        __syncthreads();  // the stripes' scores and maxima published
        m0 = m1 = -INFINITY;
        for (int st = grp; st < nst; st += 2) {  // the stripes holding this group's rows
          m0 = fmaxf(m0, MX[st * CH + cq]);
          m1 = fmaxf(m1, MX[st * CH + cq + 1]);
        }
      }
      // softmax weights of this group's rows: e = exp(s - m_g) (lane sj: every 8th row)
      if (!spread || cq < 32) {
        float sum0 = 0.f, sum1 = 0.f;
        for (int r = grp + G * sj; r < nrp; r += 8 * G) {
          float e0 = 0.f, e1 = 0.f;
          if (r < nr) {
            e0 = __expf(S[cq * SST + r] - m0);
            e1 = __expf(S[(cq + 1) * SST + r] - m1);
            const float wr = r < nv ? 1.f : (float)npad;
            sum0 = fmaf(wr, e0, sum0);
            sum1 = fmaf(wr, e1, sum1);
          }
          S[cq * SST + r] = e0;
          S[(cq + 1) * SST + r] = e1;
        }
        sum0 = oct_sum(sum0);
        sum1 = oct_sum(sum1);
        if (sj == 0) {
          MS[(2 * grp) * CH + cq] = m0;
          MS[(2 * grp) * CH + cq + 1] = m1;
          MS[(2 * grp + 1) * CH + cq] = sum0;
          MS[(2 * grp + 1) * CH + cq + 1] = sum1;
        }
      }
      __syncthreads();  // S (softmax weights), MS published; U' dead (h1 takes its place)

      // ---- 3. h1 = relu(Q1 + (e R) / sum e + c1) ----------------------------
      if (16 * qct < nc) {
        // A operand: candidate ca = 16 qct + l15, rows 32 ks + 8 l4 + jj (group
        // jj mod 2) scaled by exp(m_g - m)
        const int ca = 16 * qct + l15;
        const float ma0 = MS[0 * CH + ca], ma1 = MS[2 * CH + ca], mm = fmaxf(ma0, ma1);
        const float sc0 = __expf(ma0 - mm), sc1 = __expf(ma1 - mm);
        // C tile rows: candidates 16 qct + 4 l4 + i
        float den[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int cc = 16 * qct + 4 * l4 + i;
          const float x0 = MS[0 * CH + cc], x1 = MS[2 * CH + cc], xm = fmaxf(x0, x1);
          den[i] = MS[1 * CH + cc] * __expf(x0 - xm) + MS[3 * CH + cc] * __expf(x1 - xm);
        }
        float rden[4];  // (a hardware reciprocal per candidate row instead of IEEE divisions)
#pragma unroll
        for (int i = 0; i < 4; ++i) rden[i] = __builtin_amdgcn_rcpf(den[i]);  // v_rcp_f32, 1 ulp
        const int nks = nrp / 32;
        bf16x8 eh[2], el[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          if (ks < nks) {
            const float4 x0 = *reinterpret_cast<const float4*>(S + ca * SST + 32 * ks + 8 * l4);
            const float4 x1 = *reinterpret_cast<const float4*>(S + ca * SST + 32 * ks + 8 * l4 + 4);
            const float xv[8] = {x0.x * sc0, x0.y * sc1, x0.z * sc0, x0.w * sc1,
                                 x1.x * sc0, x1.y * sc1, x1.z * sc0, x1.w * sc1};
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
              short h, l;
              split_bf16(xv[jj], h, l);
              eh[ks][jj] = h;
              el[ks][jj] = l;
            }
          }
        }
#pragma unroll
        for (int i = 0; i < NQT; ++i) {
          const int ft = (w >> 2) + 2 * i;
          {
            f32x4 acc;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const float qv = PROJ ? Q1s[(16 * qct + 4 * l4 + k) * F + 16 * ft + l15] : q1[i][k];
              acc[k] = qv * den[k];
            }
            const int f = 16 * ft + l15;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
              if (ks < nks) {
                const bf16x8 rh = *reinterpret_cast<const bf16x8*>(Rth + f * LP + 32 * ks + 8 * l4);
                const bf16x8 rl = *reinterpret_cast<const bf16x8*>(Rtl + f * LP + 32 * ks + 8 * l4);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(el[ks], rh, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(eh[ks], rl, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(eh[ks], rh, acc, 0, 0, 0);
              }
            }
            const float cb = c1s[f];
#pragma unroll
            for (int k = 0; k < 4; ++k) H1s[(16 * qct + 4 * l4 + k) * (F + 4) + f] = fmaxf(acc[k] * rden[k] + cb, 0.f);
          }
        }
      }
      __syncthreads();  // h1 published

      // ---- 4. h2 = relu(H2 h1 + c2), partial logits h3 . h2 per 16-unit tile --
      {
        const int nt2 = 4 * (F2 / 16);
        for (int t = w; t < nt2; t += 8) {
          const int ct = t & 3, t2 = t >> 2;
          if (16 * ct >= nc) continue;  // an empty tile of a short chunk
          const int ca = 16 * ct + l15, v = 16 * t2 + l15;
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
          for (int ks = 0; ks < F / 32; ++ks) {
            const float4 x0 = *reinterpret_cast<const float4*>(H1s + ca * (F + 4) + 32 * ks + 8 * l4);
            const float4 x1 = *reinterpret_cast<const float4*>(H1s + ca * (F + 4) + 32 * ks + 8 * l4 + 4);
            const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            bf16x8 hh, hl;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
              short h, l;
              split_bf16(xv[jj], h, l);
              hh[jj] = h;
              hl[jj] = l;
            }
            const uint16_t* h2h = lo_.h2l ? H2h : pinned(a.H2_hi);
            const uint16_t* h2l = lo_.h2l ? H2l : pinned(a.H2_lo);
            const bf16x8 bh = *reinterpret_cast<const bf16x8*>(h2h + v * F + 32 * ks + 8 * l4);
            const bf16x8 bl = *reinterpret_cast<const bf16x8*>(h2l + v * F + 32 * ks + 8 * l4);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hl, bh, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hh, bl, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hh, bh, acc, 0, 0, 0);
          }
          const float cv = c2s[v], hv = h3s[v];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float z = row_sum16(hv * fmaxf(acc[k] + cv, 0.f));
            const int cc = 16 * ct + 4 * l4 + k;
            if constexpr (F2 == 16) {  // one unit tile: the logit is complete here
              if (l15 == 0 && cc < nc) a.out[ooff + c0 + cc] = cvb[cc] ? a.c3 + z : -INFINITY;
            } else {
              if (l15 == 0) LGP[t2 * CH + cc] = z;
            }
          }
        }
      }
      if constexpr (F2 > 16) {
        __syncthreads();  // partial logits published
        // ---- 5. logits -----------------------------------------------------
        if (tid < nc) {
          float lg = a.c3;
          for (int t2 = 0; t2 < F2 / 16; ++t2) lg += LGP[t2 * CH + tid];
          a.out[ooff + c0 + tid] = cvb[tid] ? lg : -INFINITY;
        }
      }
    }
    if (nchunk == 0) {  // nothing to score: the next user's history still has to be staged
      un = qslot[1];
      if (un < a.nU) {
        if constexpr (PROJ) issue_hist_proj(un, load_hid(un), vm);
        else issue_hist(load_hid(un), vm);
      }
    }
    u = un;
  }
}

template <int D, int A, int F, bool PROJ>
int launch(const RerankArgs& a, hipStream_t st) {
  constexpr Lds<D, A, F, PROJ> l{};
  static_assert(l.total <= 160 * 1024, "din_rerank: LDS");
  int grid = a.nU < 256 ? a.nU : 256;
  hipLaunchKernelGGL((din_rerank_kernel<D, A, F, PROJ>), dim3(grid), dim3(NT), (size_t)l.total, st, a);
  NRK_CHECK_LAUNCH("din_rerank_kernel");
  return NRK_OK;
}

template <int D, int A, bool PROJ>
int launch_f(const RerankArgs& a, hipStream_t st) {
  switch (a.F) {
    case 32: return launch<D, A, 32, PROJ>(a, st);
    case 64: return launch<D, A, 64, PROJ>(a, st);
    case 96: return launch<D, A, 96, PROJ>(a, st);
    default: return launch<D, A, 128, PROJ>(a, st);
  }
}

template <int D, bool PROJ>
int launch_a(int A, const RerankArgs& a, hipStream_t st) {
  switch (A) {
    case 32: return launch_f<D, 32, PROJ>(a, st);
    case 64: return launch_f<D, 64, PROJ>(a, st);
    case 96: return launch_f<D, 96, PROJ>(a, st);
    default: return launch_f<D, 128, PROJ>(a, st);
  }
}

// ---- row projections (nrk_din_rerank_project / _project_hist): the
// row-only halves of the re-rank, so that the main kernel (PROJ) reads
// projections instead of table rows.
//   candidates: [U' = w2 . (W1q q + b1) (A, slice order) | Q1 = H1q q (F)]
//   history slots: [P' = w2 . (W1k k) (A, slice order) | R = H1p k (F)]
// For a bf16 table this is the main kernel's own MFMA sequence (acc += a.Wlo,
// acc += a.Whi per k-step), so its logits stay bit-identical; an f32 table is
// split per element into bf16 hi + lo (16 mantissa bits) and enters as
// acc += lo.Whi, acc += hi.Wlo, acc += hi.Whi (the lo.lo product, 2^-16 of the
// others, is the only term dropped).  64 rows per 256-thread block; wave w
// takes the unit tiles w, w + 4, ... of [Wa ; Wb] (fragments from L2) over the
// block's four 16-row tiles.
struct ProjArgs {
  const void* table;
  int64_t n_table;
  const int32_t* rows;
  int64_t n;
  const uint16_t *Wa_hi, *Wa_lo, *Wb_hi, *Wb_lo;  // [A][d], [F][d]
  const float *b1, *w2;                           // b1: null for the history (P' has no bias)
  int A, F;
  float* out;  // [n][A + F]
};


// A chunk's rows in flight, in registers (no lambdas over arrays: the
// compiler left such captured arrays in scratch).  Thread piece k covers row
// row_of(tid, k); consecutive lanes take consecutive pieces of a row, so each
// load instruction reads whole rows (contiguous bytes).
template <int D, bool F32>
struct ProjStage {  // f32 rows: pieces of 4 floats, split into bf16 hi + lo planes
  static constexpr int PPR = D / 4, NPC = CH * PPR / 512;
  f32x4 v[NPC];
  // (PPR = 64: a wave's pieces are one row, its id wave-uniform: scalar registers)
  __device__ static int row_of(int tid, int k) {
    const int r = (tid + 512 * k) / PPR;
    return PPR == 64 ? __builtin_amdgcn_readfirstlane(r) : r;
  }
  __device__ __forceinline__ void issue(const ProjArgs& a, const int (&idn)[NPC], int tid) {
#pragma unroll
    for (int k = 0; k < NPC; ++k) {
      const int c4 = (tid + 512 * k) % PPR;
      v[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (idn[k] >= 0 && idn[k] < a.n_table)
        v[k] = __builtin_nontemporal_load(
            reinterpret_cast<const f32x4*>(static_cast<const float*>(a.table) + (int64_t)idn[k] * D + 4 * c4));
    }
  }
  __device__ __forceinline__ void store(unsigned char* hi, unsigned char* lo, int tid) const {
#pragma unroll
    for (int k = 0; k < NPC; ++k) {
      const int e = tid + 512 * k, row = e / PPR, c4 = e % PPR;
      bf16x4 h, l;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        short hj, lj;
        split_bf16(v[k][j], hj, lj);
        h[j] = hj;
        l[j] = lj;
      }
      const int o = img_off<D>(row, c4 >> 1) + 8 * (c4 & 1);
      *reinterpret_cast<bf16x4*>(hi + o) = h;
      *reinterpret_cast<bf16x4*>(lo + o) = l;
    }
  }
};
template <int D>
struct ProjStage<D, false> {  // bf16 rows: pieces of 8 elements
  static constexpr int PPR = D / 8, NPC = CH * PPR / 512;
  bf16x8 v[NPC];
  __device__ static int row_of(int tid, int k) { return (tid + 512 * k) / PPR; }
  __device__ __forceinline__ void issue(const ProjArgs& a, const int (&idn)[NPC], int tid) {
#pragma unroll
    for (int k = 0; k < NPC; ++k) {
      const int cc = (tid + 512 * k) % PPR;
      v[k] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (idn[k] >= 0 && idn[k] < a.n_table)
        v[k] = __builtin_nontemporal_load(
            reinterpret_cast<const bf16x8*>(static_cast<const uint16_t*>(a.table) + (int64_t)idn[k] * D + 8 * cc));
    }
  }
  __device__ __forceinline__ void store(unsigned char* hi, unsigned char*, int tid) const {
#pragma unroll
    for (int k = 0; k < NPC; ++k) {
      const int e = tid + 512 * k, row = e / PPR, cc = e % PPR;
      *reinterpret_cast<bf16x8*>(hi + img_off<D>(row, cc)) = v[k];
    }
  }
};

template <int D, bool F32>
__global__ __launch_bounds__(512, 1) void din_rerank_project_kernel(ProjArgs a) {
  // Persistent over 64-row chunks (one workgroup per CU): wave w owns the unit
  // tiles w and w + 8 of [Wa ; Wb] (at most 16), whose hi / lo fragments stay
  // in its registers for the whole launch (no per-chunk L2 re-reads); the next
  // chunk's rows are in flight (registers) during this chunk's MFMAs, their ids
  // one chunk further ahead.  HBM-bound: a chunk's MFMAs (<= 2 tiles x 4 row
  // tiles per wave) take less than its rows' share of the bandwidth.
  constexpr int KSD = D / 32, NT = 512;
  constexpr int NPT = ProjStage<D, F32>::NPC;  // row pieces per thread per chunk
  static_assert(NPT >= 1 && CH * ProjStage<D, F32>::PPR % NT == 0, "din_rerank_project: staging split");
  extern __shared__ __attribute__((aligned(16))) unsigned char pimg[];  // hi image [CH][D] bf16 (+ lo image)
  unsigned char* iml = pimg + CH * D * 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l15 = lane & 15, l4 = lane >> 4;
  const int NUT = a.A / 16, T = NUT + a.F / 16, AF = a.A + a.F;
  const int64_t nchunk = (a.n + CH - 1) / CH;
  const int64_t G = gridDim.x;

  // ---- the wave's tiles: fragments, and where their outputs go
  bf16x8 fh[2][KSD], fl[2][KSD];
  float b1u[2], w2u[2];
  int oc[2];
  bool isA[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int t = w + 8 * j;
    const int tt = t < T ? t : 0;  // (an absent tile loads tile 0's and is skipped)
    isA[j] = tt < NUT;
    const int urow = isA[j] ? 16 * tt + l15 : 16 * (tt - NUT) + l15;
    const uint16_t* bh = (isA[j] ? a.Wa_hi : a.Wb_hi) + (int64_t)urow * D + 8 * l4;
    const uint16_t* bl = (isA[j] ? a.Wa_lo : a.Wb_lo) + (int64_t)urow * D + 8 * l4;
#pragma unroll
    for (int s = 0; s < KSD; ++s) {
      fh[j][s] = *reinterpret_cast<const bf16x8*>(bh + 32 * s);
      fl[j][s] = *reinterpret_cast<const bf16x8*>(bl + 32 * s);
    }
    b1u[j] = isA[j] && a.b1 ? a.b1[urow] : 0.f;
    w2u[j] = isA[j] ? a.w2[urow] : 0.f;
    oc[j] = isA[j] ? slice_col(urow, a.A) : a.A + urow;
  }
  const int ntile = (w < T ? 1 : 0) + (w + 8 < T ? 1 : 0);

  // ---- staging (registers): ids a chunk ahead of the rows they name
  int idn[NPT];
  auto load_ids = [&](int64_t c) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int64_t r = c * CH + ProjStage<D, F32>::row_of(tid, k);
      idn[k] = c < nchunk && r < a.n ? a.rows[r] : -1;
    }
  };
  ProjStage<D, F32> stg;
  int64_t c = blockIdx.x;
  load_ids(c);
  stg.issue(a, idn, tid);
  load_ids(c + G);
  for (; c < nchunk; c += G) {
    __syncthreads();  // the previous chunk's MFMAs are done with the image
    stg.store(pimg, iml, tid);
    __syncthreads();
    if (c + G < nchunk) {  // the next chunk's rows in flight during the MFMAs, the one after's ids
      stg.issue(a, idn, tid);
      load_ids(c + 2 * G);
    }
    const int64_t r0 = c * CH;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j < ntile) {
        // two row tiles at a time, their A fragments one k-step ahead (pinned
        // by scheduling barriers: left alone the scheduler put every MFMA
        // right behind its own LDS read and waited out the latency each time)
#pragma unroll 1
        for (int cp = 0; cp < 2; ++cp) {
          f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
          bf16x8 ah[2][2], al[2][2];  // [buffer][row tile]
          auto rd = [&](int s, int nb) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const int o = img_off<D>(16 * (2 * cp + q) + l15, 4 * s + l4);
              ah[nb][q] = *reinterpret_cast<const bf16x8*>(pimg + o);
              if constexpr (F32) al[nb][q] = *reinterpret_cast<const bf16x8*>(iml + o);
            }
          };
          rd(0, 0);
#pragma unroll
          for (int s = 0; s < KSD; ++s) {
            if (s + 1 < KSD) rd(s + 1, (s + 1) & 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              if constexpr (F32) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[s & 1][q], fh[j][s], acc[q], 0, 0, 0);
              acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[s & 1][q], fl[j][s], acc[q], 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 2; ++q)
              acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[s & 1][q], fh[j][s], acc[q], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
          for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int64_t row = r0 + 16 * (2 * cp + q) + 4 * l4 + i;
              // (candidates: w2 (acc + b1), as the main kernel forms U'; history:
              // w2 acc, as it forms P')
              if (row < a.n) a.out[row * AF + oc[j]] = isA[j] ? w2u[j] * (a.b1 ? acc[q][i] + b1u[j] : acc[q][i]) : acc[q][i];
            }
        }
      }
    }
  }
}

template <int D, bool F32>
int launch_proj(const ProjArgs& a, hipStream_t st) {
  const int64_t nchunk = (a.n + CH - 1) / CH;
  const int grid = nchunk < 256 ? (int)nchunk : 256;  // persistent: one workgroup per CU
  const size_t lds = (size_t)CH * D * 2 * (F32 ? 2 : 1);
  hipLaunchKernelGGL((din_rerank_project_kernel<D, F32>), dim3(grid), dim3(512), lds, st, a);
  NRK_CHECK_LAUNCH("din_rerank_project_kernel");
  return NRK_OK;
}

template <bool F32>
int launch_proj_d(int d, const ProjArgs& a, hipStream_t st) {
  if (d == 256) return launch_proj<256, F32>(a, st);
  if (d == 128) return launch_proj<128, F32>(a, st);
  return launch_proj<64, F32>(a, st);
}


// ---- the evaluate() tail per user (DIN.py:176-189 as pipeline.rerank_clusters
// states it), over the logits of user u = [seg[u], seg[u + 1]): the BCE sum
// over the valid (finite) candidates in f64 (label 1 at pos[u], -1 = none),
// their count, and #{j : p_j > p_pos or (p_j == p_pos and j < pos)} for the
// NDCG rank, p = the sigmoid probabilities the caller computed.  One block per
// user, fixed-order reductions.
__global__ __launch_bounds__(256) void user_stats_kernel(const float* __restrict__ logits, const float* __restrict__ prob,
                                                         const int64_t* __restrict__ seg, const int64_t* __restrict__ pos,
                                                         double* __restrict__ loss_sum, int64_t* __restrict__ nval,
                                                         int64_t* __restrict__ before) {
  const int u = blockIdx.x, tid = threadIdx.x;
  const int64_t lo = seg[u], hi = seg[u + 1];
  const int64_t ps = pos[u] >= lo && pos[u] < hi ? pos[u] : -1;  // (a position outside the user's logits: none)
  const float pp = ps >= 0 ? prob[ps] : 0.f;
  double ls = 0.0;
  int64_t nv = 0, nb = 0;
  for (int64_t i = lo + tid; i < hi; i += 256) {
    const float x = logits[i];
    if (isfinite(x)) {
      const double xd = x;
      ls += (xd > 0.0 ? xd : 0.0) - (i == ps ? xd : 0.0) + log1p(exp(-fabs(xd)));
      ++nv;
    }
    if (ps >= 0) {
      const float p = prob[i];
      nb += (p > pp || (p == pp && i < ps)) ? 1 : 0;
    }
  }
  __shared__ double sl[256];
  __shared__ int64_t sv[256], sb[256];
  sl[tid] = ls;
  sv[tid] = nv;
  sb[tid] = nb;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (tid < h) {
      sl[tid] += sl[tid + h];
      sv[tid] += sv[tid + h];
      sb[tid] += sb[tid + h];
    }
    __syncthreads();
  }
  if (tid == 0) {
    loss_sum[u] = sl[0];
    nval[u] = sv[0];
    before[u] = sb[0];
  }
}

}  // namespace rr
}  // namespace nrk

using namespace nrk;

extern "C" int nrk_din_rerank_workspace(size_t* ws_bytes) {
  NRK_CHECK_ARG(ws_bytes, "din_rerank_workspace: null");
  *ws_bytes = 1024;  // [0, 4): the user queue; [64, 64 + 2 A): sgn(w2) per projection column (f16)
  return NRK_OK;
}

static int rerank_impl(const void* table, int64_t n_table, int32_t dtype, const int32_t* hist, int32_t nU,
                       int32_t L, const int32_t* cand, const int64_t* cand_off, const int32_t* cand_len,
                       const int32_t* extra, const int64_t* out_off, float* out, int32_t d, int32_t A, int32_t F,
                       const nrk_din_rerank_params* p, const float* cand_proj, const float* extra_proj,
                       const float* hist_proj, void* ws, size_t ws_bytes, void* stream) {
  // (the projected form never reads the table: any dtype)
  NRK_CHECK_ARG(cand_proj || dtype == NRK_DTYPE_BF16, "din_rerank: the table must be bf16 (f32: the projected form)");
  NRK_CHECK_ARG(dtype == NRK_DTYPE_BF16 || dtype == NRK_DTYPE_F32, "din_rerank: bad table dtype %d", dtype);
  NRK_CHECK_ARG(d == 64 || d == 128 || d == 256, "din_rerank: emb_dim %d unsupported (64, 128, 256)", d);
  NRK_CHECK_ARG(A >= 32 && A <= 128 && A % 32 == 0, "din_rerank: attn_units %d unsupported (32..128 step 32)", A);
  NRK_CHECK_ARG(F >= 32 && F <= 128 && F % 32 == 0, "din_rerank: fc_units %d unsupported (32..128 step 32)", F);
  const int maxl = cand_proj ? rr::lane_max_l(A, F) : rr::LP;  // (the lane kernel holds up to 128 rows)
  NRK_CHECK_ARG(L >= 1 && L <= maxl, "din_rerank: history length %d unsupported (1..%d)", L, maxl);
  NRK_CHECK_ARG(nU >= 0, "din_rerank: bad user count %d", nU);
  if (nU == 0) return NRK_OK;
  NRK_CHECK_ARG(table && hist && cand_off && cand_len && out_off && out && p && ws, "din_rerank: null pointer");
  NRK_CHECK_ARG(p->W1q_hi && p->W1q_lo && p->W1k_hi && p->W1k_lo && p->b1 && p->w2 && p->H1q_hi && p->H1q_lo &&
                    p->H1p_hi && p->H1p_lo && p->c1 && p->H2_hi && p->H2_lo && p->c2 && p->h3,
                "din_rerank: null parameter pointer");
  NRK_CHECK_ARG(!extra || !cand_proj || extra_proj, "din_rerank_projected: extra without extra_proj");
  NRK_CHECK_ARG(!cand_proj || hist_proj, "din_rerank_projected: null hist_proj");
  if (ws_bytes < 1024) return fail(NRK_EWORKSPACE, "din_rerank: workspace %zu < 1024", ws_bytes);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(ws, 0, 4, st) != hipSuccess) return fail(NRK_ELAUNCH, "din_rerank: memset failed");
  rr::RerankArgs a;
  a.table = static_cast<const uint16_t*>(table);
  a.n_table = n_table;
  a.hist = hist;
  a.L = L;
  a.nU = nU;
  a.cand = cand;
  a.cand_off = cand_off;
  a.cand_len = cand_len;
  a.extra = extra;
  a.out_off = out_off;
  a.out = out;
  a.W1q_hi = static_cast<const uint16_t*>(p->W1q_hi);
  a.W1q_lo = static_cast<const uint16_t*>(p->W1q_lo);
  a.W1k_hi = static_cast<const uint16_t*>(p->W1k_hi);
  a.W1k_lo = static_cast<const uint16_t*>(p->W1k_lo);
  a.b1 = p->b1;
  a.w2 = p->w2;
  a.H1q_hi = static_cast<const uint16_t*>(p->H1q_hi);
  a.H1q_lo = static_cast<const uint16_t*>(p->H1q_lo);
  a.H1p_hi = static_cast<const uint16_t*>(p->H1p_hi);
  a.H1p_lo = static_cast<const uint16_t*>(p->H1p_lo);
  a.c1 = p->c1;
  a.H2_hi = static_cast<const uint16_t*>(p->H2_hi);
  a.H2_lo = static_cast<const uint16_t*>(p->H2_lo);
  a.c2 = p->c2;
  a.h3 = p->h3;
  a.c3 = p->c3;
  a.F = F;
  a.queue = static_cast<int*>(ws);
  a.cproj = cand_proj;
  a.xproj = extra_proj;
  a.hproj = hist_proj;
  a.sgn = static_cast<char*>(ws) + 64;
  // (the projected kernels do not depend on d)
  // the lane kernel: F <= 64, and every F for histories of 65..128 slots
  if (cand_proj && (F <= 64 || L > rr::LP)) return rr::launch_lane(A, a, st);
  if (cand_proj) return rr::launch_a<64, true>(A, a, st);
  if (d == 256) return rr::launch_a<256, false>(A, a, st);
  if (d == 128) return rr::launch_a<128, false>(A, a, st);
  return rr::launch_a<64, false>(A, a, st);
}

extern "C" int nrk_din_rerank(const void* table, int64_t n_table, int32_t dtype, const int32_t* hist, int32_t nU,
                              int32_t L, const int32_t* cand, const int64_t* cand_off, const int32_t* cand_len,
                              const int32_t* extra, const int64_t* out_off, float* out, int32_t d, int32_t A, int32_t F,
                              const nrk_din_rerank_params* p, void* ws, size_t ws_bytes, void* stream) {
  return rerank_impl(table, n_table, dtype, hist, nU, L, cand, cand_off, cand_len, extra, out_off, out, d, A, F, p,
                     nullptr, nullptr, nullptr, ws, ws_bytes, stream);
}

extern "C" int nrk_din_rerank_max_history(int32_t A, int32_t F, int32_t* max_l) {
  NRK_CHECK_ARG(max_l, "din_rerank_max_history: null");
  NRK_CHECK_ARG(A >= 32 && A <= 128 && A % 32 == 0 && F >= 32 && F <= 128 && F % 32 == 0,
                "din_rerank_max_history: A %d / F %d unsupported", A, F);
  *max_l = rr::lane_max_l(A, F);  // (the projected form; nrk_din_rerank itself holds rr::LP)
  return NRK_OK;
}

extern "C" int nrk_din_rerank_projected(const void* table, int64_t n_table, int32_t dtype, const int32_t* hist,
                                        int32_t nU, int32_t L, const int32_t* cand, const int64_t* cand_off,
                                        const int32_t* cand_len, const int32_t* extra, const int64_t* out_off,
                                        float* out, int32_t d, int32_t A, int32_t F, const nrk_din_rerank_params* p,
                                        const float* cand_proj, const float* extra_proj, const float* hist_proj,
                                        void* ws, size_t ws_bytes, void* stream) {
  NRK_CHECK_ARG(cand_proj, "din_rerank_projected: null cand_proj");
  return rerank_impl(table, n_table, dtype, hist, nU, L, cand, cand_off, cand_len, extra, out_off, out, d, A, F, p,
                     cand_proj, extra_proj, hist_proj, ws, ws_bytes, stream);
}

static int project_impl(const char* what, bool hist, const void* table, int64_t n_table, int32_t dtype,
                        const int32_t* rows, int64_t n, int32_t d, int32_t A, int32_t F, const nrk_din_rerank_params* p,
                        float* out, void* stream) {
  NRK_CHECK_ARG(dtype == NRK_DTYPE_BF16 || dtype == NRK_DTYPE_F32, "%s: table dtype %d unsupported (bf16, f32)", what,
                dtype);
  NRK_CHECK_ARG(d == 64 || d == 128 || d == 256, "%s: emb_dim %d unsupported (64, 128, 256)", what, d);
  NRK_CHECK_ARG(A >= 32 && A <= 128 && A % 32 == 0, "%s: attn_units %d unsupported", what, A);
  NRK_CHECK_ARG(F >= 32 && F <= 128 && F % 32 == 0, "%s: fc_units %d unsupported", what, F);
  NRK_CHECK_ARG(n >= 0, "%s: bad row count", what);
  if (n == 0) return NRK_OK;
  NRK_CHECK_ARG(n <= (int64_t)UINT32_MAX * rr::CH, "%s: %lld rows: too many for one launch", what, (long long)n);
  NRK_CHECK_ARG(table && rows && p && out && p->w2, "%s: null pointer", what);
  rr::ProjArgs a;
  a.table = table;
  a.n_table = n_table;
  a.rows = rows;
  a.n = n;
  a.Wa_hi = static_cast<const uint16_t*>(hist ? p->W1k_hi : p->W1q_hi);
  a.Wa_lo = static_cast<const uint16_t*>(hist ? p->W1k_lo : p->W1q_lo);
  a.Wb_hi = static_cast<const uint16_t*>(hist ? p->H1p_hi : p->H1q_hi);
  a.Wb_lo = static_cast<const uint16_t*>(hist ? p->H1p_lo : p->H1q_lo);
  a.b1 = hist ? nullptr : p->b1;
  a.w2 = p->w2;
  a.A = A;
  a.F = F;
  a.out = out;
  NRK_CHECK_ARG(a.Wa_hi && a.Wa_lo && a.Wb_hi && a.Wb_lo && (hist || a.b1), "%s: null parameter pointer", what);
  hipStream_t st = (hipStream_t)stream;
  return dtype == NRK_DTYPE_F32 ? rr::launch_proj_d<true>(d, a, st) : rr::launch_proj_d<false>(d, a, st);
}

extern "C" int nrk_din_rerank_project(const void* table, int64_t n_table, int32_t dtype, const int32_t* rows, int64_t n,
                                      int32_t d, int32_t A, int32_t F, const nrk_din_rerank_params* p, float* out,
                                      void* stream) {
  return project_impl("din_rerank_project", false, table, n_table, dtype, rows, n, d, A, F, p, out, stream);
}

extern "C" int nrk_din_rerank_project_hist(const void* table, int64_t n_table, int32_t dtype, const int32_t* rows,
                                           int64_t n, int32_t d, int32_t A, int32_t F, const nrk_din_rerank_params* p,
                                           float* out, void* stream) {
  return project_impl("din_rerank_project_hist", true, table, n_table, dtype, rows, n, d, A, F, p, out, stream);
}

extern "C" int nrk_rerank_user_stats(const float* logits, const float* prob, const int64_t* seg_off, const int64_t* pos,
                                     int32_t nU, double* loss_sum, int64_t* nval, int64_t* before, void* stream) {
  NRK_CHECK_ARG(nU >= 0, "rerank_user_stats: bad user count %d", nU);
  if (nU == 0) return NRK_OK;
  NRK_CHECK_ARG(logits && prob && seg_off && pos && loss_sum && nval && before, "rerank_user_stats: null pointer");
  hipLaunchKernelGGL(rr::user_stats_kernel, dim3(nU), dim3(256), 0, (hipStream_t)stream, logits, prob, seg_off, pos,
                     loss_sum, nval, before);
  NRK_CHECK_LAUNCH("user_stats_kernel");
  return NRK_OK;
}
