// screen16.h — the flat inner-product main pass (K-GEMM-TOPK, screen MODE 0) on
// v_mfma_f32_16x16x32_bf16.  Same contract, grid, LDS staging and outputs as
// screen_kernel<DP, QT, M, WAVES, false, 0, *, true, TIL> (screen.h): every
// (query, chunk) gets two lane streams of M candidates + their (M+1)-th score.
//
// Why a second form: per FLOP the 16x16x32 instruction takes the same cycles
// as 32x32x16, but on random data the chip holds a higher clock under it
// (MI355X_MICROARCH.md: ~1.12-1.15x FLOP/s in bare loops), and the main pass is
// MFMA-bound.
//
// Layout.  A = items (16 rows), B = queries (16 columns), K = 32 per MFMA.  A
// wave's QT tiles of 32 queries are 2 QT half-tiles of 16; lane l holds query
// (l & 15) of every half-tile and items 4 (l >> 4) + v (v < 4) of every 16-item
// half of a 32-item sub-tile, so each (query, chunk) is scanned by FOUR lane
// streams (lane groups g = l >> 4).  At the end the lists of groups g and g ^ 2
// (lanes l and l ^ 32) are merged into one top-(M+1) list: the merged (M+1)-th
// score bounds every item either stream left out (each stream's own (M+1)-th
// entry is in the union the merged list is the top of), so the two merged
// streams per (query, chunk) satisfy exactly what merge_rescore_kernel assumes
// of the two lane halves of the 32x32 form.
#pragma once

#include "screen.h"

namespace nrk {

// sorted (descending score, ascending id on ties) insertion for list merges
template <int N>
__device__ __forceinline__ void list_insert_tie(float (&ls)[N], int (&li)[N], float v, int id) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const bool gt = v > ls[j] || (v == ls[j] && id < li[j]);
    const float ts = gt ? v : ls[j];
    const int ti = gt ? id : li[j];
    v = gt ? ls[j] : v;
    id = gt ? li[j] : id;
    ls[j] = ts;
    li[j] = ti;
  }
}

// PD: A-fragment prefetch depth in K steps.  Each K step's two fragments are read
// PD steps before their MFMAs, into a ring of 2 PD registers sets: PD = DP / 32
// reads the whole next sub-tile during the current chain; a shallower ring
// (the M = 16 lists, which would not fit beside a full prefetch) reads the
// current sub-tile's later steps during its own chain, so the tile being
// consumed is never the refill target: three LDS buffers instead of two.
template <int DP, int QT, int M, int WAVES, int TIL, bool SCHED = true, int PD = DP / 32>
__global__ __launch_bounds__(WAVES * 64, 2) void screen16_kernel(
    const uint16_t* __restrict__ qh, const uint16_t* __restrict__ xbh, const float* __restrict__ xmeta, int64_t nq,
    int64_t nb, int64_t chunk, int nch, int nqt, int tstride, float* __restrict__ part_s, int* __restrict__ part_i,
    float* __restrict__ part_t, const float* __restrict__ tau_q, IvfScreen iv) {
  (void)xmeta;
  (void)tstride;
  (void)iv;
  constexpr int CPR = DP / 8;   // 16-B chunks per row
  constexpr int TI = TIL;       // items per tile between barriers
  constexpr int NSUB = TI / 32; // 32-item sub-tiles per tile
  static_assert(NSUB % 2 == 0, "sub-tiles alternate between two accumulator sets");
  constexpr int TCH = TI * CPR;
  constexpr int NT = WAVES * 64;
  constexpr int GPT = TCH / NT;
  static_assert(TCH % NT == 0, "tile must split evenly over the workgroup");
  constexpr int KS2 = DP / 32;  // K steps of 32
  constexpr int NQ2 = 2 * QT;   // 16-query half-tiles per wave
  constexpr int WQ = WAVES * 32 * QT;
  constexpr int BUF = TI * DP;
  static_assert(PD >= 1 && PD <= KS2 && KS2 % PD == 0, "prefetch depth: a divisor of the K steps (fragment ring)");
  constexpr int NBUF = PD == KS2 ? 2 : 3;
  __shared__ __attribute__((aligned(16))) uint16_t lds[NBUF * BUF];

  const int nblk = gridDim.x, b = blockIdx.x;
  const int xg = b & 7, jj = b >> 3, q8 = nblk >> 3, r8 = nblk & 7;
  const int logical = (xg < r8 ? xg * (q8 + 1) : r8 * (q8 + 1) + (xg - r8) * q8) + jj;
  const int c = logical / nqt, qt = logical - c * nqt;
  const int64_t ibeg = (int64_t)c * chunk;
  const int64_t iend = ibeg + chunk < nb ? ibeg + chunk : nb;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int q16 = lane & 15, g = lane >> 4;
  const int ntiles = (int)cdiv(iend - ibeg, TI);

  bf16x8 qf[NQ2][KS2];
  int64_t qidx[NQ2];
  float tau[NQ2];
  float ls[NQ2][M + 1];
  int li[NQ2][M + 1];
#pragma unroll
  for (int t = 0; t < NQ2; ++t) {
    qidx[t] = (int64_t)qt * WQ + (int64_t)w * QT * 32 + 16 * t + q16;  // < nq_pad (zero rows)
    const bf16x8* src = reinterpret_cast<const bf16x8*>(qh + qidx[t] * DP + 8 * g);
#pragma unroll
    for (int s = 0; s < KS2; ++s) qf[t][s] = src[4 * s];
    tau[t] = (tau_q && qidx[t] < nq) ? tau_q[qidx[t]] : -INFINITY;
#pragma unroll
    for (int j = 0; j <= M; ++j) {
      ls[t][j] = -INFINITY;
      li[t][j] = -1;
    }
  }

  const int64_t cnt = iend - ibeg > 0 ? iend - ibeg : 0;
  const BufRsrc xrs = make_rsrc(xbh + ibeg * DP, (int)(cnt * DP * 2));
  int voff[GPT];
#pragma unroll
  for (int u = 0; u < GPT; ++u) {
    const int p = u * NT + tid;
    const int row = p / CPR, pc = p % CPR;
    voff[u] = row * DP * 2 + 16 * (pc ^ swz<CPR>(row));
  }
  auto issue_tile = [&](int it, auto buf_c) {
    constexpr int buf = decltype(buf_c)::value;
    const int soff = it * TI * DP * 2;
#pragma unroll
    for (int u = 0; u < GPT; ++u) buffer_load_lds16(xrs, lds + buf * BUF + (u * NT + w * 64) * 8, voff[u], soff);
  };
  // A fragment: row `row` of a tile image, K step s (lane group g reads chunk 4 s + g)
  auto afrag = [&](const uint16_t* tl, int row, int s) {
    return *reinterpret_cast<const bf16x8*>(tl + row * DP + 8 * ((4 * s + g) ^ swz<CPR>(row)));
  };

  // deferred epilogue: sub-tile s's scores are reduced while sub-tile s+1's
  // MFMA chain runs (A: even sub-tiles, B: odd ones)
  f32x4 accA[NQ2][2], accB[NQ2][2];
  int64_t baseA = -1, baseB = -1;
  int nvA = 0, nvB = 0;
  bf16x8 af[2][PD];
  auto mask_rows = [&](f32x4 (&pa)[NQ2][2], int nv) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < NQ2; ++t)
#pragma unroll
      for (int ih = 0; ih < 2; ++ih)
#pragma unroll
        for (int v = 0; v < 4; ++v)
          if (16 * ih + 4 * g + v >= nv) pa[t][ih][v] = -INFINITY;
  };
  auto tree = [&](f32x4 (&pa)[NQ2][2], float (&m2)[NQ2][2], float (&m)[NQ2]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < NQ2; ++t) {
#pragma unroll
      for (int ih = 0; ih < 2; ++ih)
        m2[t][ih] = fmax_ieee(fmax_ieee(pa[t][ih][0], pa[t][ih][1]), fmax_ieee(pa[t][ih][2], pa[t][ih][3]));
      m[t] = fmax_ieee(m2[t][0], m2[t][1]);
    }
  };
  auto drain = [&](f32x4 (&pa)[NQ2][2], int64_t pbase, const float (&m2)[NQ2][2], const float (&m)[NQ2])
      __attribute__((always_inline)) {
    bool hit = false;
#pragma unroll
    for (int t = 0; t < NQ2; ++t) hit |= m[t] > fmaxf(ls[t][M], tau[t]);
    if (!__any(hit)) return;
#pragma unroll
    for (int t = 0; t < NQ2; ++t) {
      if (__any(m[t] > fmaxf(ls[t][M], tau[t]))) {
#pragma unroll
        for (int ih = 0; ih < 2; ++ih) {
          if (__any(m2[t][ih] > fmaxf(ls[t][M], tau[t]))) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const float thr = fmaxf(ls[t][M], tau[t]);
              if (pa[t][ih][v] > thr)
                list_insert<M + 1>(ls[t], li[t], pa[t][ih][v], (int)(pbase + 16 * ih + 4 * g + v));
            }
          }
        }
      }
    }
  };
  auto sub_tile = [&](auto st_c, int64_t i0, int nvalid, const uint16_t* next_tl, const uint16_t* cur_tl)
      __attribute__((always_inline)) {
    constexpr int st = decltype(st_c)::value;
    constexpr int par = st & 1;
    f32x4(&cur)[NQ2][2] = par ? accB : accA;
    f32x4(&pend)[NQ2][2] = par ? accA : accB;
    const int64_t pbase = par ? baseA : baseB;
    const int pnv = par ? nvA : nvB;
    if (pbase >= 0 && pnv < 32) mask_rows(pend, pnv);
    // next sub-tile: the next 32 rows of this tile, or rows 0..31 of the next tile
    const int nrow = (st + 1 < NSUB ? 32 * (st + 1) : 0) + q16;
    const f32x4 zero = {};
#pragma unroll
    for (int s = 0; s < KS2; ++s) {
#pragma unroll
      for (int ih = 0; ih < 2; ++ih) {
#pragma unroll
        for (int t = 0; t < NQ2; ++t)
          cur[t][ih] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ih][s % PD], qf[t][s],
                                                             s == 0 ? zero : cur[t][ih], 0, 0, 0);
        // refill the slot with the fragment PD steps ahead: this sub-tile's, or the next one's
        if (s + PD < KS2) af[ih][s % PD] = afrag(cur_tl, 32 * st + 16 * ih + q16, s + PD);
        else af[ih][s % PD] = afrag(next_tl, nrow + 16 * ih, s + PD - KS2);
      }
    }
    float m2[NQ2][2], m[NQ2];
    tree(pend, m2, m);
#pragma unroll
    for (int t = 0; t < NQ2; ++t) m[t] = pbase >= 0 ? m[t] : -INFINITY;  // nothing pending: drain is a no-op
    if constexpr (SCHED) {
#pragma unroll
      for (int s = 0; s < 2 * KS2; ++s) {
        __builtin_amdgcn_sched_group_barrier(0x008, NQ2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 2 * NQ2 > 6 ? 6 : 2 * NQ2, 0);
      }
    }
    drain(pend, pbase, m2, m);
    if constexpr (par == 0) {
      baseA = i0 + 32 * st;
      nvA = nvalid - 32 * st;
    } else {
      baseB = i0 + 32 * st;
      nvB = nvalid - 32 * st;
    }
  };
  auto tile_d = [&](int it, auto buf_c) __attribute__((always_inline)) {
    constexpr int buf = decltype(buf_c)::value;
    constexpr int nbuf = (buf + 1) % NBUF;  // tile it + 1
    constexpr int rbuf = (buf + 2) % NBUF;  // refilled with tile it + 2
    const uint16_t* tl = lds + buf * BUF;
    const int64_t i0 = ibeg + (int64_t)it * TI;
    const int nvalid = (int)((iend - i0) < TI ? (iend - i0) : TI);
    sub_tile(std::integral_constant<int, 0>{}, i0, nvalid, tl, tl);
    if constexpr (NSUB == 4) {
      sub_tile(std::integral_constant<int, 1>{}, i0, nvalid, tl, tl);
      sub_tile(std::integral_constant<int, 2>{}, i0, nvalid, tl, tl);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // tile it+1 landed; every wave is done with rbuf: with two buffers the last
    // sub-tile's fragments are all in registers already (PD = K steps), with
    // three rbuf held tile it-1, which every wave has finished
    __syncthreads();
    if (it + 2 < ntiles) issue_tile(it + 2, std::integral_constant<int, rbuf>{});
    sub_tile(std::integral_constant<int, NSUB - 1>{}, i0, nvalid, lds + nbuf * BUF, tl);
  };
  if (ntiles > 0) {
    issue_tile(0, std::integral_constant<int, 0>{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // tile 0 landed
    if (ntiles > 1) issue_tile(1, std::integral_constant<int, 1>{});
#pragma unroll
    for (int ih = 0; ih < 2; ++ih)
#pragma unroll
      for (int s = 0; s < PD; ++s) af[ih][s] = afrag(lds, 16 * ih + q16, s);
  }
  for (int it = 0; it < ntiles; it += NBUF) {
    tile_d(it, std::integral_constant<int, 0>{});
    if (it + 1 < ntiles) tile_d(it + 1, std::integral_constant<int, 1>{});
    if constexpr (NBUF == 3) {
      if (it + 2 < ntiles) tile_d(it + 2, std::integral_constant<int, 2 % NBUF>{});
    }
  }
  if (baseB >= 0) {  // the last sub-tile's epilogue
    if (nvB < 32) mask_rows(accB, nvB);
    float m2[NQ2][2], m[NQ2];
    tree(accB, m2, m);
    drain(accB, baseB, m2, m);
  }

  // merge the streams of lane groups g and g ^ 2, write from groups 0 and 1
#pragma unroll
  for (int t = 0; t < NQ2; ++t) {
    float ps[M + 1];
    int pi[M + 1];
#pragma unroll
    for (int j = 0; j <= M; ++j) {
      ps[j] = __shfl_xor(ls[t][j], 32);
      pi[j] = __shfl_xor(li[t][j], 32);
    }
    if (g < 2) {
#pragma unroll
      for (int j = 0; j <= M; ++j) list_insert_tie<M + 1>(ls[t], li[t], ps[j], pi[j]);
      const int64_t qi = qidx[t];
      if (qi < nq) {
        const int64_t base = (qi * nch + c) * 2 + g;
#pragma unroll
        for (int j = 0; j < M; ++j) {
          part_s[base * M + j] = ls[t][j];
          part_i[base * M + j] = li[t][j];
        }
        part_t[base] = ls[t][M];
      }
    }
  }
}

// IVF collect (screen.h MODE 3) on v_mfma_f32_16x16x32_bf16: MODE 3's work items
// (a list chunk x a tile of the list's probing queries, a persistent grid over the
// device work table) and its LDS candidate staging, in screen16's layout with the
// deferred epilogue.  A wave runs the MFMAs of its 16-query half-tiles up to the
// last one holding a real probing query: list segments are padded to the work
// item's rows, and the padding a wave still computes is now < 16 rows instead of
// < 32.  L2: the accumulators start at -|x|^2 / 2 (the rows' norms are staged
// with each tile), so they end at s / 2 for the score s = 2 ip - |x|^2 and the
// epilogue compares them with half the threshold (collect_threshold's bound
// covers the roundings of the norm inside the MFMA chain).
template <int DP, int QT, int WAVES, int TIL, bool L2, int NB = 2>
__global__ __launch_bounds__(WAVES * 64, 2) void screen16_collect_kernel(
    const uint16_t* __restrict__ qh, const uint16_t* __restrict__ xbh, const float* __restrict__ xmeta, int64_t nq,
    int64_t nb, int64_t chunk, int nch, int nqt, int tstride, float* __restrict__ part_s, int* __restrict__ part_i,
    float* __restrict__ part_t, const float* __restrict__ tau_q, IvfScreen iv) {
  (void)chunk;
  (void)nch;
  (void)nqt;
  (void)tstride;
  (void)part_s;
  (void)part_i;
  (void)part_t;
  (void)tau_q;
  constexpr int CPR = DP / 8;
  constexpr int TI = TIL;
  constexpr int NSUB = TI / 32;
  static_assert(NSUB % 2 == 0, "sub-tiles alternate between two accumulator sets");
  constexpr int TCH = TI * CPR;
  constexpr int NT = WAVES * 64;
  constexpr int GPT = TCH / NT;
  static_assert(TCH % NT == 0, "tile must split evenly over the workgroup");
  constexpr int KS2 = DP / 32;
  constexpr int NQ2 = 2 * QT;
  constexpr int WQ = WAVES * 32 * QT;
  static_assert(WQ <= 1024, "collect rows: 10 bits");
  constexpr int BUF = TI * DP;  // uint16 per buffer
  // NB tile buffers: at tile it's barrier tile it + NB is issued into tile it's
  // buffer (its last sub-tile's A fragments are all in registers), NB - 1 tiles
  // ahead of its use
  constexpr int PD = KS2;
  static_assert(NB >= 2 && NB <= 4, "tile buffers");
  constexpr int NSLOT = NB + 1;
  typedef CollectLds<WQ> CL;
  __shared__ __attribute__((aligned(16))) uint16_t lds[NB * BUF];
  // L2: the tiles' row norms in a ring of NB + 1 slots (tile it in slot it % (NB + 1))
  __shared__ __attribute__((aligned(16))) float nrm[L2 ? NSLOT * TI : 4];
  __shared__ CL cl;
  __shared__ int next_item;

  // Work items are split into 8 contiguous ranges, one per XCD (block b runs on
  // XCD b mod 8), and each XCD's workgroups take its items in order from a
  // ticket counter: the query tiles of a list chunk start together on one XCD
  // (the chunk is read once into its L2), and items of uneven cost (partly
  // filled query tiles, short list tails) balance dynamically.
  const int nblk = gridDim.x, b = blockIdx.x;
  const int nx = nblk >= 8 ? 8 : 1, xg = b % nx;
  const int total = iv.work_off[iv.nlist];
  const int per = total / nx, rem = total % nx;
  const int xbeg = xg < rem ? xg * (per + 1) : rem * (per + 1) + (xg - rem) * per;
  const int xend = xbeg + per + (xg < rem ? 1 : 0);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q16 = lane & 15, g = lane >> 4;
  if (tid == 0) next_item = xbeg + atomicAdd(&iv.ticket[xg], 1);
  for (;;) {
    __syncthreads();  // next_item published; the previous item is done with the LDS buffers and staging
    const int logical = next_item;
    if (logical >= xend) break;
    int nxt = 0;  // the following item's ticket, fetched under this item's work
    if (tid == 0) nxt = xbeg + atomicAdd(&iv.ticket[xg], 1);
    int lo = 0, hi = iv.nlist;  // largest l with work_off[l] <= logical (empty lists own no items)
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (iv.work_off[mid] <= logical) lo = mid;
      else hi = mid;
    }
    const int64_t lb = iv.list_off[lo], le = iv.list_off[lo + 1];
    const int nchl = (int)cdiv(le - lb, (int64_t)iv.ch);
    const int local = logical - iv.work_off[lo];
    const int nqtl = (iv.work_off[lo + 1] - iv.work_off[lo]) / nchl;
    const int c = local / nqtl, qt = local - c * nqtl;  // query tile innermost (the chunk stays in L2)
    const int64_t ibeg = lb + (int64_t)c * iv.ch;
    const int64_t iend = ibeg + iv.ch < le ? ibeg + iv.ch : le;
    const int64_t seg0 = iv.seg_off[lo];

    bf16x8 qf[NQ2][KS2];
    float cthr[NQ2];  // collect threshold of the lane's query (+inf: padding row)
    // (Wave-major rows: a wave's half-tiles share each A fragment.  Spreading a
    // partly filled item's rows over all waves measured slower, 2.99 -> 3.10 ms.)
    int nact = 0;     // half-tiles up to the last one holding a real row (padding is a suffix)
#pragma unroll
    for (int t = 0; t < NQ2; ++t) {
      const int row = w * QT * 32 + 16 * t + q16;
      const int64_t gr = seg0 + (int64_t)qt * WQ + row;
      const bf16x8* src = reinterpret_cast<const bf16x8*>(qh + gr * DP + 8 * g);
#pragma unroll
      for (int s = 0; s < KS2; ++s) qf[t][s] = src[4 * s];
      const int pair = iv.slot_pair[gr];
      const int qy = pair >= 0 ? pair / iv.nprobe : -1;
      cthr[t] = pair >= 0 ? (L2 ? 0.5f : 1.f) * iv.thr_q[qy] : INFINITY;  // (L2: scores held halved)
      if (g == 0) {
        cl.qid[row] = qy;
        cl.qcnt[row] = 0;
      }
      if (__any(pair >= 0)) nact = t + 1;
    }
    nact = __builtin_amdgcn_readfirstlane(nact);
    if (tid == 0) cl.n = 0;  // ordered before any append by the first tile's barrier

    const int64_t cnt = iend - ibeg > 0 ? iend - ibeg : 0;
    const i32x4 xrs = dma_rsrc(xbh + ibeg * DP, (int)(cnt * DP * 2));
    const i32x4 nrs = dma_rsrc(xmeta + 2 * ibeg, (int)(cnt * 8));
    const int ntiles = (int)cdiv(cnt, (int64_t)TI);
    // a thread's rows of a tile are NT / CPR apart, a multiple of the swizzle's
    // 16-row period: one vector offset, the rest in the scalar offset
    static_assert((NT / CPR) % 16 == 0, "staging rows per pass: a multiple of the swizzle period");
    const int voff = (tid / CPR) * DP * 2 + 16 * ((tid % CPR) ^ swz<CPR>(tid / CPR));
    auto issue_tile = [&](int it, auto buf_c) {
      constexpr int buf = decltype(buf_c)::value;
      const int soff = it * TI * DP * 2;
#pragma unroll
      for (int u = 0; u < GPT; ++u)
        dma_lds<16>(xrs, lds + buf * BUF + (u * NT + w * 64) * 8, voff, soff + u * (NT / CPR) * DP * 2);
      if constexpr (L2) {
        if (w == 0) {
          float* ns = nrm + (it % NSLOT) * TI;
#pragma unroll
          for (int u = 0; u < TI / 64; ++u) dma_lds<4>(nrs, ns + 64 * u, lane * 8, it * TI * 8 + 512 * u);
        }
      }
    };
    auto afrag = [&](const uint16_t* tl, int row, int s) {
      return *reinterpret_cast<const bf16x8*>(tl + row * DP + 8 * ((4 * s + g) ^ swz<CPR>(row)));
    };
    // wait until at most k tiles' DMA (the k issued last) are outstanding
    auto wait_tiles = [&](int k) __attribute__((always_inline)) {
      constexpr int LPT = GPT;                        // loads per tile and thread
      constexpr int LPT0 = GPT + (L2 ? TI / 64 : 0);  // wave 0: + the norms
      auto wc = [](auto n_c) {
        constexpr int n = decltype(n_c)::value;  // vmcnt only (expcnt, lgkmcnt at their maxima)
        __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8));
      };
      if (k <= 0) wc(std::integral_constant<int, 0>{});
      else if (NB < 3 || k == 1) {
        if (w == 0) wc(std::integral_constant<int, LPT0>{});
        else wc(std::integral_constant<int, LPT>{});
      } else {
        if (w == 0) wc(std::integral_constant<int, 2 * LPT0>{});
        else wc(std::integral_constant<int, 2 * LPT>{});
      }
    };
    // staged append of one candidate (position pos) of half-tile t's query
    auto append = [&](int t, int pos) __attribute__((always_inline)) {
      const int e = atomicAdd(&cl.n, 1);
      if (e < CL::CAP) {
        const int row = w * QT * 32 + 16 * t + q16;
        const int rank = atomicAdd(&cl.qcnt[row], 1);
        cl.ent[e] = make_int2(row | (rank << 10), pos);
      } else {
        const int qy = cl.qid[w * QT * 32 + 16 * t + q16];
        if (guard_ok((uint64_t)qy < (uint64_t)nq, iv.err, GUARD_COLLECT_QUERY) &&
            guard_ok((uint64_t)pos < (uint64_t)nb, iv.err, GUARD_COLLECT_POS) &&
            __builtin_nontemporal_load(&iv.cand_cnt[qy]) <= iv.cap) {
          // staging full: append directly (stop once the query overflowed)
          const int slot = atomicAdd(&iv.cand_cnt[qy], 1);
          if (slot < iv.cap) iv.cand_pos[(int64_t)qy * iv.cap + slot] = pos;
        }
      }
    };

    // the tile pipeline for NA active half-tiles (NA = 0: staging and barriers only)
    auto run = [&](auto na_c) __attribute__((always_inline)) {
      constexpr int NA = decltype(na_c)::value;
      f32x4 accA[NQ2][2], accB[NQ2][2];
      int64_t baseA = -1, baseB = -1;
      int nvA = 0, nvB = 0;
      bf16x8 af[2][PD];
      auto mask_rows = [&](f32x4 (&pa)[NQ2][2], int nv) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < NA; ++t)
#pragma unroll
          for (int ih = 0; ih < 2; ++ih)
#pragma unroll
            for (int v = 0; v < 4; ++v)
              if (16 * ih + 4 * g + v >= nv) pa[t][ih][v] = -INFINITY;
      };
      // L2: -|x|^2 / 2 of the next chain's rows 16 ih + 4 g + v (its accumulators' start)
      f32x4 ninit[2];
      auto load_ninit = [&](const float* ns, int row0) __attribute__((always_inline)) {
#pragma unroll
        for (int ih = 0; ih < 2; ++ih) {
          const float4 x = *reinterpret_cast<const float4*>(ns + row0 + 16 * ih + 4 * g);
          ninit[ih] = f32x4{-0.5f * x.x, -0.5f * x.y, -0.5f * x.z, -0.5f * x.w};
        }
      };
      auto tree = [&](f32x4 (&pa)[NQ2][2], float (&m2)[NQ2][2], float (&m)[NQ2]) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < NA; ++t) {
#pragma unroll
          for (int ih = 0; ih < 2; ++ih) {
            m2[t][ih] = fmax_ieee(fmax_ieee(pa[t][ih][0], pa[t][ih][1]), fmax_ieee(pa[t][ih][2], pa[t][ih][3]));
          }
          m[t] = fmax_ieee(m2[t][0], m2[t][1]);
        }
      };
      auto drain = [&](f32x4 (&pa)[NQ2][2], int64_t pbase, const float (&m2)[NQ2][2], const float (&m)[NQ2])
          __attribute__((always_inline)) {
        bool hit = false;
#pragma unroll
        for (int t = 0; t < NA; ++t) hit |= m[t] >= cthr[t];
        if (!__any(hit)) return;
#pragma unroll
        for (int t = 0; t < NA; ++t) {
          if (__any(m[t] >= cthr[t])) {
#pragma unroll
            for (int ih = 0; ih < 2; ++ih) {
              if (__any(m2[t][ih] >= cthr[t])) {
#pragma unroll
                for (int v = 0; v < 4; ++v)
                  if (pa[t][ih][v] >= cthr[t]) append(t, (int)(pbase + 16 * ih + 4 * g + v));
              }
            }
          }
        }
      };
      auto sub_tile = [&](auto st_c, int64_t i0, int nvalid, const uint16_t* next_tl, const uint16_t* cur_tl,
                          const float* cur_ns, const float* next_ns) __attribute__((always_inline)) {
        constexpr int st = decltype(st_c)::value;
        constexpr int par = st & 1;
        f32x4(&cur)[NQ2][2] = par ? accB : accA;
        f32x4(&pend)[NQ2][2] = par ? accA : accB;
        const int64_t pbase = par ? baseA : baseB;
        const int pnv = par ? nvA : nvB;
        if (pbase >= 0 && pnv < 32) mask_rows(pend, pnv);
        const int nrow = (st + 1 < NSUB ? 32 * (st + 1) : 0) + q16;
        const f32x4 zero = {};
#pragma unroll
        for (int s = 0; s < KS2; ++s) {
#pragma unroll
          for (int ih = 0; ih < 2; ++ih) {
#pragma unroll
            for (int t = 0; t < NA; ++t)
              cur[t][ih] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ih][s % PD], qf[t][s],
                                                                   s == 0 ? (L2 ? ninit[ih] : zero) : cur[t][ih], 0, 0, 0);
            if (s + PD < KS2) af[ih][s % PD] = afrag(cur_tl, 32 * st + 16 * ih + q16, s + PD);
            else af[ih][s % PD] = afrag(next_tl, nrow + 16 * ih, s + PD - KS2);
          }
        }
        // the next chain's norms: this tile's next sub-tile, or the next tile's first
        // (landed: the last sub-tile runs after the tile barrier)
        if constexpr (L2) {
          if constexpr (st + 1 < NSUB) load_ninit(cur_ns, 32 * (st + 1));
          else load_ninit(next_ns, 0);
        }
        (void)cur_ns;
        (void)next_ns;
        float m2[NQ2][2], m[NQ2];
        tree(pend, m2, m);
#pragma unroll
        for (int t = 0; t < NA; ++t) m[t] = pbase >= 0 ? m[t] : -INFINITY;  // nothing pending: drain is a no-op
        drain(pend, pbase, m2, m);
        if constexpr (par == 0) {
          baseA = i0 + 32 * st;
          nvA = nvalid - 32 * st;
        } else {
          baseB = i0 + 32 * st;
          nvB = nvalid - 32 * st;
        }
      };
      auto tile_d = [&](int it, auto buf_c) __attribute__((always_inline)) {
        constexpr int buf = decltype(buf_c)::value;
        constexpr int nbuf = (buf + 1) % NB;
        const uint16_t* tl = lds + buf * BUF;
        const int64_t i0 = ibeg + (int64_t)it * TI;
        const int nvalid = (int)((iend - i0) < TI ? (iend - i0) : TI);
        const float* ns = nrm + (it % NSLOT) * TI;            // (L2 only)
        const float* nns = nrm + ((it + 1) % NSLOT) * TI;
        sub_tile(std::integral_constant<int, 0>{}, i0, nvalid, tl, tl, ns, nns);
        if constexpr (NSUB == 4) {
          sub_tile(std::integral_constant<int, 1>{}, i0, nvalid, tl, tl, ns, nns);
          sub_tile(std::integral_constant<int, 2>{}, i0, nvalid, tl, tl, ns, nns);
        }
        // tile it+1 landed (tiles up to it + NB - 1 were issued); every wave is done
        // with this tile's rows and with norm slot (it + NB) % (NB + 1) (tile it-1's
        // norms were last read before this tile)
        wait_tiles(ntiles - 2 - it < NB - 2 ? ntiles - 2 - it : NB - 2);
        __syncthreads();
        if (it + NB < ntiles) issue_tile(it + NB, buf_c);
        sub_tile(std::integral_constant<int, NSUB - 1>{}, i0, nvalid, lds + nbuf * BUF, tl, ns, nns);
      };
      if (ntiles > 0) {
        issue_tile(0, std::integral_constant<int, 0>{});
        if (ntiles > 1) issue_tile(1, std::integral_constant<int, 1 % NB>{});
        if constexpr (NB >= 3) {
          if (ntiles > 2) issue_tile(2, std::integral_constant<int, 2 % NB>{});
        }
        if constexpr (NB >= 4) {
          if (ntiles > 3) issue_tile(3, std::integral_constant<int, 3 % NB>{});
        }
        wait_tiles(ntiles - 1 < NB - 1 ? ntiles - 1 : NB - 1);
        __syncthreads();  // tile 0 landed
        if constexpr (L2) load_ninit(nrm, 0);
#pragma unroll
        for (int ih = 0; ih < 2; ++ih)
#pragma unroll
          for (int s = 0; s < PD; ++s) af[ih][s] = afrag(lds, 16 * ih + q16, s);
      }
      for (int it = 0; it < ntiles; it += NB) {
        tile_d(it, std::integral_constant<int, 0>{});
        if (it + 1 < ntiles) tile_d(it + 1, std::integral_constant<int, 1>{});
        if constexpr (NB >= 3) {
          if (it + 2 < ntiles) tile_d(it + 2, std::integral_constant<int, 2 % NB>{});
        }
        if constexpr (NB >= 4) {
          if (it + 3 < ntiles) tile_d(it + 3, std::integral_constant<int, 3 % NB>{});
        }
      }
      if (baseB >= 0) {  // the last sub-tile's epilogue
        if (nvB < 32) mask_rows(accB, nvB);
        float m2[NQ2][2], m[NQ2];
        tree(accB, m2, m);
        drain(accB, baseB, m2, m);
      }
    };
    if (nact == NQ2) run(std::integral_constant<int, NQ2>{});
    else if (nact == 0) run(std::integral_constant<int, 0>{});
    else if constexpr (NQ2 == 4) {
      if (nact == 3) run(std::integral_constant<int, 3>{});
      else if (nact == 2) run(std::integral_constant<int, 2>{});
      else run(std::integral_constant<int, 1>{});
    } else {
      run(std::integral_constant<int, 1>{});
    }

    // flush the staged candidates: one global atomic per query row
    __syncthreads();
    for (int row = tid; row < WQ; row += NT) {
      const int n_r = cl.qcnt[row];
      const int qy = cl.qid[row];
      cl.base[row] = n_r > 0 && guard_ok((uint64_t)qy < (uint64_t)nq, iv.err, GUARD_COLLECT_QUERY)
                         ? atomicAdd(&iv.cand_cnt[qy], n_r) : iv.cap;
    }
    __syncthreads();
    const int ne = cl.n < CL::CAP ? cl.n : CL::CAP;
    for (int e = tid; e < ne; e += NT) {
      const int2 en = cl.ent[e];
      const int row = en.x & 1023, dst = cl.base[row] + (en.x >> 10);
      if (dst < iv.cap && guard_ok((uint64_t)en.y < (uint64_t)nb, iv.err, GUARD_COLLECT_POS))
        iv.cand_pos[(int64_t)cl.qid[row] * iv.cap + dst] = en.y;
    }
    if (tid == 0) next_item = nxt;  // (every thread read this item's index before its first barrier)
  }
}

// IVF collect on the 16x16x32 form for (DP, l2), or nullptr (screen.h's MODE 3)
screen_fn pick_collect16_dp128(bool l2);

// the 16x16x32 main pass for (DP, qt, M), or nullptr (no such form: use screen.h's)
screen_fn pick_screen16_dp128(int qt, int M);
screen_fn pick_screen16_dp256_w8(int M);

}  // namespace nrk
