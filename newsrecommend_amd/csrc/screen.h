// screen.h — the bf16 MFMA screening kernel (K-GEMM-TOPK / K-IVF-SCAN) and
// its per-padded-dimension dispatch.  The template is instantiated in one
// translation unit per padded dimension (screen_dp{32,64,128,256}.hip) so the
// build compiles the ~200 instantiations in parallel; knn_flat.hip only calls
// pick_screen().
#pragma once

#include <math.h>

#include <type_traits>

#include "nrk_common.h"

namespace nrk {

// ================================================================ screen ==
// LDS swizzle so that the ds_read_b128 A-fragment reads (32 rows, one 16-B
// chunk each, 16-lane groups) hit 16 distinct bank slots.
template <int CPR>
__device__ __forceinline__ int swz(int row) {
  if constexpr (CPR >= 16) return row & 15;
  else return (row / (16 / CPR)) & (CPR - 1);
}

__device__ __forceinline__ float fmax_ieee(float a, float b) { return __builtin_elementwise_maximum(a, b); }

// Buffer-descriptor LDS-DMA.  The AMDGPU buffer-resource builtins exist only in
// the device compilation pass; the host pass (which only needs the kernel
// stubs) silently drops every kernel whose body names them.
struct BufRsrc {
#if defined(__HIP_DEVICE_COMPILE__)
  __amdgpu_buffer_rsrc_t r;
#endif
};
__device__ __forceinline__ BufRsrc make_rsrc(const void* base, int bytes) {
  BufRsrc b;
#if defined(__HIP_DEVICE_COMPILE__)
  b.r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
#else
  (void)base;
  (void)bytes;
#endif
  return b;
}
#if defined(__HIP_DEVICE_COMPILE__)
#define NRK_BUFFER_LOAD_LDS(SIZE)                                                                         \
  __device__ __forceinline__ void buffer_load_lds##SIZE(const BufRsrc& b, void* lds_dst, int vo, int so) { \
    __builtin_amdgcn_raw_ptr_buffer_load_lds(b.r, (__attribute__((address_space(3))) void*)lds_dst, SIZE, vo, \
                                             so, 0, 0);                                                  \
  }
#else
#define NRK_BUFFER_LOAD_LDS(SIZE) \
  __device__ __forceinline__ void buffer_load_lds##SIZE(const BufRsrc&, void*, int, int) {}
#endif
NRK_BUFFER_LOAD_LDS(16)
NRK_BUFFER_LOAD_LDS(4)
#undef NRK_BUFFER_LOAD_LDS

// The same LDS DMA issued from inline assembly.  The compiler tracks a
// builtin's LDS write; where it cannot tell an LDS read apart from it (the
// screen16 collect kernel's dynamically indexed norm ring) it puts an s_waitcnt
// vmcnt(0) before that read, i.e. right after a tile prefetch it waits for the
// prefetch to land.  Issued here, the write is invisible to it: the kernel
// orders the tile's reads itself (an explicit vmcnt wait for that tile's loads,
// then the workgroup barrier).  The compiler's own vmcnt waits stay correct
// (they only count the loads it knows of, so they are stricter than needed).
// The flat screen kernels keep the builtin: no such waits there, and the asm
// form measured slower (0.92 -> 1.32 ms at configs[1], profiles/r04_dma_asm_flat_ab.log).
typedef int __attribute__((ext_vector_type(4))) i32x4;
__device__ __forceinline__ i32x4 dma_rsrc(const void* base, int bytes) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xffffu));  // stride 0
  r.z = __builtin_amdgcn_readfirstlane(bytes);                                 // num_records
  r.w = 0x00020000;
  return r;
}
template <int SIZE>
__device__ __forceinline__ void dma_lds(const i32x4& r, const void* lds_dst, int vo, int so) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int la = __builtin_amdgcn_readfirstlane(
      (int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)lds_dst);
  const int sof = __builtin_amdgcn_readfirstlane(so);
  // s_nop 4: the VMEM instruction may read SGPRs a VALU (readfirstlane) just wrote
  if constexpr (SIZE == 16)
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 4\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :: "s"(la), "v"(vo), "s"(r), "s"(sof) : "memory", "m0");
  else
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 4\n\tbuffer_load_dword %1, %2, %3 offen lds"
                 :: "s"(la), "v"(vo), "s"(r), "s"(sof) : "memory", "m0");
#else
  (void)r;
  (void)lds_dst;
  (void)vo;
  (void)so;
#endif
}

// Sorted (descending) insertion into a register list of N entries.  Ties keep
// the resident entry first (it has the lower id: a lane scans ids upward).
template <int N>
__device__ __forceinline__ void list_insert(float (&ls)[N], int (&li)[N], float v, int id) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
    bool gt = v > ls[j];
    float ts = gt ? v : ls[j];
    int ti = gt ? id : li[j];
    v = gt ? ls[j] : v;
    id = gt ? li[j] : id;
    ls[j] = ts;
    li[j] = ti;
  }
}

// One workgroup = WAVES waves; wave w owns QT tiles of 32 queries; the
// workgroup streams one corpus chunk in 64-item tiles, staged HBM -> LDS with
// global_load_lds (double buffered; the XOR swizzle is applied to the SOURCE
// address since the DMA writes LDS lane-linearly).  MFMA 32x32x16 bf16 with
// A = items (rows), B = queries (cols): each lane holds ONE query (lane & 31)
// and 16 items of each 32-item sub-tile.
//
// MODE 1 (threshold pre-pass): visits every TSTRIDE-th tile of its chunk and
//   writes each lane's maximum screened score: many short, disjoint lane
//   streams, so the R-th largest of a query's lane maxima (tau_select_kernel)
//   is a proven lower bound on that query's global R-th best screened score.
// MODE 0 (main pass): every lane keeps its top-(M+1) screened scores in
//   registers, admitting only scores above max(its (M+1)-th, tau[q]); the
//   pre-pass bound removes the warm-up insertions that otherwise dominate.
//   The merge's certificate includes tau[q] in theta.
//
// MODE 2 (IVF list scan): the block's work item comes from a device table —
//   (list l, tile of the queries probing l, chunk of l).  qh holds the probing
//   queries gathered list-major (segments padded to WQ rows); slot_pair maps a
//   gathered row back to its (query, probe) pair, whose candidates land at
//   [(pair * cmax + chunk) * 2 + half].
// MODE 3 (IVF collect): MODE 2's work items, no lane lists: every item whose
//   screened score reaches the query's threshold is appended to the query's
//   candidate buffer (rare: the threshold sits just below the k-th best).
// MODE 4 (IVF lane maxima): MODE 2's work items, MODE 1's epilogue (each lane
//   writes the maximum screened score of its stream).
struct IvfScreen {
  const int* work_off;     // [nlist + 1] prefix of work items per list
  const int64_t* list_off; // [nlist + 1] list ranges in the list-major corpus
  const int* seg_off;      // [nlist] first gathered query row of each list
  const int* slot_pair;    // [slots] q * nprobe + p, or -1 for padding
  int nlist, ch, cmax;
  // MODE 3 (collect): append every item whose screened score >= thr_q[query]
  const float* thr_q;
  int* cand_cnt;           // [nq]
  int* cand_pos;           // [nq][cap] list-major positions
  int cap, nprobe;
  // screen16 collect: per-XCD work tickets (8 ints, zero at launch)
  int* ticket;
  // MODE 3: the search's guard word (GuardCode bits; nullptr: unchecked)
  int* err;
};

// MODE 3 block-local candidate staging: hits are appended with LDS atomics and
// flushed at the end of the work item with ONE global atomic per query row
// (returning global atomics in the epilogue would stall the wave for ~1 us).
template <int WQ>
struct CollectLds {
  static constexpr int CAP = 4 * WQ > 1024 ? 4 * WQ : 1024;  // the QT = 1 forms keep 1024 entries
  int n;
  int qcnt[WQ];
  int qid[WQ];
  int base[WQ];
  int2 ent[CAP];  // {row | rank << 10, position}
};
struct NoLds {};

// DEFER (flat modes 0 and 1): the epilogue of sub-tile s runs while the MFMA
// chain of sub-tile s+1 is in flight.  Two accumulator sets alternate (A: even
// sub-tiles, B: odd ones, whose epilogue falls into the next tile); the
// straight-line part of the epilogue (L2 correction, max tree, threshold
// test) is scheduled between the MFMAs, only the rare list insertions follow
// the chain.  Without it every chain's results are waited for and reduced
// before the next chain issues (an MFMA-only ablation was 30 % faster).
// TIL: items per tile (deferred IP main pass may use 128: half the barriers).
template <int DP, int QT, int M, int WAVES, bool L2, int MODE, bool AFRAG_GROUP = true, bool DEFER = false,
          int TIL = 64>
__global__ __launch_bounds__(WAVES * 64, (MODE == 3 && WAVES == 8) ? 1 : 2) void screen_kernel(
    const uint16_t* __restrict__ qh, const uint16_t* __restrict__ xbh, const float* __restrict__ xmeta,
    int64_t nq, int64_t nb, int64_t chunk, int nch, int nqt, int tstride, float* __restrict__ part_s,
    int* __restrict__ part_i, float* __restrict__ part_t, const float* __restrict__ tau_q, IvfScreen iv) {
  constexpr int CPR = DP / 8;        // 16-B chunks per row
  constexpr int TI = TIL;  // items per tile (TI/32 sub-tiles of 32) between barriers
  static_assert(TIL == 64 || (TIL == 128 && DEFER && !L2 && MODE == 0), "128-item tiles: deferred IP main pass");
  constexpr int TCH = TI * CPR;      // 16-B chunks per tile
  constexpr int NT = WAVES * 64;
  constexpr int GPT = TCH / NT;      // glds instructions per thread per tile
  static_assert(TCH % NT == 0, "tile must split evenly over the workgroup");
  static_assert(WAVES * 32 * QT <= 1024, "collect rows: 10 bits");
  constexpr int KS = DP / 16;
  constexpr int WQ = WAVES * 32 * QT;
  constexpr int BUF = TI * DP + 2 * TI;  // uint16 per buffer: rows + TI float norms
  static_assert(!DEFER || MODE <= 1 || MODE == 3 || MODE == 4, "deferred epilogue: flat modes, IVF collect / lane maxima");
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * BUF];
  __shared__ std::conditional_t<MODE == 3, CollectLds<WQ>, NoLds> cl;

  const int nblk = gridDim.x, b = blockIdx.x;
  const int xg = b & 7, jj = b >> 3, q8 = nblk >> 3, r8 = nblk & 7;
  const int logical0 = (xg < r8 ? xg * (q8 + 1) : r8 * (q8 + 1) + (xg - r8) * q8) + jj;
  // IVF modes loop persistently over the device work table; flat modes run
  // exactly one item per block
  const int total = MODE >= 2 ? iv.work_off[iv.nlist] : nblk;
  for (int logical = logical0; logical < total; logical += nblk) {
    if (logical != logical0) __syncthreads();  // the previous item is done with the LDS buffers
    int c, qt;
    int64_t ibeg, iend, seg0 = 0;
    if constexpr (MODE >= 2) {
      int lo = 0, hi = iv.nlist;  // largest l with work_off[l] <= logical (empty lists own no items)
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (iv.work_off[mid] <= logical) lo = mid;
        else hi = mid;
      }
      const int64_t lb = iv.list_off[lo], le = iv.list_off[lo + 1];
      const int nchl = (int)cdiv(le - lb, (int64_t)iv.ch);
      // query tile innermost: the tiles sharing a chunk are consecutive work
      // items, i.e. run together on one XCD and read the chunk through its L2
      const int local = logical - iv.work_off[lo];
      const int nqtl = (iv.work_off[lo + 1] - iv.work_off[lo]) / nchl;
      c = local / nqtl;
      qt = local - c * nqtl;
      ibeg = lb + (int64_t)c * iv.ch;
      iend = ibeg + iv.ch < le ? ibeg + iv.ch : le;
      seg0 = iv.seg_off[lo];
    } else {
      c = logical / nqt;
      qt = logical - c * nqt;
      ibeg = (int64_t)c * chunk;
      iend = ibeg + chunk < nb ? ibeg + chunk : nb;
    }

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int ntiles = (int)cdiv(cdiv(iend - ibeg, TI), tstride);  // visited tiles

    bf16x8 qf[QT][KS];
    int64_t qidx[QT];
  #pragma unroll
    for (int t = 0; t < QT; ++t) {
      qidx[t] = (int64_t)qt * WQ + (w * QT + t) * 32 + r;  // < nq_pad (zero rows)
      const bf16x8* src = reinterpret_cast<const bf16x8*>(qh + (seg0 + qidx[t]) * DP + 8 * h);
  #pragma unroll
      for (int s = 0; s < KS; ++s) qf[t][s] = src[2 * s];
    }
    // query tiles of this wave holding a real row (IVF: padding rows are a suffix of the segment)
    int nact = QT;
    if constexpr (MODE >= 2) {
      nact = 0;
  #pragma unroll
      for (int t = 0; t < QT; ++t)
        if (__any(iv.slot_pair[seg0 + qidx[t]] >= 0)) nact = t + 1;
      nact = __builtin_amdgcn_readfirstlane(nact);
    }
    float ls[QT][M + 1];
    int li[QT][M + 1];
    float tau[QT];
    float cthr[QT];  // MODE 3: collect threshold of the lane's query
    int cq[QT];      // MODE 3: the lane's query (-1: padding row)
  #pragma unroll
    for (int t = 0; t < QT; ++t) {
      tau[t] = (MODE == 0 && tau_q && qidx[t] < nq) ? tau_q[qidx[t]] : -INFINITY;
      if constexpr (MODE == 3) {
        const int pair = iv.slot_pair[seg0 + qidx[t]];
        cq[t] = pair >= 0 ? pair / iv.nprobe : -1;
        cthr[t] = pair >= 0 ? iv.thr_q[cq[t]] : INFINITY;
        const int row = (w * QT + t) * 32 + r;
        if (h == 0) {
          cl.qid[row] = cq[t];
          cl.qcnt[row] = 0;
        }
      }
  #pragma unroll
      for (int j = 0; j <= M; ++j) {
        ls[t][j] = -INFINITY;
        li[t][j] = -1;
      }
    }

    // HBM -> LDS through chunk-relative buffer descriptors: rows past the chunk
    // fall outside num_records and read as 0 (masked in the epilogue); each
    // lane's inverse-swizzled 32-bit offset is fixed, only the scalar tile
    // offset changes, so staging costs no per-tile vector address math.
    typedef __attribute__((address_space(3))) void* lds_ptr;
    const int64_t cnt = iend - ibeg > 0 ? iend - ibeg : 0;
    const BufRsrc xrs = make_rsrc(xbh + ibeg * DP, (int)(cnt * DP * 2));
    const BufRsrc nrs = make_rsrc(xmeta + 2 * ibeg, (int)(cnt * 8));
    int voff[GPT];
  #pragma unroll
    for (int u = 0; u < GPT; ++u) {
      const int p = u * NT + tid;
      const int row = p / CPR, pc = p % CPR;
      voff[u] = row * DP * 2 + 16 * (pc ^ swz<CPR>(row));
    }
    auto issue_tile = [&](int it, auto buf_c) {
      constexpr int buf = decltype(buf_c)::value;
      const int soff = it * tstride * TI * DP * 2;
  #pragma unroll
      for (int u = 0; u < GPT; ++u)
        buffer_load_lds16(xrs, lds + buf * BUF + (u * NT + w * 64) * 8, voff[u], soff);
      if constexpr (L2) {
        if (w == 0)
          buffer_load_lds4(nrs, lds + buf * BUF + TI * DP, lane * 8, it * tstride * TI * 8);
      }
    };

    // one 64-item tile (buffer index is a compile-time constant: immediate LDS offsets).
    // NACT: query tiles of this wave that hold any real row (IVF modes: a list's
    // gathered segment is padded to the workgroup's rows, padding is a suffix, so a
    // wave past the list's last prober skips its MFMAs and leaves the SIMD's MFMA
    // pipe to the co-resident workgroup's wave)
    auto compute = [&](int it, auto buf_c, auto nact_c) {
      constexpr int buf = decltype(buf_c)::value;
      constexpr int NACT = decltype(nact_c)::value;
      const uint16_t* tl = lds + buf * BUF;
      const float* lnorm = reinterpret_cast<const float*>(tl + TI * DP);
      const int64_t i0 = ibeg + (int64_t)it * tstride * TI;
      const int nvalid = (int)((iend - i0) < TI ? (iend - i0) : TI);
  #pragma unroll
      for (int st = 0; st < TI / 32; ++st) {
        f32x16 acc[QT];
  #pragma unroll
        for (int t = 0; t < QT; ++t)
  #pragma unroll
          for (int g = 0; g < 16; ++g) acc[t][g] = 0.f;
        const int row = 32 * st + r;
        const uint16_t* arow = tl + row * DP;
        const int sw = swz<CPR>(row);
        // all KS A-fragments of the sub-tile are read first (one LDS round
        // trip instead of KS dependent ones), then the MFMA chain
        bf16x8 af[KS];
  #pragma unroll
        for (int s = 0; s < KS; ++s) af[s] = *reinterpret_cast<const bf16x8*>(arow + 8 * ((2 * s + h) ^ sw));
  #pragma unroll
        for (int s = 0; s < KS; ++s) {
  #pragma unroll
          for (int t = 0; t < NACT; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], qf[t][s], acc[t], 0, 0, 0);
        }
        if constexpr (AFRAG_GROUP && NACT > 0) {  // scheduler: the KS LDS reads first, then the MFMA chain
          __builtin_amdgcn_sched_group_barrier(0x100, KS, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, KS * NACT, 0);
        }
        // Epilogue.  MASKED only for the (rare) partial last tile of a chunk: a
        // wave-uniform branch, so full tiles carry no per-score selects.
        auto epilogue = [&](auto masked_tag) {
          constexpr bool MASKED = decltype(masked_tag)::value;
  #pragma unroll
          for (int t = 0; t < NACT; ++t) {
            float sc[16];
  #pragma unroll
            for (int g = 0; g < 16; ++g) {
              const int ir = 32 * st + (g & 3) + 8 * (g >> 2) + 4 * h;
              float v = acc[t][g];
              if constexpr (L2) v = fmaf(2.f, v, -lnorm[ir]);
              if constexpr (MASKED) v = ir < nvalid ? v : -INFINITY;
              sc[g] = v;
            }
            // IEEE maximum (v_maximum3_f32): no canonicalising moves on MFMA outputs
            float m4[4];
  #pragma unroll
            for (int j = 0; j < 4; ++j)
              m4[j] = fmax_ieee(fmax_ieee(sc[4 * j], sc[4 * j + 1]), fmax_ieee(sc[4 * j + 2], sc[4 * j + 3]));
            const float m = fmax_ieee(fmax_ieee(m4[0], m4[1]), fmax_ieee(m4[2], m4[3]));
            if constexpr (MODE == 3) {  // collect: append every score at or above the threshold
              if (__any(m >= cthr[t])) {
  #pragma unroll
                for (int g = 0; g < 16; ++g) {
                  if (sc[g] >= cthr[t]) {
                    const int ir = 32 * st + (g & 3) + 8 * (g >> 2) + 4 * h;
                    const int e = atomicAdd(&cl.n, 1);
                    if (e < CollectLds<WQ>::CAP) {
                      const int row = (w * QT + t) * 32 + r;
                      const int rank = atomicAdd(&cl.qcnt[row], 1);
                      cl.ent[e] = make_int2(row | (rank << 10), (int)(i0 + ir));
                    } else if (guard_ok((uint64_t)cq[t] < (uint64_t)nq, iv.err, GUARD_COLLECT_QUERY) &&
                               __builtin_nontemporal_load(&iv.cand_cnt[cq[t]]) <= iv.cap) {
                      // staging full: append directly (stop once the query overflowed)
                      const int pos = atomicAdd(&iv.cand_cnt[cq[t]], 1);
                      if (pos < iv.cap) iv.cand_pos[(int64_t)cq[t] * iv.cap + pos] = (int)(i0 + ir);
                    }
                  }
                }
              }
              continue;
            }
            if constexpr (MODE == 4) {  // lane maximum and its position (new maxima are rare)
              if (__any(m > ls[t][0])) {
  #pragma unroll
                for (int g = 0; g < 16; ++g) {
                  if (sc[g] > ls[t][0]) {
                    ls[t][0] = sc[g];
                    li[t][0] = (int)(i0 + 32 * st + (g & 3) + 8 * (g >> 2) + 4 * h);
                  }
                }
              }
              continue;
            }
            if constexpr (MODE == 1) {  // pre-pass: lane maximum only
              ls[t][0] = fmax_ieee(ls[t][0], m);
              continue;
            }
            // rare path: descend only into 4-row groups that beat the threshold
            if (__any(m > fmaxf(ls[t][M], tau[t]))) {
  #pragma unroll
              for (int j = 0; j < 4; ++j) {
                if (__any(m4[j] > fmaxf(ls[t][M], tau[t]))) {
  #pragma unroll
                  for (int i = 0; i < 4; ++i) {
                    const int g = 4 * j + i;
                    const int ir = 32 * st + i + 8 * j + 4 * h;
                    const float thr = fmaxf(ls[t][M], tau[t]);
                    if (sc[g] > thr) list_insert<M + 1>(ls[t], li[t], sc[g], (int)(i0 + ir));
                  }
                }
              }
            }
          }
        };
        if (nvalid >= 32 * (st + 1)) epilogue(std::false_type{});
        else epilogue(std::true_type{});
      }
    };
    // two buffers: tile it+1 in flight while tile it is computed
    auto tile = [&](int it, auto buf_c) {
      constexpr int buf = decltype(buf_c)::value;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // tile `it` landed; everyone is done with the other buffer
      if (it + 1 < ntiles) issue_tile(it + 1, std::integral_constant<int, buf ^ 1>{});
      if (nact == QT) compute(it, buf_c, std::integral_constant<int, QT>{});
      else if constexpr (QT > 1) {
        if (nact == 1) compute(it, buf_c, std::integral_constant<int, 1>{});
      }
    };
    // ---- deferred epilogue (DEFER): see the comment at the template ----
    constexpr int NSUB = TI / 32;  // sub-tiles per tile (2 or 4)
    f32x16 accA[QT], accB[QT];
    int64_t baseA = -1, baseB = -1;  // item index of the pending sub-tile's row 0 (-1: nothing pending)
    int nvA = 0, nvB = 0;            // its rows inside the chunk
    float pnB[16];                   // L2: norms of sub-tile B's rows (its buffer is refilled before its epilogue)
    // rows of a pending sub-tile past the chunk (only in a chunk's last tile)
    auto mask_rows = [&](f32x16 (&pa)[QT], int nv) __attribute__((always_inline)) {
  #pragma unroll
      for (int t = 0; t < QT; ++t)
  #pragma unroll
        for (int g = 0; g < 16; ++g)
          if ((g & 3) + 8 * (g >> 2) + 4 * h >= nv) pa[t][g] = -INFINITY;
    };
    // straight-line part: L2 scores 2 ip - |x|^2 (in place), 4-row maxima, lane maximum
    auto tree = [&](f32x16 (&pa)[QT], const float (&n16)[16], float (&m4)[QT][4], float (&m)[QT]) __attribute__((always_inline)) {
  #pragma unroll
      for (int t = 0; t < QT; ++t) {
        if constexpr (L2) {
  #pragma unroll
          for (int g = 0; g < 16; ++g) pa[t][g] = fmaf(2.f, pa[t][g], -n16[g]);
        }
  #pragma unroll
        for (int j = 0; j < 4; ++j)
          m4[t][j] = fmax_ieee(fmax_ieee(pa[t][4 * j], pa[t][4 * j + 1]), fmax_ieee(pa[t][4 * j + 2], pa[t][4 * j + 3]));
        m[t] = fmax_ieee(fmax_ieee(m4[t][0], m4[t][1]), fmax_ieee(m4[t][2], m4[t][3]));
      }
    };
    // rare part: lane-list insertions (MODE 0) or the lane maximum (MODE 1)
    auto drain = [&](f32x16 (&pa)[QT], int64_t pbase, const float (&m4)[QT][4], const float (&m)[QT]) __attribute__((always_inline)) {
      if constexpr (MODE == 3) {  // IVF collect: append every score at or above the query's threshold
  #pragma unroll
        for (int t = 0; t < QT; ++t) {
          if (__any(m[t] >= cthr[t])) {
  #pragma unroll
            for (int g = 0; g < 16; ++g) {
              if (pa[t][g] >= cthr[t]) {
                const int pos = (int)(pbase + (g & 3) + 8 * (g >> 2) + 4 * h);
                const int e = atomicAdd(&cl.n, 1);
                if (e < CollectLds<WQ>::CAP) {
                  const int row = (w * QT + t) * 32 + r;
                  const int rank = atomicAdd(&cl.qcnt[row], 1);
                  cl.ent[e] = make_int2(row | (rank << 10), pos);
                } else if (guard_ok((uint64_t)cq[t] < (uint64_t)nq, iv.err, GUARD_COLLECT_QUERY) &&
                           __builtin_nontemporal_load(&iv.cand_cnt[cq[t]]) <= iv.cap) {
                  const int slot = atomicAdd(&iv.cand_cnt[cq[t]], 1);
                  if (slot < iv.cap) iv.cand_pos[(int64_t)cq[t] * iv.cap + slot] = pos;
                }
              }
            }
          }
        }
        return;
      }
      if constexpr (MODE == 4) {  // IVF lane maximum and its position
  #pragma unroll
        for (int t = 0; t < QT; ++t) {
          if (__any(m[t] > ls[t][0])) {
  #pragma unroll
            for (int g = 0; g < 16; ++g) {
              if (pa[t][g] > ls[t][0]) {
                ls[t][0] = pa[t][g];
                li[t][0] = (int)(pbase + (g & 3) + 8 * (g >> 2) + 4 * h);
              }
            }
          }
        }
        return;
      }
      if constexpr (MODE == 1) {
  #pragma unroll
        for (int t = 0; t < QT; ++t) ls[t][0] = fmax_ieee(ls[t][0], m[t]);
        return;
      }
      // one test for all query tiles (keeps every tile's max tree ahead of the branch)
      bool hit = false;
  #pragma unroll
      for (int t = 0; t < QT; ++t) hit |= m[t] > fmaxf(ls[t][M], tau[t]);
      if (!__any(hit)) return;
  #pragma unroll
      for (int t = 0; t < QT; ++t) {
        if (__any(m[t] > fmaxf(ls[t][M], tau[t]))) {
  #pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (__any(m4[t][j] > fmaxf(ls[t][M], tau[t]))) {
  #pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int g = 4 * j + i;
                const float thr = fmaxf(ls[t][M], tau[t]);
                if (pa[t][g] > thr) list_insert<M + 1>(ls[t], li[t], pa[t][g], (int)(pbase + i + 8 * j + 4 * h));
              }
            }
          }
        }
      }
    };
    // one sub-tile: its MFMA chain with, scheduled between the MFMAs, the
    // pending sub-tile's straight-line epilogue and the LDS reads of the NEXT
    // sub-tile's A fragments (af[s] is refilled right after its last MFMA, so
    // the chain never waits on LDS); then the pending one's rare part
    bf16x8 af[KS];  // A fragments of the sub-tile computed next
    float pnA[16];  // L2: norms of sub-tile A's rows
    auto sub_tile = [&](auto st_c, int64_t i0, int nvalid, const uint16_t* next_tl) __attribute__((always_inline)) {
      constexpr int st = decltype(st_c)::value;
      constexpr int par = st & 1;  // even sub-tiles accumulate into A, odd ones into B
      f32x16(&cur)[QT] = par ? accB : accA;
      f32x16(&pend)[QT] = par ? accA : accB;
      const int64_t pbase = par ? baseA : baseB;
      const int pnv = par ? nvA : nvB;
      if (pbase >= 0 && pnv < 32) mask_rows(pend, pnv);
      float n16[16];
      if constexpr (L2) {
  #pragma unroll
        for (int g = 0; g < 16; ++g) n16[g] = par ? pnA[g] : pnB[g];
      }
      // next sub-tile: the next 32 rows of this tile, or rows 0..31 of the next tile
      // (last sub-tile); past the last tile the reads hit the idle buffer, unused
      const int nrow = (st + 1 < NSUB ? 32 * (st + 1) : 0) + r;
      const uint16_t* narow = next_tl + nrow * DP;
      const int nsw = swz<CPR>(nrow);
      const f32x16 zero = {};
  #pragma unroll
      for (int s = 0; s < KS; ++s) {
  #pragma unroll
        for (int t = 0; t < QT; ++t)
          cur[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], qf[t][s], s == 0 ? zero : cur[t], 0, 0, 0);
        af[s] = *reinterpret_cast<const bf16x8*>(narow + 8 * ((2 * s + h) ^ nsw));
      }
      float m4[QT][4], m[QT];
      tree(pend, n16, m4, m);
  #pragma unroll
      for (int t = 0; t < QT; ++t) m[t] = pbase >= 0 ? m[t] : -INFINITY;  // nothing pending: drain is a no-op
      constexpr int VPM = L2 ? 4 : 2;
  #pragma unroll
      for (int s = 0; s < KS; ++s) {
        __builtin_amdgcn_sched_group_barrier(0x008, QT, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, VPM * QT, 0);
      }
      drain(pend, pbase, m4, m);
      if constexpr (par == 0) {
        baseA = i0 + 32 * st;
        nvA = nvalid - 32 * st;
      } else {
        baseB = i0 + 32 * st;
        nvB = nvalid - 32 * st;
      }
    };
    // tile it (buffer buf): sub-tile 0; then the tile barrier (tile it+1 landed,
    // every wave is done with buffer buf: its fragments and norms are all in
    // registers) and the DMA of tile it+2 into buf; then sub-tile 1, which
    // reads tile it+1's first fragments
    auto tile_d = [&](int it, auto buf_c) __attribute__((always_inline)) {
      constexpr int buf = decltype(buf_c)::value;
      const uint16_t* tl = lds + buf * BUF;
      const int64_t i0 = ibeg + (int64_t)it * tstride * TI;
      const int nvalid = (int)((iend - i0) < TI ? (iend - i0) : TI);
      sub_tile(std::integral_constant<int, 0>{}, i0, nvalid, tl);
      if constexpr (NSUB == 4) {
        sub_tile(std::integral_constant<int, 1>{}, i0, nvalid, tl);
        sub_tile(std::integral_constant<int, 2>{}, i0, nvalid, tl);
      }
      if constexpr (L2) {  // (NSUB == 2)
        const float* lnorm = reinterpret_cast<const float*>(tl + TI * DP);
  #pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 va = *reinterpret_cast<const float4*>(lnorm + 8 * j + 4 * h);
          const float4 vb = *reinterpret_cast<const float4*>(lnorm + 32 + 8 * j + 4 * h);
          pnA[4 * j] = va.x; pnA[4 * j + 1] = va.y; pnA[4 * j + 2] = va.z; pnA[4 * j + 3] = va.w;
          pnB[4 * j] = vb.x; pnB[4 * j + 1] = vb.y; pnB[4 * j + 2] = vb.z; pnB[4 * j + 3] = vb.w;
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (it + 2 < ntiles) issue_tile(it + 2, buf_c);
      sub_tile(std::integral_constant<int, NSUB - 1>{}, i0, nvalid, lds + (buf ^ 1) * BUF);
    };
    if constexpr (MODE == 3) {
      if (tid == 0) cl.n = 0;  // ordered before any append by the first tile's barrier
    }
    if constexpr (DEFER) {
      if (ntiles > 0) {
        issue_tile(0, std::integral_constant<int, 0>{});
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // tile 0 landed
        if (ntiles > 1) issue_tile(1, std::integral_constant<int, 1>{});
        const uint16_t* arow = lds + r * DP;
        const int sw = swz<CPR>(r);
  #pragma unroll
        for (int s = 0; s < KS; ++s) af[s] = *reinterpret_cast<const bf16x8*>(arow + 8 * ((2 * s + h) ^ sw));
      }
      for (int it = 0; it < ntiles; it += 2) {
        tile_d(it, std::integral_constant<int, 0>{});
        if (it + 1 < ntiles) tile_d(it + 1, std::integral_constant<int, 1>{});
      }
      if (baseB >= 0) {  // the last sub-tile's epilogue
        if (nvB < 32) mask_rows(accB, nvB);
        float m4[QT][4], m[QT];
        tree(accB, pnB, m4, m);
        drain(accB, baseB, m4, m);
      }
    } else {
      if (ntiles > 0) issue_tile(0, std::integral_constant<int, 0>{});
      for (int it = 0; it < ntiles; it += 2) {
        tile(it, std::integral_constant<int, 0>{});
        if (it + 1 < ntiles) tile(it + 1, std::integral_constant<int, 1>{});
      }
    }

    if constexpr (MODE == 3) {  // flush the staged candidates
      __syncthreads();
      for (int row = tid; row < WQ; row += NT) {
        const int n_r = cl.qcnt[row];
        const int qy = cl.qid[row];
        cl.base[row] = n_r > 0 && guard_ok((uint64_t)qy < (uint64_t)nq, iv.err, GUARD_COLLECT_QUERY)
                           ? atomicAdd(&iv.cand_cnt[qy], n_r) : iv.cap;
      }
      __syncthreads();
      const int ne = cl.n < CollectLds<WQ>::CAP ? cl.n : CollectLds<WQ>::CAP;
      for (int e = tid; e < ne; e += NT) {
        const int2 en = cl.ent[e];
        const int row = en.x & 1023, dst = cl.base[row] + (en.x >> 10);
        if (dst < iv.cap && guard_ok((uint64_t)en.y < (uint64_t)nb, iv.err, GUARD_COLLECT_POS))
          iv.cand_pos[(int64_t)cl.qid[row] * iv.cap + dst] = en.y;
      }
      continue;
    }

  #pragma unroll
    for (int t = 0; t < QT; ++t) {
      const int64_t qi = qidx[t];
      int64_t base = -1;
      if constexpr (MODE == 3) {
        continue;  // collect mode writes its candidates as it goes
      } else if constexpr (MODE == 2 || MODE == 4) {
        const int pair = iv.slot_pair[seg0 + qi];
        if (pair >= 0) base = ((int64_t)pair * iv.cmax + c) * 2 + h;
      } else if (qi < nq) {
        base = (qi * nch + c) * 2 + h;
      }
      if (base >= 0) {
        if constexpr (MODE == 1 || MODE == 4) {
          part_t[base] = ls[t][0];
          if constexpr (MODE == 4) part_i[base] = li[t][0];
        } else {
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
}


typedef void (*screen_fn)(const uint16_t*, const uint16_t*, const float*, int64_t, int64_t, int64_t, int, int, int,
                          float*, int*, float*, const float*, IvfScreen);

// The one kernel variant per (DP, QT, M, L2, MODE).  Flat modes (main pass and
// pre-pass) defer each sub-tile's epilogue into the next MFMA chain, except
// where the second accumulator set and the fragment prefetch would spill (DP =
// 256, L2 with two query tiles, the DP = 128 two-tile pre-pass); the IP main
// pass streams 128-item tiles (half the barriers, measured +9 %).  The IVF
// modes read each sub-tile's A fragments as one group before the MFMA chain
// (measured faster there).  DESIGN.md "K-GEMM-TOPK" has the ablations.
template <int DP, int QT, int M, bool L2, int MODE>
constexpr screen_fn screen_variant() {
  constexpr bool defer = MODE <= 1 && DP < 256 && !(L2 && QT == 2) && !(DP == 128 && QT == 2 && MODE == 1);
  if constexpr (defer)
    return screen_kernel<DP, QT, M, 4, L2, MODE, false, true, (MODE == 0 && !L2) ? 128 : 64>;
  else
    return screen_kernel<DP, QT, M, 4, L2, MODE, (MODE >= 2)>;
}

// mode: 0 main pass, 1 threshold pre-pass, 2 IVF list scan, 3 IVF collect, 4 IVF lane maxima.
// DP = 256 always runs one query tile per wave.
template <int DP, bool L2>
screen_fn screen_for(int qt, int M, int mode) {
  constexpr int Q2 = DP == 256 ? 1 : 2;
  const bool two = qt == 2;
  switch (mode) {
    case 1: return two ? screen_variant<DP, Q2, 1, L2, 1>() : screen_variant<DP, 1, 1, L2, 1>();
    case 3: return two ? screen_variant<DP, Q2, 1, L2, 3>() : screen_variant<DP, 1, 1, L2, 3>();
    case 4: return two ? screen_variant<DP, Q2, 1, L2, 4>() : screen_variant<DP, 1, 1, L2, 4>();
    case 0:
    case 2: {
      if (mode == 0) {
        if (M == 4) return two ? screen_variant<DP, Q2, 4, L2, 0>() : screen_variant<DP, 1, 4, L2, 0>();
        if (M == 8) return screen_variant<DP, 1, 8, L2, 0>();
        return screen_variant<DP, 1, 16, L2, 0>();
      }
      if (M == 4) return two ? screen_variant<DP, Q2, 4, L2, 2>() : screen_variant<DP, 1, 4, L2, 2>();
      if (M == 8) return screen_variant<DP, 1, 8, L2, 2>();
      return screen_variant<DP, 1, 16, L2, 2>();
    }
  }
  return nullptr;
}

// one translation unit per padded dimension (screen_dp*.hip) instantiates these
screen_fn pick_screen_dp32(int qt, int M, bool l2, int mode);
screen_fn pick_screen_dp64(int qt, int M, bool l2, int mode);
screen_fn pick_screen_dp128(int qt, int M, bool l2, int mode);
screen_fn pick_screen_dp256(int qt, int M, bool l2, int mode);
// DP = 256, QT = 1, 8 waves (256 queries per workgroup and corpus pass):
// the flat main pass with M = 4 or 16 (mode 0) and its pre-pass (mode 1).
// (Lane lists kept in LDS instead of registers for M = 16 measured slower at
// k = 200: 18.8 -> 21.6 ms; each lane stream admits ~30 items above tau.)
screen_fn pick_screen_dp256_w8(int M, bool l2, int mode);

#define NRK_SCREEN_DP(DP)                                                  \
  screen_fn pick_screen_dp##DP(int qt, int M, bool l2, int mode) {         \
    return l2 ? screen_for<DP, true>(qt, M, mode) : screen_for<DP, false>(qt, M, mode); \
  }

inline screen_fn pick_screen(int dp, int qt, int M, bool l2, int mode) {
  switch (dp) {
    case 32: return pick_screen_dp32(qt, M, l2, mode);
    case 64: return pick_screen_dp64(qt, M, l2, mode);
    case 128: return pick_screen_dp128(qt, M, l2, mode);
    case 256: return pick_screen_dp256(qt, M, l2, mode);
  }
  return nullptr;
}

}  // namespace nrk
