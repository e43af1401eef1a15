// din_rerank_lane.hip — nrk_din_rerank_projected for F <= 64 (DIN.py:166-189
// evaluate() over the row projections; see din_rerank.hip for the algebra).
// Built with -fno-slp-vectorize (build.py): the SLP vectorizer turns the
// scoring's |y|-fmas into v_and + v_pk_fma pairs, more instructions than the
// fmas with an |.| source modifier.
#include <math.h>

#include "din_rerank.h"

namespace nrk {
namespace rr {

// ---- the projected re-rank, one wave per 32 candidates (nrk_din_rerank_projected
// for F <= 64).  The scoring is the VALU-bound part: per (candidate, history
// row, attention unit) one add and one |.|-fma, the add packed two units at a
// time.  Lane (pc, q) = (candidate pair pc of the wave's 32 candidates, unit
// quarter q): the pair's U' quarter stays in registers for all rows, each P'
// row is read by one LDS wave-instruction for all 32 candidates (four
// addresses, one per quarter, on different banks) and each value it brings
// serves two candidates (one LDS read per 12 VALU; one per 6 with a candidate
// per lane over unit halves cost 5 % more), the quarter's unit signs sgn(w2)
// are f16 pairs in A / 8 registers (v_fma_mix operands), and the quarters'
// partial sums meet by a reduce-scatter of the four (candidate, row) values of
// a row pair (three permlane swaps).  Every other step of a candidate (softmax,
// e R, the head) is wave-local too: a wave waits for another only when the
// block moves to the next user (one staging of the history projections
// [P' | R], three barriers per user, against five per 64-candidate chunk in
// din_rerank_kernel).
//   s[c][r] = (SU[c] + SP[r] + sum_n sgn_n |U'[c][n] + P'[r][n]|) / 2
//   e = exp(s - max_r s) (the padding row weighted L - nv), as bf16 hi + lo;
//   h1 = relu((Q1 den + e R^T) / den + c1) on MFMA (three products), h2 and
//   the logit on MFMA as in din_rerank_kernel.
namespace lk {
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
constexpr int CPI = 32;  // candidates per wave item
// LPK: history rows held.  64: 8 waves per block, two per SIMD (the partner
// wave's LDS reads issue beside this one's VALU); 128 (histories of 65..128
// slots, the reference's max_history range): 4 waves, the LDS holds twice the
// rows and four waves' score regions.
// RG (128 rows where [P' | R^T] and H2 do not fit the LDS together: (A, F) =
// (96, 64), (128, 64) and every F in {96, 128}): only P' is staged; the e R
// product reads R from the history projections in global memory (the user's
// rows, L2-resident after the staging read them), the softmax weights laid out
// by history SLOT instead of by compacted row (an invalid slot's R is zero), and
// the head's H2 comes from global memory too.
template <int A, int F, int LPK, bool RG = false>
struct Lay {  // byte offsets
  static constexpr int LP = LPK, NW = LPK == 64 ? 8 : 4, NT = 64 * NW;
  static constexpr int F2 = F / 2;
  static constexpr int QST = A / 4 + 4;  // P' unit quarter q at q QST floats: the four quarters on other banks
  static constexpr int PST = 4 * QST;     // P' row stride (floats)
  static constexpr int SST = LP + 2;      // scores [CPI][SST] f32: lanes (cs, h) write 2 cs + h apart, no conflicts
  static constexpr int EST = LP + 8;      // e planes [CPI][EST] bf16: conflict-free 16-B fragment reads
  static constexpr int c1 = 0;                          // [F]
  static constexpr int c2 = c1 + F * 4;                 // [F2]
  static constexpr int h3 = c2 + F2 * 4;                // [F2]
  static constexpr int h2 = h3 + F2 * 4;                // H2 hi, lo bf16 [F2][F] (RG: none)
  static constexpr int pp = h2 + (RG ? 0 : 2 * F2 * F * 2);  // P' [LP][PST] f32
  static constexpr int hsp = pp + LP * PST * 4;         // SP / 2 [LP]
  static constexpr int rt = hsp + LP * 4;               // R^T hi, lo bf16 [F][LP] (RG: none)
  static constexpr int wv = rt + (RG ? 0 : 2 * F * LP * 2);  // per wave: scores, then e hi / lo, then h1
  static constexpr int SB = CPI * SST * 4, EB = 2 * CPI * EST * 2, HB = CPI * (F + 4) * 4;
  static constexpr int XB = SB > EB ? SB : EB;
  static constexpr int WB = ((XB > HB ? XB : HB) + 2 * CPI * 4 + 15) & ~15;  // + den, valid [CPI]
  static constexpr int qs = wv + NW * WB;
  static constexpr int total = qs + 16;
};

template <int A, int F, int LPK, bool RG>
__global__ __launch_bounds__((LPK == 64 ? 512 : 256), 1) void din_rerank_lane_kernel(RerankArgs a) {
  using LY = Lay<A, F, LPK, RG>;
  constexpr int F2 = F / 2, AQ = A / 4, NG = AQ / 8, AF = A + F, PST = LY::PST, QST = LY::QST, SST = LY::SST, EST = LY::EST;
  constexpr int LP = LPK, NT = LY::NT, NW = LY::NW;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* c1s = reinterpret_cast<float*>(smem + LY::c1);
  float* c2s = reinterpret_cast<float*>(smem + LY::c2);
  float* h3s = reinterpret_cast<float*>(smem + LY::h3);
  uint16_t* H2s = reinterpret_cast<uint16_t*>(smem + LY::h2);
  float* Pp = reinterpret_cast<float*>(smem + LY::pp);
  float* hSP = reinterpret_cast<float*>(smem + LY::hsp);
  uint16_t* Rth = reinterpret_cast<uint16_t*>(smem + LY::rt);
  uint16_t* Rtl = Rth + F * LP;
  int* qslot = reinterpret_cast<int*>(smem + LY::qs);
  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned char* wreg = smem + LY::wv + w * LY::WB;
  float* Sw = reinterpret_cast<float*>(wreg);              // scores [CPI][SST]
  uint16_t* Eh = reinterpret_cast<uint16_t*>(wreg);        // e hi [CPI][EST] (over the scores, once read)
  uint16_t* El = Eh + CPI * EST;
  float* H1w = reinterpret_cast<float*>(wreg);             // h1 [CPI][F + 4] (over e, once read)
  const int XB = (LY::XB > LY::HB ? LY::XB : LY::HB);
  float* dnw = reinterpret_cast<float*>(wreg + XB);        // sum_r e [CPI]
  int* cvw = reinterpret_cast<int*>(dnw + CPI);            // candidate valid [CPI]

  for (int i = tid; i < F; i += NT) c1s[i] = a.c1[i];
  for (int i = tid; i < F2; i += NT) {
    c2s[i] = a.c2[i];
    h3s[i] = a.h3[i];
  }
  if constexpr (!RG) {
    for (int i = tid; i < F2 * F; i += NT) {
      H2s[i] = a.H2_hi[i];
      H2s[F2 * F + i] = a.H2_lo[i];
    }
  }
  if (tid == 0) qslot[0] = atomicAdd(a.queue, 1);
  __syncthreads();
  // sgn(w2) of this lane's unit quarter, resident as f16 pairs (+-1 exactly;
  // the |y|-fmas take them as v_fma_mix operands): A / 8 registers
  h2 sgh[A / 8];
#pragma unroll
  for (int j = 0; j < A / 8; ++j) sgh[j] = reinterpret_cast<const h2*>(a.sgn)[((tid >> 4) & 3) * (A / 8) + j];
  int u = qslot[0];

  while (u < a.nU) {
    const int64_t coff = a.cand_off[u];
    const int clen = a.cand_len[u];
    const int ctot = clen + (a.extra ? 1 : 0);
    const int ln = tid & 63;
    const int hid = ln < a.L ? a.hist[(int64_t)u * a.L + ln] : -1;
    const uint64_t vm = __ballot(ln < a.L && hid >= 0 && hid < a.n_table);
    uint64_t vm1 = 0;  // slots 64 .. 127 (LPK = 128)
    if constexpr (LP > 64) {
      const int hid1 = ln + 64 < a.L ? a.hist[(int64_t)u * a.L + ln + 64] : -1;
      vm1 = __ballot(ln + 64 < a.L && hid1 >= 0 && hid1 < a.n_table);
    }
    const int nv0 = __popcll(vm), nv = nv0 + __popcll(vm1), npad = a.L - nv, nr = nv + (npad > 0 ? 1 : 0);
    const int nrp = (nr + 31) & ~31;
    __syncthreads();  // the previous user's items are done with P', SP, R
    if (tid == 0) qslot[1] = atomicAdd(a.queue, 1);
    if (ctot > 0) {
      // [P' | R] of the valid slots, compacted; rows nv .. LP - 1 zero (the
      // shared padding row, and the e R MFMA's K padding)
      constexpr int SPARTS = RG ? A / 4 : AF / 4;  // float4 parts staged per row (RG: P' only)
      for (int e = tid; e < LP * SPARTS; e += NT) {
        const int row = e / SPARTS, part = e % SPARTS;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (row < nv) {
          const int slot = row < nv0 ? nth_set_bit(vm, row) : 64 + nth_set_bit(vm1, row - nv0);
          v = *reinterpret_cast<const float4*>(a.hproj + ((int64_t)u * a.L + slot) * AF + 4 * part);
        }
        if (RG || part < A / 4) {
          const int c = 4 * part;
          *reinterpret_cast<float4*>(Pp + row * PST + (c / AQ) * QST + c % AQ) = v;
        } else {
          const int f0 = 4 * (part - A / 4);
          const float x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            short hi, lo;
            split_bf16(x[j], hi, lo);
            const int rs = row ^ (((f0 + j) & 7) << 3);  // 8-row chunks XOR-swizzled per f (h1 reads)
            Rth[(f0 + j) * LP + rs] = (uint16_t)hi;
            Rtl[(f0 + j) * LP + rs] = (uint16_t)lo;
          }
        }
      }
    }
    __syncthreads();
    if (ctot > 0) {  // SP / 2 per row: thread = (row, eighth of the units)
      for (int r = tid >> 3; r < LP; r += NT / 8) {
        const int j = tid & 7;
        const float* pr = Pp + r * PST + (j >> 1) * QST + (j & 1) * (A / 8);  // (an eighth never straddles the quarters)
        float sp = 0.f;
#pragma unroll
        for (int i = 0; i < A / 8; ++i) sp += pr[i];
        sp = oct_sum(sp);
        if (j == 0) hSP[r] = 0.5f * sp;
      }
    }
    __syncthreads();
    const int un = qslot[1];
    const int nitem = (ctot + CPI - 1) / CPI;

    // U' of this lane's two candidates (2 pc, 2 pc + 1 of the item, unit quarter
    // q) for item it_: loaded one item ahead (during the previous item's
    // softmax and head).  An absent candidate reads a valid row (a history
    // projection): finite values in its own row of every product, never
    // written out.  (A macro: see NRK_LK_RDG.)
    float uq[2][AQ];
#define NRK_LK_LDU(it_)                                                                                  \
  {                                                                                                      \
    int tq_ = threadIdx.x;                                                                               \
    asm volatile("" : "+v"(tq_));                                                                        \
    _Pragma("unroll") for (int c_ = 0; c_ < 2; ++c_) {                                                  \
      const int ci_ = (it_) * CPI + 2 * (tq_ & 15) + c_;                                                 \
      const float* src_ = ci_ < clen ? a.cproj + (coff + ci_) * AF                                       \
                                     : (ci_ == clen && a.extra ? a.xproj + (int64_t)u * AF : a.hproj);   \
      const float* us_ = src_ + ((tq_ >> 4) & 3) * AQ;                                                   \
      _Pragma("unroll") for (int q_ = 0; q_ < AQ / 4; ++q_) {                                           \
        const float4 x_ = *reinterpret_cast<const float4*>(us_ + 4 * q_);                                \
        uq[c_][4 * q_] = x_.x;                                                                           \
        uq[c_][4 * q_ + 1] = x_.y;                                                                       \
        uq[c_][4 * q_ + 2] = x_.z;                                                                       \
        uq[c_][4 * q_ + 3] = x_.w;                                                                       \
      }                                                                                                  \
    }                                                                                                    \
  }
    if (w < nitem) NRK_LK_LDU(w)

    for (int it = w; it < nitem; it += NW) {
      // lane indices re-derived per item from a thread id the compiler cannot
      // see through: otherwise it hoists every per-lane LDS / global address
      // of the item to the kernel entry and spills them
      int tq = threadIdx.x;
      asm volatile("" : "+v"(tq));
      const int lane = tq & 63, l15 = lane & 15, l4 = lane >> 4;
      // scoring lanes: candidate pair pc, unit quarter q; after the quarters'
      // sums meet, lane q keeps candidate cs = 2 pc + (q >> 1), rows of parity h = q & 1
      const int pc = lane & 15, qq = lane >> 4, cs = 2 * pc + (qq >> 1), h = qq & 1;
      const int c0 = it * CPI, nci = ctot - c0 < CPI ? ctot - c0 : CPI;
      {  // validity of this lane's kept candidate (its id; -1 past the list)
        const int ci = c0 + cs;
        const int cid = ci < clen ? a.cand[coff + ci] : (ci == clen && a.extra ? a.extra[u] : -1);
        if (h == 0) cvw[cs] = cid >= 0 && cid < a.n_table ? 1 : 0;
      }
      float hsu;  // SU / 2 of the kept candidate
      {
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int j = 0; j < AQ; ++j) {
          s0 += uq[0][j];
          s1 += uq[1][j];
        }
        s0 = half_swap_sum(s0);
        s1 = half_swap_sum(s1);
        const auto r0 = __builtin_amdgcn_permlane16_swap(__float_as_uint(s0), __float_as_uint(s0), false, false);
        const auto r1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(s1), __float_as_uint(s1), false, false);
        s0 = __uint_as_float(r0[0]) + __uint_as_float(r0[1]);
        s1 = __uint_as_float(r1[0]) + __uint_as_float(r1[1]);
        hsu = 0.5f * ((qq >> 1) ? s1 : s0);
      }

      // ---- scores: step p = rows 2p, 2p + 1 for both candidates over this
      // lane's unit quarter; the quarters' partial sums meet by a reduce-
      // scatter of the four (candidate, row) values (two permlane32 and one
      // permlane16 swap), lane q keeping value q.  P' in groups of 8 units per
      // row, the next group read during this one (the next step's first during
      // the last), pinned by scheduling barriers.
      const float* const pbase = Pp + qq * QST;
      float4 pa[2][2], pb[2][2];  // [buffer][float4 of the group] of the two rows
      // (a macro, not a lambda: arrays captured by a lambda were left in scratch)
#define NRK_LK_RDG(p_, g, nb)                                                     \
  {                                                                               \
    const float* r0_ = pbase + (2 * (p_)) * PST + 8 * (g);                        \
    _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_) {                           \
      pa[nb][i_] = *reinterpret_cast<const float4*>(r0_ + 4 * i_);               \
      pb[nb][i_] = *reinterpret_cast<const float4*>(r0_ + PST + 4 * i_);         \
    }                                                                             \
  }
      float m = -INFINITY;
      NRK_LK_RDG(0, 0, 0)
      for (int p = 0; 2 * p < nr; ++p) {
        float acc[2][2][2] = {};  // [candidate][row][even / odd unit]
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          // (the next step's first group unconditionally: past the last step it
          // reads rows < 66, inside the block's LDS, and is never used)
          if (g + 1 < NG) NRK_LK_RDG(p, g + 1, (g + 1) & 1)
          else if (NG % 2 == 0) NRK_LK_RDG(p + 1, 0, 0)
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int qf = 2 * g + i;  // float4 of the quarter row
            const float4 x0 = pa[g & 1][i], x1 = pb[g & 1][i];
            const h2 sa = sgh[2 * qf], sb = sgh[2 * qf + 1];
            const f32x2 p0a = {x0.x, x0.y}, p0b = {x0.z, x0.w}, p1a = {x1.x, x1.y}, p1b = {x1.z, x1.w};
#pragma unroll
            for (int c = 0; c < 2; ++c) {
              const f32x2 ua = {uq[c][4 * qf], uq[c][4 * qf + 1]}, ub = {uq[c][4 * qf + 2], uq[c][4 * qf + 3]};
              const f32x2 y0a = ua + p0a, y0b = ub + p0b, y1a = ua + p1a, y1b = ub + p1b;
              acc[c][0][0] = fmaf(fabsf(y0a.x), (float)sa.x, acc[c][0][0]);
              acc[c][0][1] = fmaf(fabsf(y0a.y), (float)sa.y, acc[c][0][1]);
              acc[c][1][0] = fmaf(fabsf(y1a.x), (float)sa.x, acc[c][1][0]);
              acc[c][1][1] = fmaf(fabsf(y1a.y), (float)sa.y, acc[c][1][1]);
              acc[c][0][0] = fmaf(fabsf(y0b.x), (float)sb.x, acc[c][0][0]);
              acc[c][0][1] = fmaf(fabsf(y0b.y), (float)sb.y, acc[c][0][1]);
              acc[c][1][0] = fmaf(fabsf(y1b.x), (float)sb.x, acc[c][1][0]);
              acc[c][1][1] = fmaf(fabsf(y1b.y), (float)sb.y, acc[c][1][1]);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        if (NG % 2 != 0) NRK_LK_RDG(p + 1, 0, 0)  // (odd group count: buffer 0 was this step's last)
        // v[k], k = 2 candidate + row; lanes q < 2 keep k in {0, 1}, q >= 2 k in {2, 3}
        const float v0 = acc[0][0][0] + acc[0][0][1], v1 = acc[0][1][0] + acc[0][1][1];
        const float v2 = acc[1][0][0] + acc[1][0][1], v3 = acc[1][1][0] + acc[1][1][1];
        const auto e02 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v0), __float_as_uint(v2), false, false);
        const auto e13 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v1), __float_as_uint(v3), false, false);
        const float t0 = __uint_as_float(e02[0]) + __uint_as_float(e02[1]);  // k = 0 (q < 2) / 2 (q >= 2)
        const float t1 = __uint_as_float(e13[0]) + __uint_as_float(e13[1]);  // k = 1 / 3
        const auto e01 = __builtin_amdgcn_permlane16_swap(__float_as_uint(t0), __float_as_uint(t1), false, false);
        const float tot = __uint_as_float(e01[0]) + __uint_as_float(e01[1]);  // k = q
        const int r = 2 * p + h;
        const float sc = fmaf(0.5f, tot, hsu + hSP[r]);
        Sw[cs * SST + r] = sc;
        if (r < nr) m = fmaxf(m, sc);
      }
#undef NRK_LK_RDG
      float q1v[2][F / 16][4];  // Q1 of the C tile's candidates (from the candidate projections)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int cc = c0 + 16 * ct + 4 * l4 + k;
          const float* qs = cc < clen ? a.cproj + (coff + cc) * AF : (cc == clen && a.extra ? a.xproj + (int64_t)u * AF : nullptr);
          const float* qa = (qs ? qs : a.hproj) + A + l15;  // (an absent candidate: finite values in its own row, never written)
#pragma unroll
          for (int ft = 0; ft < F / 16; ++ft) q1v[ct][ft][k] = qa[16 * ft];
        }
      // the next item's U' (after the Q1 loads: the h1 MFMA's wait for Q1 then
      // does not cover them)
      __builtin_amdgcn_sched_barrier(0);
      if (it + NW < nitem) NRK_LK_LDU(it + NW)
      __builtin_amdgcn_sched_barrier(0);
      {  // the kept candidate's other row parity: lane ^ 16
        const auto mm = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
        m = fmaxf(__uint_as_float(mm[0]), __uint_as_float(mm[1]));
      }
      // ---- softmax weights -> bf16 hi + lo planes (rows nr .. nrp - 1 zero), sum e
      // (RG: planes by history slot, slots nks * 32 of them; invalid slots zero)
      float sum = 0.f;
      const int nks = RG ? (a.L + 31) / 32 : nrp / 32;
      if constexpr (RG) {
        // every score is read before the planes are written over them
        float es[LP / 2];
#pragma unroll
        for (int p = 0; p < LP / 2; ++p) {
          const int sl = 2 * p + h;  // history slot
          es[p] = 0.f;
          if (sl < a.L) {
            const uint64_t bits = sl < 64 ? vm : vm1;
            const int b = sl & 63;
            if ((bits >> b) & 1ull) {
              const int r = (sl < 64 ? 0 : nv0) + __popcll(bits & ((1ull << b) - 1ull));  // its compacted row
              es[p] = __expf(Sw[cs * SST + r] - m);
              sum += es[p];
            }
          }
        }
        if (npad > 0 && h == 0) sum = fmaf((float)npad, __expf(Sw[cs * SST + nv] - m), sum);  // the padding row
#pragma unroll
        for (int p = 0; p < LP / 2; ++p) {
          const int sl = 2 * p + h;
          if (sl < 32 * nks) {
            short hi, lo;
            split_bf16(es[p], hi, lo);
            Eh[cs * EST + sl] = (uint16_t)hi;
            El[cs * EST + sl] = (uint16_t)lo;
          }
        }
      } else {
        float ev[LP / 2];
#pragma unroll
        for (int p = 0; p < LP / 2; ++p) {
          const int r = 2 * p + h;
          ev[p] = 0.f;
          if (r < nr) {
            ev[p] = __expf(Sw[cs * SST + r] - m);
            sum = fmaf(r < nv ? 1.f : (float)npad, ev[p], sum);
          }
        }
#pragma unroll
        for (int p = 0; p < LP / 2; ++p) {
          const int r = 2 * p + h;
          if (r < nrp) {
            short hi, lo;
            split_bf16(ev[p], hi, lo);
            Eh[cs * EST + r] = (uint16_t)hi;
            El[cs * EST + r] = (uint16_t)lo;
          }
        }
      }
      {
        const auto ss = __builtin_amdgcn_permlane16_swap(__float_as_uint(sum), __float_as_uint(sum), false, false);
        sum = __uint_as_float(ss[0]) + __uint_as_float(ss[1]);
      }
      if (h == 0) dnw[cs] = sum;

      // ---- h1 = relu(Q1 + (e R) / sum e + c1): C tile rows = candidates 16 ct + 4 l4 + k
      constexpr int KS = LP / 32;
      bf16x8 eh[2][KS], el[2][KS];  // [ct][ks] (all read before h1 is written over them)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int o = (16 * ct + l15) * EST + 32 * ks + 8 * l4;
          eh[ct][ks] = *reinterpret_cast<const bf16x8*>(Eh + o);
          el[ct][ks] = *reinterpret_cast<const bf16x8*>(El + o);
        }
      float dv[2][4];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int k = 0; k < 4; ++k) dv[ct][k] = dnw[16 * ct + 4 * l4 + k];
      if constexpr (RG) {
        // R from the user's history projections: rows (slots) 32 ks + 8 l4 .. + 7 of
        // column A + f, split into bf16 hi + lo in registers; each fragment serves
        // both candidate tiles
        const float* hb = a.hproj + (int64_t)u * a.L * AF + A;
#pragma unroll
        for (int ft = 0; ft < F / 16; ++ft) {
          const int f = 16 * ft + l15;
          f32x4 acc[2];
#pragma unroll
          for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[ct][k] = q1v[ct][ft][k] * dv[ct][k];
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            if (ks < nks) {
              bf16x8 rh, rl;
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const int sl = 32 * ks + 8 * l4 + j;
                const float x = sl < a.L ? hb[(int64_t)sl * AF + f] : 0.f;
                short hi, lo;
                split_bf16(x, hi, lo);
                rh[j] = hi;
                rl[j] = lo;
              }
#pragma unroll
              for (int ct = 0; ct < 2; ++ct) {
                if (16 * ct < nci) {
                  acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(el[ct][ks], rh, acc[ct], 0, 0, 0);
                  acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(eh[ct][ks], rl, acc[ct], 0, 0, 0);
                  acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(eh[ct][ks], rh, acc[ct], 0, 0, 0);
                }
              }
            }
          }
          const float cb = c1s[f];
#pragma unroll
          for (int ct = 0; ct < 2; ++ct) {
            if (16 * ct >= nci) continue;
#pragma unroll
            for (int k = 0; k < 4; ++k)
              H1w[(16 * ct + 4 * l4 + k) * (F + 4) + f] =
                  fmaxf(acc[ct][k] * __builtin_amdgcn_rcpf(dv[ct][k]) + cb, 0.f);
          }
        }
      } else {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        if (16 * ct >= nci) continue;
        float rden[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) rden[k] = __builtin_amdgcn_rcpf(dv[ct][k]);
#pragma unroll
        for (int ft = 0; ft < F / 16; ++ft) {
          const int f = 16 * ft + l15;
          f32x4 acc;
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[k] = q1v[ct][ft][k] * dv[ct][k];
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            if (ks < nks) {
              // rows 32 ks + 8 l4 .. +7: chunk 4 ks + l4, stored XOR (f & 7) (a 128-B / 256-B row
              // stride would put every f of a lane group on the same banks)
              const int rc = (32 * ks + 8 * l4) ^ ((f & 7) << 3);
              const bf16x8 rh = *reinterpret_cast<const bf16x8*>(Rth + f * LP + rc);
              const bf16x8 rl = *reinterpret_cast<const bf16x8*>(Rtl + f * LP + rc);
              acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(el[ct][ks], rh, acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(eh[ct][ks], rl, acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(eh[ct][ks], rh, acc, 0, 0, 0);
            }
          }
          const float cb = c1s[f];
#pragma unroll
          for (int k = 0; k < 4; ++k) H1w[(16 * ct + 4 * l4 + k) * (F + 4) + f] = fmaxf(acc[k] * rden[k] + cb, 0.f);
        }
      }
      }  // (RG)

      // ---- h2 = relu(H2 h1 + c2), logit = h3 . h2 + c3 (16-unit tiles t2)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        if (16 * ct >= nci) continue;
        const int ca = 16 * ct + l15;
        float z[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t2 = 0; t2 < F2 / 16; ++t2) {
          const int v = 16 * t2 + l15;
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < F / 32; ++ks) {
            const float4 x0 = *reinterpret_cast<const float4*>(H1w + ca * (F + 4) + 32 * ks + 8 * l4);
            const float4 x1 = *reinterpret_cast<const float4*>(H1w + ca * (F + 4) + 32 * ks + 8 * l4 + 4);
            const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            bf16x8 hh, hl;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
              short hi, lo;
              split_bf16(xv[jj], hi, lo);
              hh[jj] = hi;
              hl[jj] = lo;
            }
            bf16x8 bh, bl;
            if constexpr (RG) {  // H2 from global memory
              bh = *reinterpret_cast<const bf16x8*>(a.H2_hi + v * F + 32 * ks + 8 * l4);
              bl = *reinterpret_cast<const bf16x8*>(a.H2_lo + v * F + 32 * ks + 8 * l4);
            } else {
              bh = *reinterpret_cast<const bf16x8*>(H2s + v * F + 32 * ks + 8 * l4);
              bl = *reinterpret_cast<const bf16x8*>(H2s + F2 * F + v * F + 32 * ks + 8 * l4);
            }
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hl, bh, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hh, bl, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hh, bh, acc, 0, 0, 0);
          }
          const float cv = c2s[v], hv = h3s[v];
#pragma unroll
          for (int k = 0; k < 4; ++k) z[k] += row_sum16(hv * fmaxf(acc[k] + cv, 0.f));
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int cc = 16 * ct + 4 * l4 + k;
          if (l15 == 0 && cc < nci) a.out[a.out_off[u] + c0 + cc] = cvw[cc] ? a.c3 + z[k] : -INFINITY;
        }
      }
    }
    u = un;
  }
#undef NRK_LK_LDU
}

// sgn(w2) per P' / U' column (the projections' slice order)
__global__ void sign_cols_kernel(const float* __restrict__ w2, int A, _Float16* __restrict__ sgn) {
  for (int n = threadIdx.x; n < A; n += blockDim.x) sgn[slice_col(n, A)] = w2[n] >= 0.f ? (_Float16)1.f : (_Float16)-1.f;
}

template <int A, int F, int LPK, bool RG>
int launch(const RerankArgs& a, hipStream_t st) {
  using LY = Lay<A, F, LPK, RG>;
  constexpr size_t lds = LY::total;
  static_assert(lds <= 160 * 1024, "din_rerank_lane: LDS");
  const int grid = a.nU < 256 ? a.nU : 256;
  hipLaunchKernelGGL((din_rerank_lane_kernel<A, F, LPK, RG>), dim3(grid), dim3(LY::NT), lds, st, a);
  NRK_CHECK_LAUNCH("din_rerank_lane_kernel");
  return NRK_OK;
}
// the 128-row form: R^T and H2 in the LDS where they fit beside P', else RG
template <int A, int F>
constexpr bool rg128() { return Lay<A, F, 128, false>::total > 160 * 1024; }
static_assert(Lay<128, 128, 128, true>::total <= 160 * 1024, "din_rerank_lane: the largest RG form must fit");
template <int A, int F>
int launch_l(const RerankArgs& a, hipStream_t st) {
  if (a.L > 64) return launch<A, F, 128, rg128<A, F>()>(a, st);
  if constexpr (F <= 64) return launch<A, F, 64, false>(a, st);
  return fail(NRK_EUNSUPPORTED, "din_rerank_lane: F = %d takes histories of 65..128 only", F);
}
template <int A>
int launch_f(const RerankArgs& a, hipStream_t st) {
  switch (a.F) {
    case 32: return launch_l<A, 32>(a, st);
    case 64: return launch_l<A, 64>(a, st);
    case 96: return launch_l<A, 96>(a, st);
    default: return launch_l<A, 128>(a, st);
  }
}
inline int launch_a(int A, const RerankArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(sign_cols_kernel, dim3(1), dim3(128), 0, st, a.w2, A, reinterpret_cast<_Float16*>(const_cast<void*>(a.sgn)));
  NRK_CHECK_LAUNCH("sign_cols_kernel");
  switch (A) {
    case 32: return launch_f<32>(a, st);
    case 64: return launch_f<64>(a, st);
    case 96: return launch_f<96>(a, st);
    default: return launch_f<128>(a, st);
  }
}
}  // namespace lk

int launch_lane(int A, const RerankArgs& a, hipStream_t st) { return lk::launch_a(A, a, st); }

int lane_max_l(int A, int F) {
  // every (A, F) of the grid: 128 (F > 64 through the RG form only, for L > 64)
  return (A % 32 == 0 && A >= 32 && A <= 128 && F % 32 == 0 && F >= 32 && F <= 128) ? 128 : 0;
}

}  // namespace rr
}  // namespace nrk
