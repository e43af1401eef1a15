// embed.hip — the corpus producer (embedding_generate.py:51-65, 109-121):
// ArticleEmbeddingModel in eval mode, out = relu(x W1^T + b1) W2'^T + b2'
// (the eval BatchNorm folded into fc.4 by the caller), for a whole corpus in
// one launch, h never leaving the chip.
//
// Precision: fp32 products from bf16 MFMAs.  Every fp32 operand is split
// EXACTLY into three bf16 planes (x = h + m + l: 8 + 8 + 8 mantissa bits), and
// a product keeps the six terms down to 2^-16 of the leading one (hh, hm, mh,
// hl, lh, mm; the dropped ml, lm, ll are below 2^-24), accumulated in fp32 by
// the MFMA: the error is that of an fp32 dot product (measured against the
// reference's own inference() in tests/test_embedding.py).  Six
// v_mfma_f32_16x16x32_bf16 per 16x16x32 block deliver 2.5 / 6 = 0.42 PF/s of
// fp32-exact products at peak, 2.65x the 157 TF/s of v_mfma_f32_32x32x2_f32.
//
// One 256-thread workgroup (4 waves, one per SIMD) per 64-row tile, one per
// CU (LDS): x tile -> three bf16 planes in LDS (swizzled 16-B chunks:
// conflict-free 16x16x32 A-fragment reads), then per chunk of HC = 128
// hidden units:
//   layer 1  H_j = relu(x W1[j]^T + b1[j]) (wave w: hidden units 32 w ..
//            32 w + 31 of the chunk, all 64 rows; W1 fragments from L2, each
//            reused over the four row tiles), split into three planes in LDS;
//   layer 2  O += H_j W2[:, j]^T (wave w: output columns 64 w .. 64 w + 63,
//            all 64 rows: 16 accumulator tiles resident over the chunks).
// Finally O + b2' -> HBM.
#include "nrk_common.h"

namespace nrk {
namespace emb {

constexpr int NT = 256;  // 4 waves: one per SIMD
constexpr int RT = 64;   // rows per workgroup
constexpr int KP = 256;  // input width, zero-padded (253 -> 256)
constexpr int HC = 128;  // hidden units per chunk
constexpr int OD = 256;  // output width

// byte offset of 16-B chunk `chunk` of `row` in a [rows][W] bf16 plane
template <int W>
__device__ __forceinline__ int poff(int row, int chunk) {
  constexpr int CPR = W / 8;
  constexpr int SW = CPR >= 16 ? 15 : CPR - 1;
  return row * 2 * W + 16 * (chunk ^ (row & SW));
}

__device__ __forceinline__ void split3(float x, short& h, short& m, short& l) {
  const __bf16 bh = (__bf16)x;
  const float r1 = x - (float)bh;  // exact
  const __bf16 bm = (__bf16)r1;
  const float r2 = r1 - (float)bm;  // exact, <= 8 significant bits: bf16-exact
  h = __builtin_bit_cast(short, bh);
  m = __builtin_bit_cast(short, bm);
  l = __builtin_bit_cast(short, (__bf16)r2);
}

// the six products of a and b (three planes each), small terms first
__device__ __forceinline__ f32x4 mfma6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);  // mm
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);  // lh
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);  // hl
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);  // mh
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);  // hm
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);  // hh
  return acc;
}

struct EmbedArgs {
  const float* x;  // [n][ldx], in_dim <= KP used
  int64_t n, ldx;
  int in_dim, H;
  // Weights as bf16 planes in MFMA B-fragment order: fragment (n16, s, plane) =
  // rows 16 n16 .. + 15, columns 32 s .. + 31 of that plane, 1 KiB, lane
  // l15 + 16 l4 holding row 16 n16 + l15, columns 32 s + 8 l4 .. + 7 — one
  // fragment is one contiguous wave load (row-major planes made each load 16
  // half-lines of 16 rows).
  const uint16_t* W1p;  // fc.0.weight, [H / 16][KP / 32][3] fragments (zero-padded columns)
  const float* b1;      // [H]
  const uint16_t* W2p;  // the folded fc.4 weight, [OD / 16][H / 32][3] fragments
  const float* b2;      // [OD]
  float* out;           // [n][OD]
};

// Register blocking: one wave per SIMD, each with a 64-row x 32-column tile of
// layer 1 (a chunk of HC = 128 hidden units over the four waves) and a 64-row
// x 64-column tile of layer 2: per K step a wave reads 4 row fragments (x 3
// planes) from LDS and 2 / 4 column fragments (x 3 planes) from L2 for 48 / 96
// MFMAs, so neither LDS nor L2 bandwidth paces the MFMA chain.  The next K
// step's weight fragments are loaded during the current one.
__global__ __launch_bounds__(NT, 1) void embed_mlp_kernel(EmbedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int XPL = RT * KP * 2;  // bytes per x plane
  constexpr int HPL = RT * HC * 2;  // bytes per H plane
  unsigned char* xs = smem;            // [3] x planes
  unsigned char* hs = smem + 3 * XPL;  // [3] H planes
  const int tid = threadIdx.x, lane = tid & 63, l15 = lane & 15, l4 = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t r0 = (int64_t)blockIdx.x * RT;

  // ---- x tile -> three planes.  Wave w loads rows 16 w .. 16 w + 15, lane l the
  // columns l, l + 64, l + 128, l + 192 of each: every load instruction reads
  // 256 contiguous bytes of one row (a (row, 8-column piece) split made each
  // instruction touch 16 cache lines for 256 B).  All loads are in flight before
  // the first is used (clamped addresses, masked afterwards); the planes are
  // written element by element.
  {
    constexpr int RPW = RT / 4;  // rows per wave
    float v[RPW][4];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int64_t r = r0 + RPW * w + i, rc = r < a.n ? r : a.n - 1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 64 * q + lane, cc = c < a.in_dim ? c : a.in_dim - 1;
        v[i][q] = __builtin_nontemporal_load(a.x + rc * a.ldx + cc);
      }
    }
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int row = RPW * w + i;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 64 * q + lane;
        short h, m, l;
        split3(r0 + row < a.n && c < a.in_dim ? v[i][q] : 0.f, h, m, l);
        const int o = poff<KP>(row, c >> 3) + 2 * (c & 7);
        *reinterpret_cast<short*>(xs + o) = h;
        *reinterpret_cast<short*>(xs + XPL + o) = m;
        *reinterpret_cast<short*>(xs + 2 * XPL + o) = l;
      }
    }
  }
  f32x4 acc2[4][4];  // layer 2: row tile rt, column tile oc (columns 64 w + 16 oc + l15)
#pragma unroll
  for (int rt = 0; rt < 4; ++rt)
#pragma unroll
    for (int oc = 0; oc < 4; ++oc) acc2[rt][oc] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nch = a.H / HC;
  // Software pipeline, pinned with scheduling barriers (the scheduler otherwise
  // sinks each load next to its first use and waits out its latency with one
  // wave per SIMD and nothing else to issue): per (K step, row tile) pair the
  // next pair's A fragments are read from LDS, and per K step the next step's
  // weight fragments are loaded from L2, one step (4 pairs) ahead.  The first
  // weight step of each layer is loaded while the other layer finishes.
  bf16x8 b1f[2][2][3];  // layer-1 weights [buffer][ct][plane]
  bf16x8 b2f[2][4][3];  // layer-2 weights [buffer][oc][plane]
  auto load_b1 = [&](int j, int s, int nb) __attribute__((always_inline)) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const uint16_t* wb = a.W1p + ((int64_t)((j * HC / 16 + 2 * w + ct) * (KP / 32) + s) * 3) * 512 + 8 * lane;
#pragma unroll
      for (int p = 0; p < 3; ++p) b1f[nb][ct][p] = *reinterpret_cast<const bf16x8*>(wb + 512 * p);
    }
  };
  auto load_b2 = [&](int j, int s, int nb) __attribute__((always_inline)) {
#pragma unroll
    for (int oc = 0; oc < 4; ++oc) {
      const uint16_t* wb = a.W2p + ((int64_t)((4 * w + oc) * (a.H / 32) + j * (HC / 32) + s) * 3) * 512 + 8 * lane;
#pragma unroll
      for (int p = 0; p < 3; ++p) b2f[nb][oc][p] = *reinterpret_cast<const bf16x8*>(wb + 512 * p);
    }
  };
  load_b1(0, 0, 0);
  for (int j = 0; j < nch; ++j) {
    __syncthreads();  // j = 0: the x planes published; else layer 2 of chunk j - 1 is done with H
    // ---- layer 1: hidden units j HC + 32 w + 16 ct + l15, all 64 rows
    {
      f32x4 c[4][2];
#pragma unroll
      for (int rt = 0; rt < 4; ++rt)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) c[rt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
      bf16x8 xa[2][3];
      auto load_a = [&](int it, int nb) __attribute__((always_inline)) {
        const int o = poff<KP>(16 * (it & 3) + l15, 4 * (it >> 2) + l4);
#pragma unroll
        for (int p = 0; p < 3; ++p) xa[nb][p] = *reinterpret_cast<const bf16x8*>(xs + p * XPL + o);
      };
      load_a(0, 0);
#pragma unroll
      for (int it = 0; it < 4 * (KP / 32); ++it) {
        const int s = it >> 2, rt = it & 3;
        if (rt == 0 && s + 1 < KP / 32) load_b1(j, s + 1, (s + 1) & 1);
        if (it + 1 < 4 * (KP / 32)) load_a(it + 1, (it + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) c[rt][ct] = mfma6(xa[it & 1], b1f[s & 1][ct], c[rt][ct]);
        __builtin_amdgcn_sched_barrier(0);
      }
      load_b2(j, 0, 0);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const int col = 32 * w + 16 * ct + l15;  // within the chunk
        const float bu = a.b1[j * HC + col];
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = 16 * rt + 4 * l4 + i;
            short h, m, l;
            split3(fmaxf(c[rt][ct][i] + bu, 0.f), h, m, l);
            const int o = poff<HC>(row, col >> 3) + 2 * (col & 7);
            *reinterpret_cast<short*>(hs + o) = h;
            *reinterpret_cast<short*>(hs + HPL + o) = m;
            *reinterpret_cast<short*>(hs + 2 * HPL + o) = l;
          }
      }
    }
    __syncthreads();  // H_j published
    // ---- layer 2: O[:, 64 w .. 64 w + 63] += H_j W2[64 w .., chunk j]^T
    {
      bf16x8 hx[2][3];
      auto load_h = [&](int it, int nb) __attribute__((always_inline)) {
        const int o = poff<HC>(16 * (it & 3) + l15, 4 * (it >> 2) + l4);
#pragma unroll
        for (int p = 0; p < 3; ++p) hx[nb][p] = *reinterpret_cast<const bf16x8*>(hs + p * HPL + o);
      };
      load_h(0, 0);
#pragma unroll
      for (int it = 0; it < 4 * (HC / 32); ++it) {
        const int s = it >> 2, rt = it & 3;
        if (rt == 0 && s + 1 < HC / 32) load_b2(j, s + 1, (s + 1) & 1);
        if (rt == 0 && s + 1 == HC / 32 && j + 1 < nch) load_b1(j + 1, 0, 0);
        if (it + 1 < 4 * (HC / 32)) load_h(it + 1, (it + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int oc = 0; oc < 4; ++oc) acc2[rt][oc] = mfma6(hx[it & 1], b2f[s & 1][oc], acc2[rt][oc]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  // ---- O + b2 -> HBM
#pragma unroll
  for (int oc = 0; oc < 4; ++oc) {
    const int col = 64 * w + 16 * oc + l15;
    const float bo = a.b2[col];
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t r = r0 + 16 * rt + 4 * l4 + i;
        if (r < a.n) __builtin_nontemporal_store(acc2[rt][oc][i] + bo, a.out + r * OD + col);  // (streamed: keep L2 for the weights)
      }
  }
}

// fp32 weights [rows][cols] -> three bf16 planes (exact split), zero-padded to
// cols_p columns, in B-fragment order (EmbedArgs::W1p); rows % 16 == 0, cols_p % 32 == 0
__global__ void split_planes_kernel(const float* __restrict__ w, int rows, int cols, int cols_p,
                                    uint16_t* __restrict__ frags) {
  const int64_t n = (int64_t)rows * cols_p;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols_p), c = (int)(i % cols_p);
    short h, m, l;
    split3(c < cols ? w[(int64_t)r * cols + c] : 0.f, h, m, l);
    const int64_t f = ((int64_t)(r >> 4) * (cols_p >> 5) + (c >> 5)) * 3 * 512 + 8 * ((r & 15) + 16 * ((c & 31) >> 3)) + (c & 7);
    frags[f] = (uint16_t)h;
    frags[f + 512] = (uint16_t)m;
    frags[f + 1024] = (uint16_t)l;
  }
}

}  // namespace emb
}  // namespace nrk

using namespace nrk;

extern "C" int nrk_embed_workspace(int32_t in_dim, int32_t hidden, int32_t out_dim, size_t* ws_bytes) {
  NRK_CHECK_ARG(ws_bytes, "embed_workspace: null");
  NRK_CHECK_ARG(in_dim >= 1 && in_dim <= emb::KP && hidden >= emb::HC && hidden % emb::HC == 0 &&
                    out_dim == emb::OD,
                "embed: dims %d -> %d -> %d unsupported (in <= %d, hidden a multiple of %d, out %d)", in_dim, hidden,
                out_dim, emb::KP, emb::HC, emb::OD);
  *ws_bytes = align_up((size_t)3 * hidden * emb::KP * 2, 256) + (size_t)3 * emb::OD * hidden * 2;
  return NRK_OK;
}

extern "C" int nrk_embed(const float* x, int64_t n, int64_t ldx, int32_t in_dim, const float* W1, const float* b1,
                         int32_t hidden, const float* W2, const float* b2, int32_t out_dim, float* out, void* ws,
                         size_t ws_bytes, void* stream) {
  size_t need = 0;
  int rc = nrk_embed_workspace(in_dim, hidden, out_dim, &need);
  if (rc) return rc;
  NRK_CHECK_ARG(n >= 0 && ldx >= in_dim, "embed: bad n=%lld / ldx=%lld", (long long)n, (long long)ldx);
  if (n == 0) return NRK_OK;
  NRK_CHECK_ARG(x && W1 && b1 && W2 && b2 && out && ws, "embed: null pointer");
  if (ws_bytes < need) return fail(NRK_EWORKSPACE, "embed: workspace %zu < %zu", ws_bytes, need);
  NRK_CHECK_ARG(n <= (int64_t)0x7fffffff * emb::RT, "embed: too many rows");
  hipStream_t st = (hipStream_t)stream;
  uint16_t* W1p = static_cast<uint16_t*>(ws);
  uint16_t* W2p = reinterpret_cast<uint16_t*>(static_cast<char*>(ws) + align_up((size_t)3 * hidden * emb::KP * 2, 256));
  hipLaunchKernelGGL(emb::split_planes_kernel, dim3(256), dim3(256), 0, st, W1, hidden, in_dim, emb::KP, W1p);
  hipLaunchKernelGGL(emb::split_planes_kernel, dim3(256), dim3(256), 0, st, W2, emb::OD, hidden, hidden, W2p);
  NRK_CHECK_LAUNCH("split_planes_kernel");
  emb::EmbedArgs a{x, n, ldx, in_dim, hidden, W1p, b1, W2p, b2, out};
  const size_t lds = (size_t)3 * emb::RT * emb::KP * 2 + (size_t)3 * emb::RT * emb::HC * 2;
  hipLaunchKernelGGL(emb::embed_mlp_kernel, dim3((unsigned)cdiv(n, emb::RT)), dim3(emb::NT), lds, st, a);
  NRK_CHECK_LAUNCH("embed_mlp_kernel");
  return NRK_OK;
}
