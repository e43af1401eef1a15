// ivf_build.hip — inverted-list construction and k-means centroid update for
// gfx950 (replaces faiss Clustering.train + the list building of
// Retrieval.py:11-23 and IndexIVFFlat.add).
//
//   group_by_list : stable counting sort of ids by list (ids ascending inside
//                   every list, like faiss's insertion order):
//                   per-4096-id block LDS histograms -> per-list running
//                   offsets -> one wave per block ranks equal labels with
//                   ballots, in id order
//   ivf_pack      : gathers the bf16 screening rows / norms into list order
//   kmeans_update : centroid = fp64 sum of its members in id order / count
//                   (deterministic; oracle/kmeans.py restates it)
// All of these are HBM-bound byte movers (no MFMA): coalesced row copies and
// LDS histograms.
#include "nrk_common.h"

namespace nrk {

constexpr int GB_CH = 4096;  // ids per histogram block

__global__ __launch_bounds__(256) void gb_hist_kernel(const int64_t* __restrict__ assign, int64_t n, int nlist,
                                                      int* __restrict__ hist, int* __restrict__ bad) {
  extern __shared__ int h[];
  for (int l = threadIdx.x; l < nlist; l += 256) h[l] = 0;
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * GB_CH;
  const int64_t hi = lo + GB_CH < n ? lo + GB_CH : n;
  for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
    const int64_t a = assign[i];
    if (a < 0 || a >= nlist) {
      atomicAdd(bad, 1);
      continue;
    }
    atomicAdd(&h[a], 1);
  }
  __syncthreads();
  for (int l = threadIdx.x; l < nlist; l += 256) hist[(int64_t)blockIdx.x * nlist + l] = h[l];
}

// thread per list: exclusive running offsets over the blocks, list sizes
__global__ void gb_colscan_kernel(int* __restrict__ hist, int nblk, int nlist, int64_t* __restrict__ sizes) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= nlist) return;
  int64_t run = 0;
  for (int b = 0; b < nblk; ++b) {
    const int v = hist[(int64_t)b * nlist + l];
    hist[(int64_t)b * nlist + l] = (int)run;
    run += v;
  }
  sizes[l] = run;
}

// one block: list_off = exclusive scan of sizes (nlist + 1 entries)
__global__ __launch_bounds__(1024) void gb_offsets_kernel(const int64_t* __restrict__ sizes, int nlist,
                                                          int64_t* __restrict__ list_off) {
  __shared__ int64_t s[1024];
  const int t = threadIdx.x;
  const int per = (nlist + 1023) / 1024;
  const int lo = t * per < nlist ? t * per : nlist, hi = lo + per < nlist ? lo + per : nlist;
  int64_t sum = 0;
  for (int l = lo; l < hi; ++l) sum += sizes[l];
  s[t] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int64_t a = t >= o ? s[t - o] : 0;
    __syncthreads();
    s[t] += a;
    __syncthreads();
  }
  int64_t e = s[t] - sum;
  for (int l = lo; l < hi; ++l) {
    list_off[l] = e;
    e += sizes[l];
  }
  if (t == 1023) list_off[nlist] = s[1023];
}

// one wave per block of GB_CH ids, in id order: rank = equal labels in lower
// lanes (ballot per distinct label), run[] advances by each label's count
__global__ __launch_bounds__(64) void gb_scatter_kernel(const int64_t* __restrict__ assign, int64_t n, int nlist,
                                                        const int* __restrict__ hist,
                                                        const int64_t* __restrict__ list_off,
                                                        int64_t* __restrict__ pos2id, int* __restrict__ pos2list) {
  extern __shared__ int run[];
  const int lane = threadIdx.x;
  for (int l = lane; l < nlist; l += 64) run[l] = hist[(int64_t)blockIdx.x * nlist + l];
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * GB_CH;
  const int64_t hi = lo + GB_CH < n ? lo + GB_CH : n;
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int64_t base = lo; base < hi; base += 64) {
    const int64_t i = base + lane;
    const int a = i < hi ? (int)assign[i] : -1;
    unsigned long long todo = __ballot(a >= 0);
    int rank = 0, total = 0;
    while (todo) {  // one round per distinct label in this group of 64
      const int leader = __ffsll((long long)todo) - 1;
      const int la = __shfl(a, leader, 64);
      const unsigned long long same = __ballot(a == la);
      if (a == la) {
        rank = __popcll(same & below);
        total = __popcll(same);
      }
      todo &= ~same;
    }
    if (a >= 0) {
      const int64_t pos = list_off[a] + run[a] + rank;
      pos2id[pos] = i;
      pos2list[pos] = a;
    }
    __syncthreads();  // all reads of run[] for this group are done
    if (a >= 0 && rank == total - 1) run[a] += total;
    __syncthreads();
  }
}

// list-major copy of the bf16 rows and per-row norms: one wave per position
__global__ void ivf_pack_kernel(const int64_t* __restrict__ pos2id, int64_t n, int dp,
                                const uint16_t* __restrict__ xbh, const float* __restrict__ meta,
                                uint16_t* __restrict__ xbh_ivf, float* __restrict__ meta_ivf) {
  const int lane = threadIdx.x & 63;
  const int64_t pos = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (pos >= n) return;
  const int64_t id = pos2id[pos];
  for (int j = lane * 4; j < dp; j += 256)
    *reinterpret_cast<uint2*>(xbh_ivf + pos * dp + j) = *reinterpret_cast<const uint2*>(xbh + id * dp + j);
  if (lane < 2) meta_ivf[2 * pos + lane] = meta[2 * id + lane];
}

// block per cluster, thread per dimension: fp64 sum over members in id order
__global__ void kmeans_update_kernel(const float* __restrict__ x, int d, const int64_t* __restrict__ list_off,
                                     const int64_t* __restrict__ pos2id, float* __restrict__ centroids) {
  const int c = blockIdx.x;
  const int64_t lo = list_off[c], hi = list_off[c + 1];
  if (hi == lo) return;  // empty: left to the caller's split step
  for (int j = threadIdx.x; j < d; j += blockDim.x) {
    double acc = 0.0;
    for (int64_t p = lo; p < hi; ++p) acc += (double)x[pos2id[p] * d + j];
    centroids[(int64_t)c * d + j] = (float)(acc / (double)(hi - lo));
  }
}

}  // namespace nrk

using namespace nrk;

extern "C" int nrk_group_by_list_workspace(int64_t n, int32_t nlist, size_t* ws_bytes) {
  NRK_CHECK_ARG(ws_bytes && n >= 0 && nlist > 0, "group_by_list_workspace: bad arguments");
  const int64_t nblk = cdiv(n, GB_CH);
  *ws_bytes = align_up((size_t)nblk * nlist * 4, 256) + align_up((size_t)nlist * 8, 256) + 256;
  return NRK_OK;
}

extern "C" int nrk_group_by_list(const int64_t* assign, int64_t n, int32_t nlist, int64_t* list_off, int64_t* pos2id,
                                 int32_t* pos2list, int32_t* n_bad, void* ws, size_t ws_bytes, void* stream) {
  NRK_CHECK_ARG(n >= 0 && nlist > 0 && nlist <= 16384, "group_by_list: bad shape n=%lld nlist=%d", (long long)n,
                nlist);
  NRK_CHECK_ARG(list_off && n_bad && ws, "group_by_list: null pointer");
  size_t need = 0;
  nrk_group_by_list_workspace(n, nlist, &need);
  if (ws_bytes < need) return fail(NRK_EWORKSPACE, "group_by_list: workspace %zu < %zu bytes", ws_bytes, need);
  hipStream_t st = (hipStream_t)stream;
  const int nblk = (int)cdiv(n, GB_CH);
  char* w = static_cast<char*>(ws);
  int* hist = reinterpret_cast<int*>(w);
  int64_t* sizes = reinterpret_cast<int64_t*>(w + align_up((size_t)nblk * nlist * 4, 256));
  if (hipMemsetAsync(n_bad, 0, 4, st) != hipSuccess) return fail(NRK_ELAUNCH, "group_by_list: memset failed");
  if (n == 0) {
    if (hipMemsetAsync(list_off, 0, (size_t)(nlist + 1) * 8, st) != hipSuccess)
      return fail(NRK_ELAUNCH, "group_by_list: memset failed");
    return NRK_OK;
  }
  NRK_CHECK_ARG(assign && pos2id && pos2list, "group_by_list: null pointer");
  hipLaunchKernelGGL(gb_hist_kernel, dim3(nblk), dim3(256), (size_t)nlist * 4, st, assign, n, nlist, hist, n_bad);
  NRK_CHECK_LAUNCH("gb_hist_kernel");
  hipLaunchKernelGGL(gb_colscan_kernel, dim3((unsigned)cdiv(nlist, 256)), dim3(256), 0, st, hist, nblk, nlist, sizes);
  NRK_CHECK_LAUNCH("gb_colscan_kernel");
  hipLaunchKernelGGL(gb_offsets_kernel, dim3(1), dim3(1024), 0, st, sizes, nlist, list_off);
  NRK_CHECK_LAUNCH("gb_offsets_kernel");
  hipLaunchKernelGGL(gb_scatter_kernel, dim3(nblk), dim3(64), (size_t)nlist * 4, st, assign, n, nlist, hist, list_off,
                     pos2id, pos2list);
  NRK_CHECK_LAUNCH("gb_scatter_kernel");
  return NRK_OK;
}

extern "C" int nrk_ivf_pack(const int64_t* pos2id, int64_t n, int32_t d, const uint16_t* xb_bf16,
                            const float* xb_meta, uint16_t* xbh_ivf, float* meta_ivf, void* stream) {
  NRK_CHECK_ARG(n >= 0 && d > 0, "ivf_pack: bad shape");
  if (n == 0) return NRK_OK;
  NRK_CHECK_ARG(pos2id && xb_bf16 && xb_meta && xbh_ivf && meta_ivf, "ivf_pack: null pointer");
  const int dp = nrk_padded_dim(d);
  hipLaunchKernelGGL(ivf_pack_kernel, dim3((unsigned)cdiv(n, 4)), dim3(256), 0, (hipStream_t)stream, pos2id, n, dp,
                     xb_bf16, xb_meta, xbh_ivf, meta_ivf);
  NRK_CHECK_LAUNCH("ivf_pack_kernel");
  return NRK_OK;
}

extern "C" int nrk_kmeans_update(const float* x, int32_t d, const int64_t* list_off, const int64_t* pos2id,
                                 int32_t k, float* centroids, void* stream) {
  NRK_CHECK_ARG(d > 0 && k > 0, "kmeans_update: bad shape d=%d k=%d", d, k);
  NRK_CHECK_ARG(x && list_off && pos2id && centroids, "kmeans_update: null pointer");
  const int threads = d >= 256 ? 256 : (int)align_up((size_t)d, 64);
  hipLaunchKernelGGL(kmeans_update_kernel, dim3(k), dim3(threads), 0, (hipStream_t)stream, x, d, list_off, pos2id,
                     centroids);
  NRK_CHECK_LAUNCH("kmeans_update_kernel");
  return NRK_OK;
}
