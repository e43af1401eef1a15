/*
 * oracle/knn_exact.c — TEST INFRASTRUCTURE ONLY (the checker, never the
 * product).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library.
 *
 * CPU restatement of the flat k-NN search contract the reference relies on:
 *   Retrieval.py:25-26  centroid_index = faiss.IndexFlatL2(d); .add(centroids)
 *   Retrieval.py:31-32  _, I = centroid_index.search(profile, 1)
 *   Retrieval.py:21     _, assignments = index.search(embeddings, 1)
 * faiss itself is an external, unvendored and unpinned dependency (no
 * requirements file in the reference; faiss is not importable in this image or
 * on the GPU box), so its PUBLISHED semantics are restated here:
 *   - IndexFlatIP: D = <q, x>, best = largest;  IndexFlatL2: D = ||q - x||^2
 *     (squared), best = smallest;
 *   - ids are insertion order (0..ntotal-1, plus the caller's id offset);
 *   - k > ntotal pads I with -1 and D with -FLT_MAX (IP) / +FLT_MAX (L2)
 *     (faiss CMin/CMax heap neutral values).
 * Where faiss leaves the order unspecified we fix it ("parity unpinned" for the
 * faiss part — there is no reference fixture to pin against):
 *   - scores are EXACT: products of two fp32 values are exact in fp64, and the
 *     sum runs sequentially over j = 0..d-1 with fma() in fp64
 *     (IP: acc = fma(q_j, x_j, acc); L2: t = q_j - x_j; acc = fma(t, t, acc));
 *   - ties on the fp64 score break toward the LOWER id;
 *   - D is the fp64 score rounded to fp32.
 * The GPU rescoring kernel uses the identical operation sequence, so its scores
 * are bit-identical to these and index parity can be asserted exactly.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define METRIC_IP 0
#define METRIC_L2 1

static inline double score_ip(const float* q, const float* x, int d) {
  double acc = 0.0;
  for (int j = 0; j < d; ++j) acc = fma((double)q[j], (double)x[j], acc);
  return acc;
}

static inline double score_l2(const float* q, const float* x, int d) {
  double acc = 0.0;
  for (int j = 0; j < d; ++j) {
    double t = (double)q[j] - (double)x[j];
    acc = fma(t, t, acc);
  }
  return acc;
}

/* a better than b? (IP: larger; L2: smaller; ties: lower id) */
static inline int better(int metric, double as, int64_t ai, double bs, int64_t bi) {
  if (metric == METRIC_IP) {
    if (as != bs) return as > bs;
  } else {
    if (as != bs) return as < bs;
  }
  return ai < bi;
}

/* Exact top-k for nq queries.  S (fp64 scores) may be NULL. */
int oracle_knn_exact(const float* xq, int64_t nq, const float* xb, int64_t nb, int d, int k,
                     int metric, float* D, int64_t* I, double* S, int64_t id_offset) {
  if (k <= 0 || d <= 0 || nq < 0 || nb < 0) return -1;
  if (metric != METRIC_IP && metric != METRIC_L2) return -1;
#pragma omp parallel
  {
    double* ls = (double*)malloc(sizeof(double) * (size_t)k);
    int64_t* li = (int64_t*)malloc(sizeof(int64_t) * (size_t)k);
#pragma omp for schedule(dynamic, 4)
    for (int64_t qi = 0; qi < nq; ++qi) {
      const float* q = xq + qi * (int64_t)d;
      int n = 0; /* filled entries, sorted best-first */
      for (int64_t i = 0; i < nb; ++i) {
        const float* x = xb + i * (int64_t)d;
        double s = metric == METRIC_IP ? score_ip(q, x, d) : score_l2(q, x, d);
        if (n == k && !better(metric, s, i, ls[k - 1], li[k - 1])) continue;
        int pos = n < k ? n : k - 1;
        while (pos > 0 && better(metric, s, i, ls[pos - 1], li[pos - 1])) {
          ls[pos] = ls[pos - 1];
          li[pos] = li[pos - 1];
          --pos;
        }
        ls[pos] = s;
        li[pos] = i;
        if (n < k) ++n;
      }
      for (int j = 0; j < k; ++j) {
        int64_t o = qi * (int64_t)k + j;
        if (j < n) {
          D[o] = (float)ls[j];
          I[o] = li[j] + id_offset;
          if (S) S[o] = ls[j];
        } else {
          D[o] = metric == METRIC_IP ? -FLT_MAX : FLT_MAX;
          I[o] = -1;
          if (S) S[o] = metric == METRIC_IP ? -DBL_MAX : DBL_MAX;
        }
      }
    }
    free(ls);
    free(li);
  }
  return 0;
}

/* Merge per-shard lists (same order as above) — the restatement of what a
 * sharded search must return: identical to one search over the whole corpus. */
int oracle_topk_merge(const double* S_parts, const int64_t* I_parts, int nparts, int64_t nq, int k,
                      int metric, float* D, int64_t* I, double* S) {
  for (int64_t qi = 0; qi < nq; ++qi) {
    int* pos = (int*)calloc((size_t)nparts, sizeof(int));
    for (int j = 0; j < k; ++j) {
      int best = -1;
      for (int p = 0; p < nparts; ++p) {
        if (pos[p] >= k) continue;
        int64_t o = ((int64_t)p * nq + qi) * k + pos[p];
        if (I_parts[o] < 0) continue;
        if (best < 0) { best = p; continue; }
        int64_t ob = ((int64_t)best * nq + qi) * k + pos[best];
        if (better(metric, S_parts[o], I_parts[o], S_parts[ob], I_parts[ob])) best = p;
      }
      int64_t oo = qi * (int64_t)k + j;
      if (best < 0) {
        D[oo] = metric == METRIC_IP ? -FLT_MAX : FLT_MAX;
        I[oo] = -1;
        if (S) S[oo] = metric == METRIC_IP ? -DBL_MAX : DBL_MAX;
      } else {
        int64_t ob = ((int64_t)best * nq + qi) * k + pos[best];
        D[oo] = (float)S_parts[ob];
        I[oo] = I_parts[ob];
        if (S) S[oo] = S_parts[ob];
        pos[best]++;
      }
    }
    free(pos);
  }
  return 0;
}
