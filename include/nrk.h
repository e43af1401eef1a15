/*
 * nrk.h — C-ABI of libnrk.so, the MI355X (gfx950) kernels behind the
 * NewsRecommend hot path.
 *
 * The reference (YuxuanZhao/NewsRecommend) has no native code: its hot path
 * runs through PyTorch ATen (DIN.py) and faiss-cpu (Retrieval.py).  Each entry
 * point below replaces one reference interface; the citation says which.  The
 * Python side (newsrecommend_amd/_lib.py) binds these with ctypes, the way a
 * maintainer of the reference would.
 *
 * Conventions (all entry points):
 *   - every pointer is a DEVICE pointer owned by the caller (torch tensors),
 *     except where a parameter says "host";
 *   - the library never allocates, frees or synchronises; all work is enqueued
 *     on `stream` (a hipStream_t passed as void*), so calls are graph-capturable;
 *   - return 0 on success, a negative NRK_E* code on failure; the message is in
 *     thread-local storage, read with nrk_last_error();
 *   - no mutable global state: the library is re-entrant.
 */
#ifndef NRK_H
#define NRK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes */
#define NRK_OK 0
#define NRK_EINVAL (-1)   /* bad argument (shape, k, metric, null pointer) */
#define NRK_EWORKSPACE (-2) /* workspace too small */
#define NRK_ELAUNCH (-3)  /* kernel launch failed */
#define NRK_EUNSUPPORTED (-4)

/* metrics: same numeric values as faiss::MetricType */
#define NRK_METRIC_INNER_PRODUCT 0
#define NRK_METRIC_L2 1

/* element types of embedding tables */
#define NRK_DTYPE_F32 0
#define NRK_DTYPE_BF16 1

struct nrk_din_head_params_s; /* typedef'd as nrk_din_head_params below */

const char* nrk_last_error(void);
int nrk_version(void);

/* ------------------------------------------------------------------------- *
 * Flat (exhaustive) k-NN search — replaces faiss IndexFlatIP / IndexFlatL2
 * `.add(x)` and `.search(x, k)` (reference call sites Retrieval.py:25-26,31-32
 * and the assignment search Retrieval.py:21).  Semantics restated in
 * oracle/knn_exact.c: exact scores, IP descending / squared L2 ascending,
 * ties broken by lower id, k > ntotal padded with id -1.
 * ------------------------------------------------------------------------- */

/* Per-corpus state built once per add():
 *   xb_bf16  [nb][dp] bf16 (uint16), dp = nrk_padded_dim(d), zero-padded
 *   xb_meta  [nb][2] float: {||x||^2 (fp32, exact-rounded), ||x - bf16(x)|| rounded up}
 *   stats    [4] float: {max ||bf16(x)||, max residual norm, max ||x||^2, 0},
 *            accumulated with atomic max, so zero it before the first prepare
 *            call of an index (prepare may be called on appended slices). */
int nrk_padded_dim(int32_t d);
/* Name of the main-pass kernel nrk_knn_flat runs for this shape (for
 * benchmark records and profiles): writes a NUL-terminated string of at most
 * len bytes into name.  No reference counterpart (faiss has no such query). */
int nrk_knn_flat_main_pass(int64_t nq, int64_t nb, int32_t d, int32_t k, int32_t metric, char* name, size_t len);
int nrk_flat_prepare(const float* xb, int64_t nb, int32_t d, uint16_t* xb_bf16,
                     float* xb_meta, float* stats, void* stream);

/* Workspace bytes needed by nrk_knn_flat for this problem.  For the screened
 * path it is about nq * (2 * 4 * U + 2 * dp + 64) bytes (U = per-query
 * candidate union, <= 2048: 32..256 at k <= 8) plus s * (16 * fb_cap + 4 * 2048
 * + 2 * dp + 32) bytes for s = min(nq, 16384) fallback / collect slots
 * (fb_cap = max(512, pow2ceil(2k + 64))): ~60 MB at nq = 4096, k = 5 and at most
 * ~256 MB + nq * 16 KB at k = 200.  Uncertified queries beyond the 16384
 * slots are answered by the block-per-query fp64 scan. */
int nrk_knn_flat_workspace(int64_t nq, int64_t nb, int32_t d, int32_t k, size_t* ws_bytes);

/* Exact top-k: bf16 MFMA screening with per-chunk candidate lists, fp64
 * rescoring of the survivors, a certificate per query, and an exact fp64 scan
 * for any query the certificate does not cover.
 *   xq [nq][d] f32; xb [nb][d] f32 (used for the exact rescoring)
 *   D  [nq][k] f32 (IP: inner product, L2: squared distance)
 *   I  [nq][k] int64 (global id = local row + id_offset; -1 padding)
 *   S  [nq][k] f64 exact scores (optional, may be NULL): the values D rounds;
 *      used by the multi-shard merge so ties break exactly as on one device.
 *   n_fallback (optional, device int32[2], diagnostic): [0] queries the
 *      screening certificate did not cover (answered by the collect pass: one
 *      more bf16 screen over the corpus for these queries only, keeping every
 *      item within the error bound of the merge's exact k-th, then exact
 *      rescoring); [1] of those, queries whose collect buffer overflowed and
 *      that the fp64 corpus scan answered.
 *   stage_events (optional, host array of NRK_KNN_STAGES+1 hipEvent_t created by
 *      the caller): recorded on `stream` before each stage and after the last,
 *      so a benchmark can time the screening kernel alone.  NULL in production. */
#define NRK_KNN_STAGES 4 /* query_prepare, screen, merge_rescore, exact fallback */
int nrk_knn_flat(const float* xq, int64_t nq, const float* xb, const uint16_t* xb_bf16,
                 const float* xb_meta, const float* stats, int64_t nb, int32_t d,
                 int32_t k, int32_t metric, float* D, int64_t* I, double* S,
                 int64_t id_offset, int32_t* n_fallback, void* ws, size_t ws_bytes,
                 void* const* stage_events, void* stream);

/* Exact brute force (fp64, sequential-d order), no screening.  Used directly
 * for small corpora (e.g. the 300-centroid coarse search, Retrieval.py:25-32)
 * and as the certificate fallback. */
int nrk_knn_exact(const float* xq, int64_t nq, const float* xb, int64_t nb, int32_t d,
                  int32_t k, int32_t metric, float* D, int64_t* I, double* S,
                  int64_t id_offset, void* stream);

/* Merge per-shard top-k lists (multi-GPU corpus sharding; no reference
 * counterpart — the reference is single-device).
 *   S_parts [nparts][nq][k] f64 exact scores, I_parts [nparts][nq][k] int64
 *   D [nq][k] f32, I [nq][k] int64, S [nq][k] f64 (optional)
 * Order: IP descending / L2 ascending on the f64 score, then lower id. */
int nrk_topk_merge(const double* S_parts, const int64_t* I_parts, int32_t nparts, int64_t nq,
                   int32_t k, int32_t metric, float* D, int64_t* I, double* S, void* stream);

/* ------------------------------------------------------------------------- *
 * DIN local-activation unit + weighted-sum pool — replaces
 * AttentionLayer.forward (DIN.py:103-111) and its autograd backward, fused
 * with the history gather of TrainDataset.__getitem__ (DIN.py:84-86).
 *
 * Keys come from one of two sources:
 *   dense:  keys [B][L][d] (dtype), hist_ids == NULL  (AttentionLayer(query, keys))
 *   ids:    table [N][d] (dtype) + hist_ids [B][L] int32; id < 0 means an
 *           all-zero padding row, as DIN.py:84-86 zero-fills the tail.
 * The query enters through U = query @ W1[:, :d]^T + b1 ([B][A] f32), computed
 * by the caller (a plain GEMM); W1k = W1[:, d:] is passed in `dtype`.
 * Softmax runs over all L slots, padding included (DIN.py:108, no mask).
 * ------------------------------------------------------------------------- */
int nrk_din_attn_fwd(const void* keys, const int32_t* hist_ids, int64_t n_table, int32_t dtype,
                     const float* U, const void* W1k, const float* w2, float b2,
                     int32_t B, int32_t L, int32_t d, int32_t A,
                     float* pooled, float* alpha, void* stream);

/* Backward of the pool w.r.t. the attention parameters (the reference's
 * embeddings are frozen inputs, so no key/query gradient is produced):
 *   in : dpooled [B][d] f32, alpha [B][L] f32 (from fwd)
 *   out: dU [B][A] f32 (= sum_j dz_j; caller forms dW1q = dU^T q, db1 = sum dU)
 *        dW1k [A][d] f32, dw2 [A] f32, db2 [1] f32 — OVERWRITTEN (not accumulated).
 *   ws  : f32 workspace of nrk_din_attn_bwd_workspace() bytes (per-workgroup slabs). */
int nrk_din_attn_bwd_workspace(int32_t B, int32_t d, int32_t A, size_t* ws_bytes);
int nrk_din_attn_bwd(const void* keys, const int32_t* hist_ids, int64_t n_table, int32_t dtype,
                     const float* U, const void* W1k, const float* w2, float b2,
                     int32_t B, int32_t L, int32_t d, int32_t A,
                     const float* dpooled, const float* alpha,
                     float* dU, float* dW1k, float* dw2, float* db2,
                     void* ws, size_t ws_bytes, void* stream);

/* The same backward with the query half folded in (train step, id form, bf16
 * table, d in {64, 128}, or 256 with dU == NULL — L 65..128 there as two
 * half-samples per sample after a softmax-term pass): also accumulates dW1q = sum_b dU[b] q[b]^T and
 * db1 = sum_b dU[b] per workgroup, and WRITES the layer's parameter gradients
 * straight into the model's tensors: gW1 [A][2d] = [dW1q | dW1k], gb1 [A],
 * gw2 [A], gb2 [1] (DIN.py:146 loss.backward() for attn.attn.{0,2}).
 *   q [B][d] f32 (the query rows), dU [B][A] optional (NULL: not written).
 *   pooled [B][d] f32: the forward's pooled rows, optional (d = 256, L > 64: the
 *   softmax term sum_l alpha_l dalpha_l is read off them as dpooled . pooled;
 *   NULL: formed from the key rows, one more pass over them).
 *   norm_part (optional, n_flat): as nrk_din_attn_bwd_params_head — gW1 .. gb2 are
 *   the start of the model's flat gradient of n_flat floats, and the reduction
 *   also writes the per-64-block squared-norm partials nrk_clip_adam_partials
 *   reads (NULL: not written).
 *   ws as nrk_din_attn_bwd_workspace(B, d, A). */
int nrk_din_attn_bwd_params(const void* table, const int32_t* hist_ids, int64_t n_table, int32_t dtype,
                            const float* q, const float* U, const void* W1k, const float* w2,
                            int32_t B, int32_t L, int32_t d, int32_t A,
                            const float* dpooled, const float* alpha, const float* pooled,
                            float* gW1, float* gb1, float* gw2, float* gb2, float* dU,
                            int64_t n_flat, double* norm_part,
                            void* ws, size_t ws_bytes, void* stream);

/* The same backward, forming dpooled itself from the train-mode head's state
 * instead of reading it (the fused train step: one launch fewer, no dpooled
 * round trip): dpooled = BN0-backward of da1 W1[:, d:] for the pooled columns,
 * from the forward's pooled [B][d] f32, the head's parameters (fc.0 weight,
 * fc.1 weight) and the workspace nrk_din_head_train left with dpooled == NULL
 * (F = 32).  d in {64, 128}, L <= 64, L * d >= 4096 (the 8-wave backward). */
int nrk_din_attn_bwd_params_head(const void* table, const int32_t* hist_ids, int64_t n_table, int32_t dtype,
                                 const float* q, const float* U, const void* W1k, const float* w2,
                                 int32_t B, int32_t L, int32_t d, int32_t A, const float* pooled, const float* alpha,
                                 int32_t F, const struct nrk_din_head_params_s* hp, const void* head_ws,
                                 size_t head_ws_bytes, float* gW1, float* gb1, float* gw2, float* gb2,
                                 int64_t n_flat, double* norm_part, void* ws, size_t ws_bytes, void* stream);
/*   norm_part (optional, device f64 [ceil(n_flat / 64)]): gW1 is then the base of
 *   the model's flat gradient buffer of n_flat floats, [gW1 | gb1 | gw2 | gb2]
 *   first and the head's (already final) gradients after; entry i receives the
 *   sum of squares of flat entries [64 i, 64 i + 64), for nrk_clip_adam_partials. */

/* One train batch from a device-resident click log (replaces TrainDataset.
 * __getitem__'s CPU gather, DIN.py:81-92, and the query GEMM of DIN.py:105-106):
 *   idx [B] int64 rows of the log; hist_all [n_rows][L] int32, tgt_all [n_rows]
 *   int32, lab_all [n_rows] f32; table [N][d] bf16; W1 [A][2d] f32, b1 [A] f32.
 * Out: hist [B][L] int32, q [B][d] f32 (= table[target], id < 0 -> zeros),
 *   y [B] f32, U [B][A] f32 = q W1[:, :d]^T + b1 (products exact in f32),
 *   W1k_bf16 [A][d] = bf16(W1[:, d:]).  Rows outside [0, n_rows) give an
 *   empty history, a zero query and label 0.  d in {64, 128, 256}. */
int nrk_din_batch(const int64_t* idx, int32_t B, const int32_t* hist_all, const int32_t* tgt_all,
                  const float* lab_all, int64_t n_rows, int32_t L, const void* table, int64_t n_table,
                  int32_t dtype, int32_t d, const float* W1, const float* b1, int32_t A, int32_t* hist,
                  float* q, float* y, float* U, void* W1k_bf16, void* stream);
/* W1 == NULL in nrk_din_batch: the gathers only (hist, q, y; b1 / U / W1k_bf16
 * unused), e.g. for the rows of K steps at once; each step then forms
 *   U [B][A] = q W1[:, :d]^T + b1 and W1k_bf16 from the gathered q [B][d] f32: */
int nrk_din_batch_u(const float* q, int32_t B, int32_t d, const float* W1, const float* b1, int32_t A,
                    float* U, void* W1k_bf16, void* stream);

/* DIN evaluate() for re-ranking, fused (DIN.py:155-189 minus the loss / NDCG
 * bookkeeping; Retrieval.py:28-34 -> finialize_retrieval.py -> DIN.py): the
 * eval-mode logits of every candidate of every user, each candidate attending
 * over its user's history (`his.expand(C, -1, -1)`, DIN.py:166-173), in ONE
 * launch that writes only the logits.
 *   table [N][d] bf16 item embeddings (f32: the projected form below); hist [nU][L] int32 history rows (-1 or
 *   >= n_table = a zero padding slot: DIN.py:84-86, 108 softmaxes over all L);
 *   user u's candidates: cand[cand_off[u] .. cand_off[u] + cand_len[u]) int32
 *   rows, then extra[u] when extra != NULL (the appended ground truth of
 *   finialize_retrieval.py:11-12; < 0 = a padded slot); rows outside [0, N)
 *   get logit -inf.  Logits of user u: out[out_off[u] + c], c < cand_len[u]
 *   (+ 1 with extra).  Candidate lists may be shared (the flow passes every
 *   user of a cluster the same offset).
 *   params: the model with its three eval-mode BatchNorms folded into the
 *   Linears after them and every weight split into bf16 hi + lo
 *   (newsrecommend_amd.pipeline.rerank_params).
 * d in {64, 128, 256}, A and F in {32, 64, 96, 128}, L <= 64.  ws: >= 1024 B
 * (nrk_din_rerank_workspace: the user queue and, for the projected form,
 * sgn(w2) per projection column), reset by the call (graph-capturable). */
typedef struct nrk_din_rerank_params_s {
  const void *W1q_hi, *W1q_lo;  /* bf16 [A][d]: W1[:, :d] (attention query half) */
  const void *W1k_hi, *W1k_lo;  /* bf16 [A][d]: W1[:, d:] (key half) */
  const float* b1;              /* [A] */
  const float* w2;              /* [A] (b2 cancels in the softmax) */
  const void *H1q_hi, *H1q_lo;  /* bf16 [F][d]: fc.1 with BN0 folded, query half */
  const void *H1p_hi, *H1p_lo;  /* bf16 [F][d]: pooled half */
  const float* c1;              /* [F] */
  const void *H2_hi, *H2_lo;    /* bf16 [F/2][F]: fc.5 with BN1 folded */
  const float* c2;              /* [F/2] */
  const float* h3;              /* [F/2]: fc.9 with BN2 folded */
  float c3;
} nrk_din_rerank_params;
int nrk_din_rerank_workspace(size_t* ws_bytes);
int nrk_din_rerank(const void* table, int64_t n_table, int32_t dtype, const int32_t* hist, int32_t nU, int32_t L,
                   const int32_t* cand, const int64_t* cand_off, const int32_t* cand_len, const int32_t* extra,
                   const int64_t* out_off, float* out, int32_t d, int32_t A, int32_t F,
                   const nrk_din_rerank_params* params, void* ws, size_t ws_bytes, void* stream);
/* Projected form (shared candidate lists, and every f32 table).  The
 * candidate half of the attention MLP and of the head's first Linear depends
 * on the item alone, and the key half on the history row alone, so rows are
 * projected once:
 *   nrk_din_rerank_project: out [n][A + F] f32 = [ U'(q) = w2 . (W1q q + b1)
 *   in the kernel's slice order (A) | Q1(q) = H1q q (F) ], q = table[rows[i]];
 *   nrk_din_rerank_project_hist: out [n][A + F] f32 = [ P'(k) = w2 . (W1k k)
 *   (slice order) | R(k) = H1p k ], k = table[rows[i]] (rows = hist [nU][L]
 *   flattened, so out is per history slot);
 * a zero row where rows[i] is outside [0, N).  table: bf16 (the MFMA sequence
 * nrk_din_rerank applies to a row) or f32 (each
 * element split into bf16 hi + lo, three products: the reference's fp32
 * embeddings, embedding_generate.py:119-122 / DIN.py:45-56, to ~2^-16).
 * nrk_din_rerank_projected then stages projections instead of rows and never
 * reads the table (any dtype): cand_proj [.][A + F] parallel to cand,
 * extra_proj [nU][A + F] (required when extra != NULL), hist_proj
 * [nU * L][A + F] (required).  cand / extra / hist still decide validity.
 * For F <= 64 it runs one wave per 32 candidates (din_rerank_lane.hip; its
 * arithmetic order differs from nrk_din_rerank's, both within 1e-4 of the
 * reference), for F in {96, 128} the per-chunk kernel of nrk_din_rerank.
 * Histories of 65..128 slots (L <= nrk_din_rerank_max_history = 128 for every
 * (A, F)) take the lane kernel's 128-row form; where [P' | R^T] and H2 do not
 * fit its LDS together ((A, F) = (96, 64), (128, 64), F in {96, 128}) it stages
 * P' only and reads R and H2 from global memory. */
int nrk_din_rerank_project(const void* table, int64_t n_table, int32_t dtype, const int32_t* rows, int64_t n,
                           int32_t d, int32_t A, int32_t F, const nrk_din_rerank_params* params, float* out,
                           void* stream);
int nrk_din_rerank_project_hist(const void* table, int64_t n_table, int32_t dtype, const int32_t* rows, int64_t n,
                                int32_t d, int32_t A, int32_t F, const nrk_din_rerank_params* params, float* out,
                                void* stream);
/* The longest history L nrk_din_rerank_projected takes for (A, F): 128 where
 * the one-wave-per-32-candidates kernel's 128-row form fits the LDS (F <= 64
 * and A * F not (96, 64) / (128, 64)), else 64 (the reference's max_history
 * reaches 128, DIN.py:207). */
int nrk_din_rerank_max_history(int32_t A, int32_t F, int32_t* max_l);
int nrk_din_rerank_projected(const void* table, int64_t n_table, int32_t dtype, const int32_t* hist, int32_t nU,
                             int32_t L, const int32_t* cand, const int64_t* cand_off, const int32_t* cand_len,
                             const int32_t* extra, const int64_t* out_off, float* out, int32_t d, int32_t A,
                             int32_t F, const nrk_din_rerank_params* params, const float* cand_proj,
                             const float* extra_proj, const float* hist_proj, void* ws, size_t ws_bytes,
                             void* stream);
/* evaluate()'s per-user tail over re-rank logits (DIN.py:176-189): user u's
 * logits are [seg_off[u], seg_off[u+1]); pos[u] the index of its positive
 * (-1: none); prob = sigmoid(logits) as the caller computes it.  Writes the f64
 * BCE-with-logits sum over the finite logits (label 1 at pos[u]), their count,
 * and before[u] = #{j : prob_j > prob_pos or (prob_j == prob_pos and j < pos)}
 * (NDCG rank - 1, the stable-sort tie rule).  One block per user. */
int nrk_rerank_user_stats(const float* logits, const float* prob, const int64_t* seg_off, const int64_t* pos,
                          int32_t nU, double* loss_sum, int64_t* nval, int64_t* before, void* stream);

/* ------------------------------------------------------ corpus producer --
 * ArticleEmbeddingModel in eval mode for a whole corpus
 * (embedding_generate.py:51-65 forward, :109-121 inference()):
 *   out [n][out_dim] = relu(x W1^T + b1) W2^T + b2,
 * x [n][ldx] f32 (in_dim <= 256 columns used: the reference's 253 features),
 * W1 [hidden][in_dim], b1 [hidden] (fc.0), W2 [out_dim][hidden], b2 [out_dim]
 * (fc.4 with the eval BatchNorm fc.3 folded in by the caller:
 * W2 = fc.4.weight diag(s), b2 = fc.4.bias + fc.4.weight t).  hidden a
 * multiple of 128, out_dim 256.  The hidden activations never leave the chip;
 * products are fp32-exact (each operand split into three bf16 planes, six
 * MFMA products).  ws: nrk_embed_workspace bytes (the weights' planes). */
int nrk_embed_workspace(int32_t in_dim, int32_t hidden, int32_t out_dim, size_t* ws_bytes);
int nrk_embed(const float* x, int64_t n, int64_t ldx, int32_t in_dim, const float* W1, const float* b1,
              int32_t hidden, const float* W2, const float* b2, int32_t out_dim, float* out, void* ws,
              size_t ws_bytes, void* stream);

/* ------------------------------------------------------ inverted lists --
 * faiss Clustering / IndexIVFFlat building blocks (Retrieval.py:11-23).
 *
 * Stable grouping of ids by list (counting sort; ids ascending inside each
 * list, i.e. faiss's insertion order):
 *   assign [n] int64 list of each id (must be in [0, nlist); *n_bad counts violations)
 *   list_off [nlist+1] int64 (out), pos2id [n] int64 (out), pos2list [n] int32 (out)
 * Replaces `cluster_to_articles[i] = ids[assign == i]` (Retrieval.py:22-23)
 * and the list append of IndexIVFFlat.add. */
int nrk_group_by_list_workspace(int64_t n, int32_t nlist, size_t* ws_bytes);
int nrk_group_by_list(const int64_t* assign, int64_t n, int32_t nlist, int64_t* list_off,
                      int64_t* pos2id, int32_t* pos2list, int32_t* n_bad, void* ws,
                      size_t ws_bytes, void* stream);

/* List-major copy of the screening rows of nrk_flat_prepare:
 * xbh_ivf[pos] = xb_bf16[pos2id[pos]] (padded dim), meta_ivf likewise. */
int nrk_ivf_pack(const int64_t* pos2id, int64_t n, int32_t d, const uint16_t* xb_bf16,
                 const float* xb_meta, uint16_t* xbh_ivf, float* meta_ivf, void* stream);

/* k-means update step (faiss Clustering.train, Retrieval.py:14-18):
 * centroids[c] = (sum over the members of c, fp64, in id order) / |c| for
 * every non-empty list of (list_off, pos2id); empty clusters are left as they
 * are (the caller splits them, as faiss does). */
int nrk_kmeans_update(const float* x, int32_t d, const int64_t* list_off, const int64_t* pos2id,
                      int32_t k, float* centroids, void* stream);

/* IVF-Flat search (faiss IndexIVFFlat.search; BASELINE configs[3]).
 *   probe [nq][nprobe] int64: the coarse quantizer's lists per query (-1: none)
 *   xb [n][d] f32 in id order (exact rescoring); xbh_ivf / meta_ivf list-major
 *   (nrk_ivf_pack); stats from nrk_flat_prepare over the same rows;
 *   list_off / pos2id / pos2list from nrk_group_by_list; max_list = largest list.
 * Result: the exact top-k (same order and ties as nrk_knn_flat) among the
 * items of the probed lists.  Outputs and stage_events as nrk_knn_flat
 * (stage 0 = query prepare + grouping by list); n_fallback[0] = queries whose
 * collect buffer overflowed (or that had fewer than k seeds), answered by the
 * tiled fp64 scan of their probed lists; n_fallback[1] = of those, the queries
 * that scan's candidate buffer could not hold either, answered by the
 * block-per-query fp64 scan (the slow path). */
int nrk_ivf_search_workspace(int64_t nq, int32_t nprobe, int32_t nlist, int64_t max_list,
                             int32_t d, int32_t k, size_t* ws_bytes);
int nrk_ivf_search(const float* xq, int64_t nq, const int64_t* probe, int32_t nprobe,
                   const float* xb, const uint16_t* xbh_ivf, const float* meta_ivf,
                   const float* stats, const int64_t* list_off, const int64_t* pos2id,
                   const int32_t* pos2list, int32_t nlist, int64_t n, int64_t max_list,
                   int32_t d, int32_t k, int32_t metric, float* D, int64_t* I, double* S,
                   int64_t id_offset, int32_t* n_fallback, void* ws, size_t ws_bytes,
                   void* const* stage_events, void* stream);
/* Guard word of the last nrk_ivf_search on workspace `ws` -> device int32
 * `guard` (async on `stream`).  Every index the search reads back from its own
 * workspace (candidate and seed positions, query slots, probed lists) is range
 * checked where it addresses memory; a violation sets a bit and skips the
 * access instead of faulting: 1 seed position, 2 candidate position, 4 collect
 * query row, 8 candidate count, 16 fallback query, 32 probed list, 64 gathered
 * (query, probe) pair, 128 collected position.  0 = all in range (the result
 * is valid); nonzero = a broken invariant, the result must not be used.
 * (Python: IndexIVFFlat.search_device(check=True) raises NrkError.) */
int nrk_ivf_search_status(const void* ws, size_t ws_bytes, int32_t* guard, void* stream);

/* ------------------------------------------------------------ DIN head --
 * The MLP head of DIN in train mode, forward and backward (DIN.py:117-123,
 * 130-133 with BCEWithLogitsLoss(mean), DIN.py:143-148):
 *   x = [q | pooled] (B x 2d) -> BN0 -> Linear(2d,F) -> ReLU -> Dropout(p)
 *     -> BN1 -> Linear(F,F/2) -> ReLU -> Dropout(p) -> BN2 -> Linear(F/2,1)
 * Parameters in nn.Module order (fc.0 ... fc.9); running statistics and
 * num_batches_tracked are updated as torch's train-mode BatchNorm1d does;
 * gradients are WRITTEN (not accumulated).  Dropout masks are a counter-based
 * hash of (seed, *step, layer, row, col).  Outputs: logits [B], loss [1]
 * (mean BCE), dpooled [B][ld] (the gradient w.r.t. pooled, the attention
 * backward's input; columns d..ld-1 zeroed; may be NULL with F = 32, then
 * nrk_din_attn_bwd_params_head forms it).  B must be a multiple of 32,
 * 2d <= 512, F even <= 64. */
typedef struct nrk_din_head_params_s {
  const float *bn0_w, *bn0_b, *fc1_w, *fc1_b, *bn1_w, *bn1_b, *fc2_w, *fc2_b, *bn2_w, *bn2_b, *fc3_w, *fc3_b;
  float *bn0_rm, *bn0_rv, *bn1_rm, *bn1_rv, *bn2_rm, *bn2_rv;
  int64_t *bn0_nb, *bn1_nb, *bn2_nb;
  float *g_bn0_w, *g_bn0_b, *g_fc1_w, *g_fc1_b, *g_bn1_w, *g_bn1_b, *g_fc2_w, *g_fc2_b, *g_bn2_w, *g_bn2_b,
      *g_fc3_w, *g_fc3_b;
} nrk_din_head_params;
int nrk_din_head_workspace(int32_t B, int32_t d, int32_t F, size_t* ws_bytes);
/* Views into a head workspace after nrk_din_head_train (F = 32 path): BN0's
 * {mean [2d], invstd [2d]}, its backward sums {sum dh0 [2d], sum dh0 xhat0
 * [2d]} (f64) and da1 [B][F] (the gradient at fc.1's output). */
int nrk_din_head_ws_views(int32_t B, int32_t d, int32_t F, const void* ws, size_t ws_bytes,
                          const float** stat0, const double** sum5, const float** da1);
int nrk_din_head_train(const float* q, const float* pooled, int64_t ld_pooled, const float* labels,
                       int32_t B, int32_t d, int32_t F, float momentum, float eps, float p_drop,
                       uint64_t seed, const float* step, const nrk_din_head_params* params,
                       float* logits, float* loss, float* dpooled, void* ws, size_t ws_bytes,
                       void* stream);

/* clip_grad_norm_(max_norm) + torch.optim.Adam (L2 weight decay) over one
 * flat parameter buffer (DIN.py:150-151): *step (device f32) is incremented,
 * grads are scaled in place by the clip coefficient, exp_avg / exp_avg_sq /
 * params updated with torch's capturable-Adam formulas.  lr_dev (device f32,
 * optional) overrides lr when non-null, so ReduceLROnPlateau (DIN.py:246,254)
 * can change the rate of a captured step between graph replays.  The
 * workspace must be ZEROED once before the first call (n <= 131072 runs one
 * launch whose completion ticket lives there and is left zero); calls sharing
 * one workspace must be stream-ordered. */
int nrk_clip_adam_workspace(int64_t n, size_t* ws_bytes);
int nrk_clip_adam(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                  float* step, float lr, const float* lr_dev, float beta1, float beta2, float eps, float weight_decay,
                  float max_norm, void* ws, size_t ws_bytes, void* stream);

/* The same clip_grad_norm_ + Adam with the squared gradient norm given as f64
 * partials (norm_part [n_part], e.g. from nrk_din_attn_bwd_params_head): no
 * pass over all gradients per block; each block scales and updates only its
 * own entries.  Workspace as nrk_clip_adam (zeroed once; its ticket). */
int nrk_clip_adam_partials(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                           float* step, float lr, const float* lr_dev, float beta1, float beta2, float eps,
                           float weight_decay, float max_norm, const double* norm_part, int32_t n_part,
                           void* ws, size_t ws_bytes, void* stream);

/* Row gather (table [N][d] dtype -> out [n][d] f32), id < 0 -> zeros.
 * Replaces the per-sample dict lookups of DIN.py:47-50,83 (target and
 * candidate embeddings). */
int nrk_gather_rows(const void* table, int64_t n_table, int32_t dtype, const int32_t* ids,
                    int64_t n, int32_t d, float* out, void* stream);

/* ------------------------------------------------------------------------- *
 * Typed click logs (HOST memory, no stream): the training-row builders.
 * A click log is CSR: user u's clicks are click_rows[click_off[u] ..
 * click_off[u+1]) (oldest -> newest), as row indices into the article list the
 * reference draws negatives from (list(article_emb.keys()) order).
 * rng_state [625] is Python's random.getstate()[1] (624 Mersenne Twister words
 * + position), read and written back advanced: the negatives are the ones
 * `random.choice` draws in the reference loop, so the rows are identical.
 * A user whose clicks cover every item returns NRK_EINVAL (the reference's
 * rejection loop would not terminate). */

/* Replaces TrainDataset.__init__ (DIN.py:66-76): per user with >= 2 clicks and
 * click i >= 1, a positive row (target clicks[i], label 1) then a negative row
 * (label 0), both with history clicks[:i][-max_history:].
 *   n_samples must be 2 * sum(max(len_u - 1, 0));
 *   user_idx, target_rows int32 [n_samples], labels f32 [n_samples];
 *   hist_rows int32 [n_samples][max_history] (-1 padded) or NULL. */
int nrk_train_samples(const int64_t* click_off, int64_t n_users, const int32_t* click_rows,
                      int64_t n_items, int32_t max_history, uint32_t* rng_state, int64_t n_samples,
                      int32_t* user_idx, int32_t* target_rows, float* labels, int32_t* hist_rows);

/* Replaces ArticleTripletDataset.__init__ (embedding_generate.py:25-39): per
 * user with >= 2 clicks and every pair i < j, (anchor clicks[i], positive
 * clicks[j], a random never-clicked negative).
 *   n_triplets must be sum(len_u * (len_u - 1) / 2) over users with >= 2 clicks;
 *   triplets int32 [n_triplets][3]. */
int nrk_triplet_samples(const int64_t* click_off, int64_t n_users, const int32_t* click_rows,
                        int64_t n_items, uint32_t* rng_state, int64_t n_triplets, int32_t* triplets);

#ifdef __cplusplus
}
#endif

#endif /* NRK_H */
