"""oracle/ivf_oracle.py — TEST INFRASTRUCTURE ONLY (checker / CPU baseline,
never the product).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module.

CPU restatement of the index-building half of the retrieval path
(Retrieval.py:11-23) and of faiss IndexIVFFlat search (BASELINE configs[3]).
faiss is an external, unvendored, unpinned dependency that is not importable
here, so these follow faiss's published algorithms with the
deterministic choices DESIGN.md records, and are "parity unpinned" against
faiss itself.  The GPU path must equal THIS restatement bit for bit.

  group_by_list  cluster_to_articles[i] = ids[assign == i]   (Retrieval.py:22-23)
                 -> list_off, pos2id (ids ascending inside a list)
  kmeans         faiss Clustering.train (Retrieval.py:12-18):
                 - n > k * max_points_per_centroid: subsample
                   x[rng(seed).permutation(n)[:k*mppc]]
                 - init: centroids = x_s[rng(seed + 1).permutation(n_s)[:k]]
                 - niter x { assign = exact nearest centroid (fp64 sequential-d,
                   ties -> lower id; faiss uses whatever index is passed — the
                   GPU path is exact);  c = fp64 sum of members in id order /
                   count -> f32;  split empty clusters (faiss split_clusters:
                   pick cluster j with probability (|j|-1)/(n-k), copy it with
                   a +-1/1024 symmetric perturbation, halve the counts;
                   rng(1234) per call) }
  ivf_search     coarse top-nprobe over the centroids with the quantizer's
                 metric, then exact top-k over the union of the probed lists
                 (fp64 scores, ties -> lower id; -1 padding).
"""
from __future__ import annotations

import numpy as np

from . import knn_oracle as ko

EPS = 1.0 / 1024.0


def group_by_list(assign, nlist):
    """-> list_off (nlist+1,) int64, pos2id (n,) int64 (stable: ids ascending per list)."""
    assign = np.asarray(assign, np.int64)
    order = np.argsort(assign, kind="stable")
    sizes = np.bincount(assign, minlength=nlist)
    off = np.zeros(nlist + 1, np.int64)
    np.cumsum(sizes, out=off[1:])
    return off, order.astype(np.int64)


def assign_nearest(x, centroids, metric=ko.METRIC_L2):
    """Exact 1-NN over the centroids (fp64 sequential-d): -> (labels, distances f64)."""
    _, I, S = ko.exact_search(x, centroids, 1, metric)
    return I[:, 0], S[:, 0]


def update_centroids(x, labels, centroids):
    """fp64 sequential sum of each cluster's members in id order / count -> f32;
    empty clusters keep their previous centroid.  Returns (centroids, counts)."""
    k = centroids.shape[0]
    off, pos2id = group_by_list(labels, k)
    out = centroids.copy()
    for c in range(k):
        lo, hi = off[c], off[c + 1]
        if hi == lo:
            continue
        xm = x[pos2id[lo:hi]].astype(np.float64)
        s = np.cumsum(xm, axis=0)[-1]  # sequential (not pairwise) summation
        out[c] = (s / float(hi - lo)).astype(np.float32)
    return out, np.diff(off)


def split_clusters(centroids, counts, n):
    """faiss split_clusters restated (rng(1234) per call; float32 arithmetic)."""
    k, d = centroids.shape
    rng = np.random.default_rng(1234)
    hassign = counts.astype(np.float64).copy()
    nsplit = 0
    for ci in range(k):
        if hassign[ci] != 0:
            continue
        cj = 0
        while True:
            p = (hassign[cj] - 1.0) / float(n - k)
            r = rng.random()
            if r < p:
                break
            cj = (cj + 1) % k
        centroids[ci] = centroids[cj]
        up = np.float32(1 + EPS)
        dn = np.float32(1 - EPS)
        even = (np.arange(d) % 2) == 0
        centroids[ci] = np.where(even, centroids[ci] * up, centroids[ci] * dn).astype(np.float32)
        centroids[cj] = np.where(even, centroids[cj] * dn, centroids[cj] * up).astype(np.float32)
        hassign[ci] = np.floor(hassign[cj] / 2)
        hassign[cj] -= hassign[ci]
        nsplit += 1
    return centroids, nsplit


def subsample(x, k, max_points_per_centroid, seed):
    n = x.shape[0]
    if n > k * max_points_per_centroid:
        perm = np.random.default_rng(seed).permutation(n)[: k * max_points_per_centroid]
        return np.ascontiguousarray(x[np.sort(perm)])
    return x


def kmeans(x, k, niter=25, seed=1234, max_points_per_centroid=256, metric=ko.METRIC_L2, spherical=False):
    """-> (centroids (k, d) f32, obj list).  See the module docstring."""
    x = np.ascontiguousarray(x, np.float32)
    xs = subsample(x, k, max_points_per_centroid, seed)
    n = xs.shape[0]
    init = np.random.default_rng(seed + 1).permutation(n)[:k]
    cent = np.ascontiguousarray(xs[init], np.float32)
    obj = []
    for _ in range(niter):
        labels, dist = assign_nearest(xs, cent, metric)
        obj.append(float(dist.sum()))
        cent, counts = update_centroids(xs, labels, cent)
        cent, _ = split_clusters(cent, counts, n)
        if spherical:
            nrm = np.sqrt((cent.astype(np.float64) ** 2).sum(1, keepdims=True))
            cent = (cent / np.maximum(nrm, 1e-20)).astype(np.float32)
    return cent, obj


def ivf_search(xq, xb, centroids, assign, nprobe, k, metric, quantizer_metric=ko.METRIC_L2):
    """IndexIVFFlat.search restated: exact top-k among the probed lists' items.
    assign: list of every corpus row.  -> D f32, I int64, S f64."""
    xq = np.ascontiguousarray(xq, np.float32)
    xb = np.ascontiguousarray(xb, np.float32)
    nq = xq.shape[0]
    nlist = centroids.shape[0]
    _, probe, _ = ko.exact_search(xq, centroids, min(nprobe, nlist), quantizer_metric)
    off, pos2id = group_by_list(assign, nlist)
    D = np.empty((nq, k), np.float32)
    I = np.full((nq, k), -1, np.int64)
    S = np.empty((nq, k), np.float64)
    for q in range(nq):
        ids = np.concatenate([pos2id[off[l]:off[l + 1]] for l in probe[q] if l >= 0] or [np.zeros(0, np.int64)])
        ids = np.sort(ids)
        if ids.size == 0:
            D[q] = np.finfo(np.float32).max if metric == ko.METRIC_L2 else -np.finfo(np.float32).max
            S[q] = np.finfo(np.float64).max if metric == ko.METRIC_L2 else -np.finfo(np.float64).max
            continue
        d_, i_, s_ = ko.exact_search(xq[q:q + 1], xb[ids], k, metric)
        D[q], S[q] = d_[0], s_[0]
        I[q] = np.where(i_[0] >= 0, ids[np.maximum(i_[0], 0)], -1)
    return D, I, S, probe
