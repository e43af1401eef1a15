"""oracle/cpu_baselines.py — TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline
leg and tests/; never the product).

faiss-cpu is not installed here or on the GPU box, so the
CPU baselines BASELINE.md asks for are restated with the same algorithms on
all host cores (torch CPU kernels, `torch.set_num_threads(n)`), labelled
kind "port" in the bench records:

  flat_search    faiss IndexFlatIP / IndexFlatL2 .search for nq >= 20
                 (faiss exhaustive_*_blas): fp32 sgemm of query blocks x
                 corpus blocks, ||x||^2 - 2<q, x> for L2 (the query norm does
                 not change the ranking and is added back), a running
                 per-query top-k over the blocks.
  ivf_search     faiss IndexIVFFlat .search: coarse top-nprobe over the
                 centroids, then every probed inverted list scanned IN PLACE
                 (list-major storage, as faiss's ArrayInvertedLists keeps its
                 codes), batched per list over the queries that probe it
                 (one sgemm per list instead of faiss's per-query SIMD loop),
                 with a running per-query top-k.
Results are approximate-rank-equal to the exact oracle (fp32 arithmetic);
they are timed, not used as a checker.
"""
from __future__ import annotations

import numpy as np
import torch

METRIC_IP, METRIC_L2 = 0, 1


def _merge(best_s, best_i, s, i, k, largest):
    cs = torch.cat([best_s, s], 1)
    ci = torch.cat([best_i, i], 1)
    v, p = torch.topk(cs, k, dim=1, largest=largest, sorted=True)
    return v, torch.gather(ci, 1, p)


def flat_search(xq: torch.Tensor, xb: torch.Tensor, k: int, metric: int, block: int = 1 << 16,
                xb_norms: torch.Tensor | None = None):
    """CPU fp32 flat search -> (D (nq, k), I (nq, k)).  xq, xb: CPU float32."""
    nq = xq.shape[0]
    largest = metric == METRIC_IP
    fill = -np.inf if largest else np.inf
    best_s = torch.full((nq, k), fill, dtype=torch.float32)
    best_i = torch.full((nq, k), -1, dtype=torch.int64)
    if metric == METRIC_L2 and xb_norms is None:
        xb_norms = (xb * xb).sum(1)
    for j0 in range(0, xb.shape[0], block):
        blk = xb[j0:j0 + block]
        ip = xq @ blk.t()
        s = ip if largest else xb_norms[j0:j0 + block][None, :] - 2.0 * ip
        kk = min(k, s.shape[1])
        v, p = torch.topk(s, kk, dim=1, largest=largest, sorted=False)
        best_s, best_i = _merge(best_s, best_i, v, p + j0, k, largest)
    if metric == METRIC_L2:
        best_s = best_s + (xq * xq).sum(1, keepdim=True)
    return best_s, best_i


class IvfLists:
    """List-major copy of the corpus (faiss's inverted lists): rows of list l
    are xl[off[l]:off[l+1]] with ids pos2id[off[l]:off[l+1]]."""

    def __init__(self, xb: np.ndarray, assign: np.ndarray, centroids: np.ndarray):
        nlist = centroids.shape[0]
        order = np.argsort(assign, kind="stable")
        self.off = np.zeros(nlist + 1, np.int64)
        np.cumsum(np.bincount(assign, minlength=nlist), out=self.off[1:])
        self.pos2id = torch.from_numpy(order.astype(np.int64))
        self.xl = torch.from_numpy(np.ascontiguousarray(xb[order], np.float32))
        self.norms = (self.xl * self.xl).sum(1)
        self.cent = torch.from_numpy(np.ascontiguousarray(centroids, np.float32))
        self.nlist = nlist


def ivf_search(xq: torch.Tensor, lists: IvfLists, nprobe: int, k: int, metric: int):
    """CPU IndexIVFFlat.search restated (L2 coarse quantizer) -> (D, I)."""
    nq = xq.shape[0]
    _, probe = flat_search(xq, lists.cent, nprobe, METRIC_L2)
    largest = metric == METRIC_IP
    fill = -np.inf if largest else np.inf
    best_s = torch.full((nq, k), fill, dtype=torch.float32)
    best_i = torch.full((nq, k), -1, dtype=torch.int64)
    flat = probe.reshape(-1)
    qid = torch.arange(nq).repeat_interleave(probe.shape[1])
    order = torch.argsort(flat, stable=True)
    lsorted, qsorted = flat[order], qid[order]
    bounds = torch.searchsorted(lsorted, torch.arange(lists.nlist + 1))
    for l in range(lists.nlist):
        a, b = int(bounds[l]), int(bounds[l + 1])
        lo, hi = int(lists.off[l]), int(lists.off[l + 1])
        if a == b or lo == hi:
            continue
        qs = qsorted[a:b]
        ip = xq[qs] @ lists.xl[lo:hi].t()
        s = ip if largest else lists.norms[lo:hi][None, :] - 2.0 * ip
        kk = min(k, hi - lo)
        v, p = torch.topk(s, kk, dim=1, largest=largest, sorted=False)
        ns, ni = _merge(best_s[qs], best_i[qs], v, lists.pos2id[lo:hi][p], k, largest)
        best_s[qs] = ns
        best_i[qs] = ni
    if metric == METRIC_L2:
        best_s = best_s + (xq * xq).sum(1, keepdim=True)
    return best_s, best_i
