"""Retrieval -> DIN re-rank, batched on the device (SURVEY.md §8f rank 1,
BASELINE configs[4]).

The reference scores candidates one user at a time (DIN.py:167-189: a
forward over (C_u, L, d), a D2H copy and a numpy argsort per user) and builds
candidate lists with one faiss call per user (Retrieval.py:28-34).  Here every
stage is a batch over users, with ids instead of embeddings:

  cluster_candidates   Retrieval.py:28-34 (nearest centroid's whole list)
  finalize_candidates  finialize_retrieval.py:5-15 (ground truth appended
                       when missing; the reference's 400-cap line discards its
                       result, so lists are NOT truncated — mirrored)
  pad_candidates       ragged per-user lists -> (U, C) rows + mask
  rerank               DIN logits for (U, C) candidates, each attending over
                       its user's history (ids into the device item table;
                       the fused HIP gather/attention kernels of din.py)
  ndcg_at_k            DIN.py:181-189 on the device (first positive, stable
                       descending order)
  retrieve_and_rerank  configs[4]: top-k_retrieve flat/IVF retrieval of the
                       user profiles, then DIN re-rank, top-k_final per user
"""
from __future__ import annotations

import numpy as np
import torch

from .din import ndcg_from_logits


def cluster_candidates(centroid_index, cluster_lists, profiles: np.ndarray, uids) -> dict:
    """Retrieval.py:28-34 batched: ONE search for all profiles, then the chosen
    cluster's article ids.  `cluster_lists` maps cluster -> id array (e.g. the
    reference's cluster_to_articles, or IndexIVFFlat.list_ids)."""
    _, I = centroid_index.search(np.ascontiguousarray(profiles, dtype=np.float32), 1)
    get = cluster_lists if callable(cluster_lists) else cluster_lists.__getitem__
    return {u: np.asarray(get(int(c))) for u, c in zip(uids, I[:, 0])}


def finalize_candidates(recs: dict, ground_truth: dict) -> dict:
    """finialize_retrieval.py:5-15: append the ground-truth article when it is
    not among the candidates."""
    out = {}
    for uid, rec in recs.items():
        gt = ground_truth.get(uid)
        if gt is not None and gt not in rec:
            rec = np.append(rec, gt)
        out[uid] = rec
    return out


def pad_candidates(cand_lists, id_to_row: dict | None = None, device=None):
    """Ragged candidate id lists -> (rows (U, C) int32 with -1 padding, mask)."""
    C = max((len(c) for c in cand_lists), default=0)
    rows = np.full((len(cand_lists), max(C, 1)), -1, np.int32)
    for i, c in enumerate(cand_lists):
        r = [id_to_row[int(a)] for a in c] if id_to_row is not None else c
        rows[i, :len(c)] = r
    t = torch.from_numpy(rows).to(device)
    return t, t >= 0


def _fold_eval_head(fc):
    """The eval-mode head DIN.py:200-204 (BN -> Linear -> ReLU -> Dropout, twice,
    then BN -> Linear) with each BatchNorm folded into the Linear after it:
    Linear(BN(x)) = x (W s)^T + (b + W t), s = gamma / sqrt(var + eps),
    t = beta - mean s.  Returns [(W', b')] for the three Linears, or None when a
    BatchNorm has no running statistics (eval then normalises per batch)."""
    out = []
    for bn, lin in ((fc[0], fc[1]), (fc[4], fc[5]), (fc[8], fc[9])):
        if bn.running_mean is None:
            return None
        s = bn.weight / torch.sqrt(bn.running_var + bn.eps)
        t = bn.bias - bn.running_mean * s
        out.append(((lin.weight * s[None, :]).contiguous(), lin.bias + lin.weight @ t))
    return out


def _rerank_shared(model, table, hist_rows, cand_rows, batch_samples):
    """Shared-history path: U = q W1q^T + b1 for all candidates (one GEMM),
    nrk_din_rerank_attn (P = K W1k^T once per user), the eval-mode head with
    its BatchNorms folded into the Linears (no [q, pooled] concatenation: the
    first layer is two GEMMs accumulating into one output)."""
    from . import _lib
    from .din import gather_rows

    U, C = cand_rows.shape
    L = hist_rows.shape[1]
    d = table.shape[1]
    W1, b1 = model.attn.attn[0].weight, model.attn.attn[0].bias
    A = W1.shape[0]
    W1k = W1[:, d:].to(torch.bfloat16).contiguous()
    w2 = model.attn.attn[2].weight.reshape(-1).contiguous()
    head = _fold_eval_head(model.fc)
    if head is not None:
        (H1, c1), (H2, c2), (H3, c3) = head
        H1q, H1p = H1[:, :d].t(), H1[:, d:].t()
    out = torch.empty((U, C), dtype=torch.float32, device=table.device)
    ub = max(1, batch_samples // max(C, 1))
    for lo in range(0, U, ub):
        hi = min(U, lo + ub)
        cr = cand_rows[lo:hi].reshape(-1).to(torch.int32).contiguous()
        q = gather_rows(table, cr)
        Uc = torch.addmm(b1, q, W1[:, :d].t())
        pooled = torch.empty_like(q)
        hr = hist_rows[lo:hi].to(torch.int32).contiguous()
        _lib.check(_lib.load().nrk_din_rerank_attn(
            _lib.ptr(table), table.shape[0], _lib.NRK_DTYPE_BF16, _lib.ptr(hr), hi - lo, L, _lib.ptr(Uc), C, d,
            _lib.ptr(W1k), _lib.ptr(w2), A, _lib.ptr(pooled), _lib.stream(table.device)), "din_rerank_attn")
        if head is None:
            lg = model.fc(torch.cat([q, pooled], dim=1)).view(hi - lo, C)
        else:
            h1 = torch.addmm(c1, q, H1q).addmm_(pooled, H1p).relu_()
            lg = torch.addmm(c3, torch.addmm(c2, h1, H2.t()).relu_(), H3.t()).view(hi - lo, C)
        out[lo:hi] = torch.where(cand_rows[lo:hi] >= 0, lg, torch.full_like(lg, -float("inf")))
    return out


@torch.no_grad()
def rerank(model, table: torch.Tensor, hist_rows: torch.Tensor, cand_rows: torch.Tensor,
           batch_samples: int = 1 << 18, shared: bool = True) -> torch.Tensor:
    """DIN logits (U, C) for candidate rows (U, C) (-1 = padding -> -inf) of
    users with history rows (U, L) (-1 = padding), all rows of `table` on the
    device.  Eval-mode BatchNorm is row-independent, so one forward over many
    users equals the reference's per-user forwards.  With a bf16 table
    (d in {64, 128, 256}, L <= 64) the attention runs shared per user
    (nrk_din_rerank_attn); otherwise every candidate is a DIN sample."""
    model.eval()
    U, C = cand_rows.shape
    L = hist_rows.shape[1]
    if (shared and table.dtype == torch.bfloat16 and table.shape[1] in (64, 128, 256) and L <= 64
            and model.attn.attn[0].weight.shape[1] == 2 * table.shape[1]):
        return _rerank_shared(model, table, hist_rows, cand_rows, batch_samples)
    out = torch.empty((U, C), dtype=torch.float32, device=table.device)
    ub = max(1, batch_samples // max(C, 1))
    for lo in range(0, U, ub):
        hi = min(U, lo + ub)
        cr = cand_rows[lo:hi].reshape(-1).to(torch.int32)
        hr = hist_rows[lo:hi, None, :].expand(hi - lo, C, L).reshape(-1, L).to(torch.int32)
        lg = model.forward_ids(table, cr, hr).view(hi - lo, C)
        out[lo:hi] = torch.where(cand_rows[lo:hi] >= 0, lg, torch.full_like(lg, -float("inf")))
    return out


def ndcg_at_k(logits: torch.Tensor, labels: torch.Tensor, k: int) -> torch.Tensor:
    """Per-user NDCG@k with one relevant item (DIN.py:181-189); padded
    candidates carry -inf logits and label 0."""
    U, C = logits.shape
    seg = torch.arange(U, device=logits.device).repeat_interleave(C)
    return ndcg_from_logits(logits.reshape(-1), labels.reshape(-1).float(), seg, U, k)


@torch.no_grad()
def retrieve_and_rerank(index, model, table: torch.Tensor, profiles: torch.Tensor, hist_rows: torch.Tensor,
                        k_retrieve: int = 200, k_final: int = 5, gt_rows: torch.Tensor | None = None):
    """configs[4]: retrieve k_retrieve candidates per user profile from `index`
    (a flat / IVF / sharded index over the rows of `table`; search_device
    returns row ids), optionally append each user's ground-truth row when it
    was not retrieved (finialize_retrieval.py), DIN re-rank, and return
    (top k_final rows (U, k_final), logits (U, C), cand_rows (U, C), ndcg@k_final
    per user or None)."""
    _, I = index.search_device(profiles, k_retrieve)
    cand = I.to(torch.int32)
    labels = None
    if gt_rows is not None:
        gt = gt_rows.to(torch.int32)
        hit = (cand == gt[:, None]).any(1)
        extra = torch.where(hit, torch.full_like(gt, -1), gt)
        cand = torch.cat([cand, extra[:, None]], 1)
        labels = (cand == gt[:, None]) & (cand >= 0)
    logits = rerank(model, table, hist_rows, cand)
    order = torch.sort(logits, dim=1, descending=True, stable=True).indices[:, :k_final]
    top = torch.gather(cand, 1, order)
    nd = ndcg_at_k(logits, labels, k_final) if labels is not None else None
    return top, logits, cand, nd
