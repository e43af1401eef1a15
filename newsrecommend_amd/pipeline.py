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

import warnings

import numpy as np
import torch

RERANK_SHARED_MAX_L = 64  # nrk_din_rerank_attn holds the history image of one user in LDS


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


def _split_bf16(w: torch.Tensor):
    """f32 weights -> (hi, lo) bf16 with hi + lo = w to 16 mantissa bits."""
    hi = w.to(torch.bfloat16)
    return hi.contiguous(), (w - hi.float()).to(torch.bfloat16).contiguous()


def _rerank_shared(model, table, hist_rows, cand_rows, batch_samples):
    """Shared-history path, three HIP kernels per batch of users:
      nrk_din_item_proj    [U | Q1] = q [W1q ; H1q]^T + [b1 ; 0] gathered from
                           the bf16 table (the attention query half and the
                           head's first-layer query half in one pass),
      nrk_din_rerank_attn  P = K W1k^T once per user, per-candidate scores,
                           softmax over the L slots, pooled = alpha K,
      nrk_din_rerank_head  the eval-mode head (BatchNorms folded into the
                           Linears) -> logits, -inf on padded candidates.
    Heads the fused kernel does not cover (F != 32, BatchNorm without running
    statistics) run as torch ops on the gathered rows."""
    from . import _lib
    from .din import gather_rows

    U, C = cand_rows.shape
    L = hist_rows.shape[1]
    d = table.shape[1]
    dev = table.device
    W1, b1 = model.attn.attn[0].weight, model.attn.attn[0].bias
    A = W1.shape[0]
    W1k = W1[:, d:].to(torch.bfloat16).contiguous()
    w2 = model.attn.attn[2].weight.reshape(-1).contiguous()
    head = _fold_eval_head(model.fc)
    fused = head is not None and head[0][0].shape[0] == 32
    if fused:
        (H1, c1), (H2, c2), (H3, c3) = head
        F = H1.shape[0]
        Wcat = torch.cat([W1[:, :d], H1[:, :d]], 0)
        bcat = torch.cat([b1, torch.zeros(F, device=dev)]).contiguous()
    else:
        Wcat, bcat = W1[:, :d], b1.contiguous()
        if head is not None:
            (H1, c1), (H2, c2), (H3, c3) = head
            H1q, H1p = H1[:, :d].t(), H1[:, d:].t()
    NO = max(128, -(-Wcat.shape[0] // 32) * 32)  # nrk_din_item_proj: 128..256 outputs, zero rows pad
    Wpad = torch.zeros((NO, d), device=dev)
    Wpad[:Wcat.shape[0]] = Wcat
    bpad = torch.zeros(NO, device=dev)
    bpad[:bcat.shape[0]] = bcat
    W_hi, W_lo = _split_bf16(Wpad)
    if fused:
        Hp_hi, Hp_lo = _split_bf16(H1[:, d:].contiguous())
        H2c, c2c, h3c = H2.contiguous(), c2.contiguous(), H3.reshape(-1).contiguous()
        c3v = float(c3.reshape(-1)[0])
    lib = _lib.load()
    st = _lib.stream(dev)
    out = torch.empty((U, C), dtype=torch.float32, device=dev)
    ub = max(1, batch_samples // max(C, 1))
    for lo in range(0, U, ub):
        hi = min(U, lo + ub)
        n = (hi - lo) * C
        cr = cand_rows[lo:hi].reshape(-1).to(torch.int32).contiguous()
        proj = torch.empty((n, NO), dtype=torch.float32, device=dev)
        _lib.check(lib.nrk_din_item_proj(_lib.ptr(table), table.shape[0], _lib.NRK_DTYPE_BF16, _lib.ptr(cr), n, d,
                                         _lib.ptr(W_hi), _lib.ptr(W_lo), _lib.ptr(bpad), NO, _lib.ptr(proj), st),
                   "din_item_proj")
        pooled = torch.empty((n, d), dtype=torch.float32, device=dev)
        hr = hist_rows[lo:hi].to(torch.int32).contiguous()
        _lib.check(lib.nrk_din_rerank_attn(
            _lib.ptr(table), table.shape[0], _lib.NRK_DTYPE_BF16, _lib.ptr(hr), hi - lo, L, _lib.ptr(proj), NO, C, d,
            _lib.ptr(W1k), _lib.ptr(w2), A, _lib.ptr(pooled), st), "din_rerank_attn")
        if fused:
            lg = torch.empty(n, dtype=torch.float32, device=dev)
            _lib.check(lib.nrk_din_rerank_head(
                _lib.ptr(pooled), n, d, _lib.ptr(proj) + 4 * A, NO, _lib.ptr(cr), _lib.ptr(Hp_hi), _lib.ptr(Hp_lo),
                _lib.ptr(c1), F, _lib.ptr(H2c), _lib.ptr(c2c), _lib.ptr(h3c), c3v, _lib.ptr(lg), st),
                "din_rerank_head")
            out[lo:hi] = lg.view(hi - lo, C)
            continue
        q = gather_rows(table, cr)
        if head is None:
            lg = model.fc(torch.cat([q, pooled], dim=1)).view(hi - lo, C)
        else:
            h1 = torch.addmm(c1, q, H1q).addmm_(pooled, H1p).relu_()
            lg = torch.addmm(c3, torch.addmm(c2, h1, H2.t()).relu_(), H3.t()).view(hi - lo, C)
        out[lo:hi] = torch.where(cand_rows[lo:hi] >= 0, lg, torch.full_like(lg, -float("inf")))
    return out


@torch.no_grad()
def rerank(model, table: torch.Tensor, hist_rows: torch.Tensor, cand_rows: torch.Tensor,
           batch_samples: int = 1 << 20, shared: bool = True) -> torch.Tensor:
    """DIN logits (U, C) for candidate rows (U, C) (-1 = padding -> -inf) of
    users with history rows (U, L) (-1 = padding), all rows of `table` on the
    device.  Eval-mode BatchNorm is row-independent, so one forward over many
    users equals the reference's per-user forwards.  With a bf16 table
    (d in {64, 128, 256}, L <= 64) the attention runs shared per user
    (nrk_din_rerank_attn); otherwise every candidate is a DIN sample."""
    model.eval()
    U, C = cand_rows.shape
    L = hist_rows.shape[1]
    why = [w for w, bad in (("shared=False", not shared), ("table is not bf16", table.dtype != torch.bfloat16),
                            (f"emb_dim {table.shape[1]} not in (64, 128, 256)", table.shape[1] not in (64, 128, 256)),
                            (f"history length {L} > {RERANK_SHARED_MAX_L}", L > RERANK_SHARED_MAX_L),
                            ("model emb_dim != table width", model.attn.attn[0].weight.shape[1] != 2 * table.shape[1]))
           if bad]
    # which path ran, for callers and benchmarks (the per-candidate one costs C x the attention work)
    rerank.path = "shared" if not why else "per-candidate: " + ", ".join(why)
    if not why:
        return _rerank_shared(model, table, hist_rows, cand_rows, batch_samples)
    if shared:
        warnings.warn(f"rerank: {rerank.path} -> per-candidate DIN forward (C x the attention work of the shared "
                      f"path)", stacklevel=2)
    out = torch.empty((U, C), dtype=torch.float32, device=table.device)
    ub = max(1, batch_samples // max(C, 1))
    for lo in range(0, U, ub):
        hi = min(U, lo + ub)
        cr = cand_rows[lo:hi].reshape(-1).to(torch.int32)
        hr = hist_rows[lo:hi, None, :].expand(hi - lo, C, L).reshape(-1, L).to(torch.int32)
        lg = model.forward_ids(table, cr, hr).view(hi - lo, C)
        out[lo:hi] = torch.where(cand_rows[lo:hi] >= 0, lg, torch.full_like(lg, -float("inf")))
    return out


rerank.path = None


@torch.no_grad()
def rerank_clusters(model, table: torch.Tensor, hist_rows: torch.Tensor, user_cluster: torch.Tensor,
                    cluster_off: torch.Tensor, cluster_rows: torch.Tensor, last_rows: torch.Tensor | None = None,
                    k: int = 5, batch_samples: int = 1 << 22, append_missing: bool = False):
    """Retrieval.py:28-34 -> DIN.py:155-193 as the reference runs it: every
    user's candidates are the WHOLE cluster its profile is nearest to
    (cluster_candidates), so all users of cluster c share one ragged list,
    rows cluster_rows[cluster_off[c]:cluster_off[c+1]] (corpus row order).
    Users are grouped by cluster and each group is re-ranked as a padding-free
    (n_users_c, C_c) batch (rerank, the shared-history kernels).

    last_rows (U,) -- the row of each user's last click -- gives
    EvalDataset's labels (one-hot at the FIRST candidate equal to it, none when
    absent; DIN.py:27-31), the per-user BCE (DIN.py:176-177) and NDCG@k
    (DIN.py:181-189, ndcg_at_k's tie rule).  append_missing: the ground truth
    (the last click) is appended to a user's list when the cluster lacks it
    (finialize_retrieval.py:11-12): one extra column per group, -1 (padding,
    excluded from the loss) where the cluster holds it.  Returns a dict:
    `logits` list of (n_users_c, C_c [+1]) per cluster, `users` list of the
    user indices of each group, and with last_rows `loss` (U,) f64 and
    `ndcg` (U,) f64."""
    dev = table.device
    U = hist_rows.shape[0]
    uc = user_cluster.to(dev).long()
    off = cluster_off.to(dev).long()
    rows = cluster_rows.to(dev).to(torch.int32)
    order = torch.sort(uc, stable=True).indices
    bounds = torch.searchsorted(uc[order], torch.arange(off.numel(), device=dev))
    bh = bounds.cpu().tolist()  # one small host read: the group boundaries
    oh = off.cpu().tolist()
    out = {"logits": [], "users": []}
    if last_rows is not None:
        loss = torch.zeros(U, dtype=torch.float64, device=dev)
        ndcg = torch.zeros(U, dtype=torch.float64, device=dev)
        last = last_rows.to(dev).to(torch.int32)
    for c in range(off.numel() - 1):
        lo, hi = bh[c], bh[c + 1]
        if hi <= lo or oh[c + 1] <= oh[c]:
            continue
        us = order[lo:hi]
        cand = rows[oh[c]:oh[c + 1]]
        C = cand.numel()
        cu = cand[None, :].expand(hi - lo, C)
        if last_rows is not None and append_missing:
            lu = last[us]
            extra = torch.where((cu == lu[:, None]).any(1), torch.full_like(lu, -1), lu)
            cu = torch.cat([cu, extra[:, None]], 1)
        lg = rerank(model, table, hist_rows[us], cu, batch_samples=batch_samples)
        out["logits"].append(lg)
        out["users"].append(us)
        if last_rows is not None:
            hit = (cu == last[us][:, None]) & (cu >= 0)
            first = torch.where(hit.any(1), hit.to(torch.int8).argmax(1), torch.full_like(us, -1))
            lab = torch.zeros(cu.shape, dtype=torch.bool, device=dev)
            has = first >= 0
            lab[has.nonzero().squeeze(1), first[has]] = True
            valid = cu >= 0
            per = torch.nn.functional.binary_cross_entropy_with_logits(lg.clamp_min(-1e30), lab.float(),
                                                                       reduction="none")
            per = torch.where(valid, per.double(), torch.zeros_like(per, dtype=torch.float64))
            loss[us] = per.sum(1) / valid.sum(1).double()
            ndcg[us] = ndcg_at_k(lg, lab, k)
    if last_rows is not None:
        out["loss"], out["ndcg"] = loss, ndcg
    return out


def ndcg_at_k(logits: torch.Tensor, labels: torch.Tensor, k: int) -> torch.Tensor:
    """Per-user NDCG@k with one relevant item (DIN.py:181-189); padded
    candidates carry -inf logits and label 0.  Same rule as
    din.ndcg_from_logits (rank of the FIRST positive = 1 + #{p_j > p_pos} +
    #{j before pos with p_j == p_pos}) on the rectangular (U, C) batch, as
    row sums instead of segment scatters.

    Ties are a deliberate deviation: the reference ranks with
    np.argsort(-probs) (DIN.py:183), whose default sort is not stable, so the
    rank of a positive tied with other candidates (f32 sigmoid saturates to 1.0
    above logit ~17) depends on numpy's sort implementation and version.  Here
    tied candidates keep column order (a stable descending sort), the same rule
    as _top_and_ndcg's top-k.  Without ties the two agree exactly (pinned by
    the din_dataset / din_rerank_c5 fixtures); tie cases are parity unpinned."""
    U, C = logits.shape
    col = torch.arange(C, device=logits.device, dtype=torch.int64)
    probs = torch.sigmoid(logits)
    labels = labels > 0.5 if labels.dtype != torch.bool else labels
    has = labels.any(1)
    pos = torch.where(has, labels.to(torch.int8).argmax(1), torch.zeros_like(has, dtype=torch.long))
    pp = probs.gather(1, pos[:, None])
    before = (probs > pp) | ((probs == pp) & (col[None, :] < pos[:, None]))
    rank = before.sum(1) + 1
    return torch.where(has & (rank <= k), 1.0 / torch.log2(rank.double() + 1.0),
                       torch.zeros_like(rank, dtype=torch.double))


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
    top, nd = _top_and_ndcg(logits, cand, labels, k_final)
    return top, logits, cand, nd


def _top_and_ndcg(logits: torch.Tensor, cand: torch.Tensor, labels: torch.Tensor | None, k: int):
    """The top-k candidates in a stable descending order of the logits (ties:
    lower column first) and, with labels, the per-user NDCG@k of
    ndcg_at_k, on the rectangular (U, C) batch: top-k over int64 keys
    (order-preserving int of the f32 logit << 16 | (65535 - column)) instead of
    a stable segmented sort, with ndcg_at_k's row-sum rank (0.42 -> 0.25 ms
    at 4096 x 201; identical outputs, ties included)."""
    U, C = logits.shape
    col = torch.arange(C, device=logits.device, dtype=torch.int64)
    if C <= 0xFFFF:
        b = (logits + 0.0).contiguous().view(torch.int32)  # + 0.0: -0.0 ties +0.0, as in the sort
        key = (b ^ ((b >> 31) & 0x7FFFFFFF)).to(torch.int64)
        order = torch.topk((key << 16) | (0xFFFF - col), min(k, C), dim=1, sorted=True).indices
    else:
        order = torch.sort(logits, dim=1, descending=True, stable=True).indices[:, :k]
    top = torch.gather(cand, 1, order)
    return top, (ndcg_at_k(logits, labels, k) if labels is not None else None)

