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

import ctypes
import warnings
import weakref

import numpy as np
import torch

RERANK_MAX_L = 64  # nrk_din_rerank holds one user's history rows (and their projections) in LDS


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


_PARAMS_CACHE: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()  # model -> (key, params)


def rerank_params(model, d: int):
    """The eval model as nrk_din_rerank takes it (include/nrk.h
    nrk_din_rerank_params): W1 = [W1q | W1k] (DIN.py:99), w2, b1; the head with
    its three BatchNorms folded into the Linears after them (_fold_eval_head);
    every weight the kernel feeds to a bf16 MFMA split into hi + lo.  Returns
    (params struct, A, F, tensors kept alive) or None when the head has no
    running statistics.  Cached per model (weakly: a dropped model frees its
    copies) until any parameter or buffer changes (torch's version counters;
    inference-mode tensors have none, so such a model is not cached)."""
    from . import _lib

    tens = list(model.parameters()) + list(model.buffers())
    cacheable = not any(t.is_inference() for t in tens)
    key = (tuple(t._version for t in tens), tuple(t.data_ptr() for t in tens)) if cacheable else None
    hit = _PARAMS_CACHE.get(model) if cacheable else None
    if hit is not None and hit[0] == key:
        return hit[1]
    head = _fold_eval_head(model.fc)
    if head is None:
        return None
    W1, b1 = model.attn.attn[0].weight, model.attn.attn[0].bias
    w2 = model.attn.attn[2].weight.reshape(-1).contiguous().float()
    (H1, c1), (H2, c2), (H3, c3) = head
    keep = {}
    for name, t in (("W1q", W1[:, :d]), ("W1k", W1[:, d:]), ("H1q", H1[:, :d]), ("H1p", H1[:, d:]), ("H2", H2)):
        keep[name + "_hi"], keep[name + "_lo"] = _split_bf16(t.detach().float().contiguous())
    keep["b1"] = b1.detach().float().contiguous()
    keep["w2"] = w2.detach()
    keep["c1"] = c1.detach().float().contiguous()
    keep["c2"] = c2.detach().float().contiguous()
    keep["h3"] = H3.detach().reshape(-1).float().contiguous()
    prm = _lib.RerankParams(**{k: v.data_ptr() for k, v in keep.items()}, c3=float(c3.detach().reshape(-1)[0]))
    out = (prm, W1.shape[0], H1.shape[0], keep)
    if cacheable:
        _PARAMS_CACHE[model] = (key, out)
    return out


def _table_dtype(table: torch.Tensor) -> int:
    from . import _lib

    if table.dtype == torch.bfloat16:
        return _lib.NRK_DTYPE_BF16
    if table.dtype == torch.float32:
        return _lib.NRK_DTYPE_F32
    raise ValueError(f"re-rank: item table dtype {table.dtype} (bf16 or f32)")


def rerank_project(model, table: torch.Tensor, rows: torch.Tensor, prm=None, hist: bool = False) -> torch.Tensor:
    """nrk_din_rerank_project: the candidate-only part of the re-rank for each
    row, [U' (A) | Q1 (F)] f32, with the arithmetic nrk_din_rerank applies per
    candidate (a shared list is projected once instead of once per user).
    hist: nrk_din_rerank_project_hist, the history-only part [P' (A) | R (F)]
    of each row.  An f32 table enters split into bf16 hi + lo (the reference's
    fp32 embeddings to ~2^-16)."""
    from . import _lib

    d = table.shape[1]
    if prm is None:
        prm = rerank_params(model, d)
    p, A, F, _keep = prm
    r = rows.to(torch.int32).contiguous()
    out = torch.empty((r.numel(), A + F), dtype=torch.float32, device=table.device)
    lib = _lib.load()
    fn = lib.nrk_din_rerank_project_hist if hist else lib.nrk_din_rerank_project
    _lib.check(fn(_lib.ptr(table), table.shape[0], _table_dtype(table), _lib.ptr(r), r.numel(), d, A, F, ctypes.byref(p),
                  _lib.ptr(out), _lib.stream(table.device)), "din_rerank_project" + ("_hist" if hist else ""))
    return out


HIST_PROJ_BUDGET = 4 << 30  # bytes of per-slot history projections per rerank_ragged launch
_RERANK_WS: dict = {}  # (device, stream) -> nrk_din_rerank workspace (each call resets what it uses)


def _rerank_workspace(dev) -> torch.Tensor:
    from . import _lib

    key = (dev, _lib.stream(dev))
    ws = _RERANK_WS.get(key)
    if ws is None:
        sz = _lib.c_size(0)
        _lib.check(_lib.load().nrk_din_rerank_workspace(sz), "din_rerank_workspace")
        ws = _RERANK_WS[key] = torch.zeros(max(sz.value, 1), dtype=torch.uint8, device=dev)
    return ws


def rerank_ragged(model, table: torch.Tensor, hist_rows: torch.Tensor, cand: torch.Tensor, cand_off: torch.Tensor,
                  cand_len: torch.Tensor, extra: torch.Tensor | None, out_off: torch.Tensor, n_out: int,
                  prm=None, shared: bool = False, direct: bool = False) -> torch.Tensor:
    """The fused re-rank, one launch for all users.  User u scores
    cand[cand_off[u] : cand_off[u] + cand_len[u]] (+ extra[u] when given, -1 =
    a padded slot) against its history hist_rows[u] and writes
    out[out_off[u] + c]; rows outside the table get -inf.  Returns out (n_out,)
    f32 (entries not covered by any user stay uninitialised).  The rows are
    projected (rerank_project: the candidates' [U' | Q1], the history slots'
    [P' | R]; an f32 table split into bf16 hi + lo) and
    nrk_din_rerank_projected scores the projections (for F <= 64 one wave per
    32 candidates, din_rerank_lane.hip).  shared: a hint only (the lists are
    shared by many users; either way every row is projected once per call).
    direct: a bf16 table through nrk_din_rerank instead (the per-chunk kernel
    that reads the rows itself; its arithmetic order differs, within the same
    tolerance of the reference)."""
    from . import _lib

    dev = table.device
    U, L = hist_rows.shape
    d = table.shape[1]
    if prm is None:
        prm = rerank_params(model, d)
    p, A, F, _keep = prm
    out = torch.empty(n_out, dtype=torch.float32, device=dev)
    if U == 0:
        return out
    if direct and table.dtype != torch.bfloat16:
        raise ValueError("rerank_ragged(direct=True) reads bf16 table rows; an f32 table takes the projected form")
    lib = _lib.load()
    ws = _rerank_workspace(dev)
    h = hist_rows.to(torch.int32).contiguous()
    c = cand.to(torch.int32).contiguous()
    co, cl, oo = cand_off.to(torch.int64).contiguous(), cand_len.to(torch.int32).contiguous(), \
        out_off.to(torch.int64).contiguous()
    ex = extra.to(torch.int32).contiguous() if extra is not None else None
    from .din import KernelTimer

    if not direct:
        tp = KernelTimer.mark("rerank_project")
        cp = rerank_project(model, table, c, prm)
        xp = rerank_project(model, table, ex, prm) if ex is not None else None
        KernelTimer.push("rerank_project", tp)
        # the history projections are per slot (U L (A + F) f32): users in chunks
        # whose projections fit HIST_PROJ_BUDGET (one chunk up to ~100K users at
        # L = 64, A + F = 160), the candidates' projections shared by all chunks
        ub = max(1, HIST_PROJ_BUDGET // (L * (A + F) * 4))
        for lo in range(0, U, ub):
            hi = min(U, lo + ub)
            tp = KernelTimer.mark("rerank_project")
            hp = rerank_project(model, table, h[lo:hi].reshape(-1), prm, hist=True)
            KernelTimer.push("rerank_project", tp)
            t0 = KernelTimer.mark("rerank")  # (the main kernel alone)
            _lib.check(lib.nrk_din_rerank_projected(
                _lib.ptr(table), table.shape[0], _table_dtype(table), _lib.ptr(h[lo:hi]), hi - lo, L, _lib.ptr(c),
                _lib.ptr(co[lo:hi]), _lib.ptr(cl[lo:hi]), _lib.ptr(ex[lo:hi]) if ex is not None else None,
                _lib.ptr(oo[lo:hi]), _lib.ptr(out), d, A, F, ctypes.byref(p), _lib.ptr(cp),
                _lib.ptr(xp[lo:hi]) if xp is not None else None, _lib.ptr(hp), _lib.ptr(ws), ws.numel(),
                _lib.stream(dev)), "din_rerank_projected")
            KernelTimer.push("rerank", t0)
            del hp
        return out
    t0 = KernelTimer.mark("rerank")
    _lib.check(lib.nrk_din_rerank(_lib.ptr(table), table.shape[0], _lib.NRK_DTYPE_BF16, _lib.ptr(h), U, L,
                                  _lib.ptr(c), _lib.ptr(co), _lib.ptr(cl), _lib.ptr(ex), _lib.ptr(oo),
                                  _lib.ptr(out), d, A, F, ctypes.byref(p), _lib.ptr(ws), ws.numel(),
                                  _lib.stream(dev)), "din_rerank")
    KernelTimer.push("rerank", t0)
    return out


def rerank_max_history(A: int, F: int) -> int:
    """nrk_din_rerank_max_history: the longest history the fused (projected)
    re-rank holds for (A, F): 128 over the whole Optuna grid (DIN.py:203-207;
    the lane kernel's 128-row form), RERANK_MAX_L outside it."""
    from . import _lib

    if A not in (32, 64, 96, 128) or F not in (32, 64, 96, 128):
        return RERANK_MAX_L
    v = ctypes.c_int32(0)
    _lib.check(_lib.load().nrk_din_rerank_max_history(A, F, ctypes.byref(v)), "din_rerank_max_history")
    return int(v.value)


def fused_ok(model, table: torch.Tensor, L: int):
    """Why the fused re-rank kernel cannot run this model / table (empty: it can)."""
    W1 = model.attn.attn[0].weight
    A, F = W1.shape[0], model.fc[1].weight.shape[0]
    d = table.shape[1]
    max_l = rerank_max_history(A, F) if L > RERANK_MAX_L else RERANK_MAX_L
    return [w for w, bad in (("table is neither bf16 nor f32", table.dtype not in (torch.bfloat16, torch.float32)),
                             (f"emb_dim {d} not in (64, 128, 256)", d not in (64, 128, 256)),
                             (f"history length {L} > {max_l}", L > max_l),
                             (f"attn_units {A} not in (32, 64, 96, 128)", A not in (32, 64, 96, 128)),
                             (f"fc_units {F} not in (32, 64, 96, 128)", F not in (32, 64, 96, 128)),
                             ("model emb_dim != table width", W1.shape[1] != 2 * d),
                             ("BatchNorm without running statistics",
                              any(model.fc[i].running_mean is None for i in (0, 4, 8)))) if bad]


@torch.no_grad()
def rerank(model, table: torch.Tensor, hist_rows: torch.Tensor, cand_rows: torch.Tensor,
           batch_samples: int = 1 << 20, shared: bool = True) -> torch.Tensor:
    """DIN logits (U, C) for candidate rows (U, C) (-1 = padding -> -inf) of
    users with history rows (U, L) (-1 = padding), all rows of `table` on the
    device.  Eval-mode BatchNorm is row-independent, so one forward over many
    users equals the reference's per-user forwards.  With a bf16 or f32
    table, d in {64, 128, 256}, L <= 128, A and F in {32, 64, 96, 128} the
    whole evaluate() forward is one fused launch over the row projections
    (rerank_ragged); otherwise every candidate is a DIN sample
    (model.forward_ids, C x the attention work)."""
    model.eval()
    U, C = cand_rows.shape
    L = hist_rows.shape[1]
    why = (["shared=False"] if not shared else []) + fused_ok(model, table, L)
    # which path ran, for callers and benchmarks (the per-candidate one costs C x the attention work)
    rerank.path = "fused" if not why else "per-candidate: " + ", ".join(why)
    dev = table.device
    if not why:
        off = torch.arange(U, device=dev, dtype=torch.int64) * C
        out = rerank_ragged(model, table, hist_rows, cand_rows.reshape(-1), off,
                            torch.full((U,), C, dtype=torch.int32, device=dev), None, off, U * C)
        return out.view(U, C)
    if shared:
        warnings.warn(f"rerank: {rerank.path} -> per-candidate DIN forward (C x the attention work of the fused "
                      f"path)", stacklevel=2)
    out = torch.empty((U, C), dtype=torch.float32, device=dev)
    ub = max(1, batch_samples // max(C, 1))
    for lo in range(0, U, ub):
        hi = min(U, lo + ub)
        cr = cand_rows[lo:hi].reshape(-1).to(torch.int32)
        hr = hist_rows[lo:hi, None, :].expand(hi - lo, C, L).reshape(-1, L).to(torch.int32)
        lg = model.forward_ids(table, cr, hr).view(hi - lo, C)
        ok = (cand_rows[lo:hi] >= 0) & (cand_rows[lo:hi] < table.shape[0])  # rows outside the table: -inf, as fused
        out[lo:hi] = torch.where(ok, lg, torch.full_like(lg, -float("inf")))
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
    Users are grouped by cluster and ALL of them are scored by one fused
    launch (nrk_din_rerank_projected: each user's offset points at its
    cluster's list, projected once).  A model / table the fused kernel cannot
    run (fused_ok) falls back, with a warning, to rerank() per cluster (every
    candidate its own DIN sample); `path` in the result says which ran.

    last_rows (U,) -- the row of each user's last click -- gives
    EvalDataset's labels (one-hot at the FIRST candidate equal to it, none when
    absent; DIN.py:27-31), the per-user BCE (DIN.py:176-177) and NDCG@k
    (DIN.py:181-189, ndcg_at_k's tie rule).  append_missing: the ground truth
    (the last click) is appended to a user's list when the cluster lacks it
    (finialize_retrieval.py:11-12): one extra column per user, -1 (padding,
    excluded from the loss) where the cluster holds it; a user whose cluster
    is empty then scores the ground truth alone.  A user left with no
    candidate at all gets loss and NDCG NaN (not 0), so means over users do
    not silently count it.  Returns a dict: `logits` list of
    (n_users_c, C_c [+1]) per non-empty group, `users` the user indices of
    each group, and with last_rows `loss` (U,) f64 and `ndcg` (U,) f64."""
    dev = table.device
    U, L = hist_rows.shape
    uc = user_cluster.to(dev).long()
    off = cluster_off.to(dev).long()
    rows = cluster_rows.to(dev).to(torch.int32)
    nl = off.numel() - 1
    why = fused_ok(model, table, L)
    model.eval()
    order = torch.sort(uc, stable=True).indices
    ucs = uc[order]
    sizes = (off[1:] - off[:-1])
    clen = sizes[ucs]  # (U,) candidates of each user (in group order)
    coff = off[ucs]
    last = last_rows.to(dev).long()[order] if last_rows is not None else None
    pos_in = None
    if last is not None:
        # position of the FIRST occurrence of the last click inside its user's
        # cluster list (-1: absent; EvalDataset's label, DIN.py:27-31), by a
        # sorted search over (cluster, row) keys -- a stable sort, so among equal
        # keys the leftmost is the earliest list position
        n_tab = table.shape[0]
        member_cl = torch.repeat_interleave(torch.arange(nl, device=dev), sizes)
        keys = member_cl * (n_tab + 1) + rows.long()
        skeys, sidx = torch.sort(keys, stable=True)
        q = ucs * (n_tab + 1) + last.clamp(0, n_tab)
        if skeys.numel():
            at = torch.searchsorted(skeys, q).clamp_max(skeys.numel() - 1)
            found = (skeys[at] == q) & (last >= 0)
            pos_in = torch.where(found, sidx[at] - coff, torch.full_like(last, -1))
        else:
            pos_in = torch.full_like(last, -1)
    extra = None
    if last is not None and append_missing:
        extra = torch.where(pos_in >= 0, torch.full_like(last, -1), last).to(torch.int32)
    width = clen + (1 if extra is not None else 0)
    oo = torch.zeros(U + 1, dtype=torch.int64, device=dev)
    torch.cumsum(width, 0, out=oo[1:])
    n_out = int(oo[-1].item())
    cnt = torch.bincount(ucs, minlength=nl)
    bh = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), torch.cumsum(cnt, 0)]).cpu().tolist()
    wh = (sizes + (1 if extra is not None else 0)).cpu().tolist()
    oh = oo.cpu().tolist()
    if not why:
        flat = rerank_ragged(model, table, hist_rows[order], rows, coff, clen, extra, oo[:-1], n_out, shared=True)
        path = "fused"
    else:
        # the fused kernel cannot run this model / table: each cluster's users
        # through rerank(), which scores every candidate as its own DIN sample
        warnings.warn("rerank_clusters: " + ", ".join(why) + " -> per-candidate DIN forward per cluster (C x the "
                      "attention work of the fused path)", stacklevel=2)
        flat = torch.empty(n_out, dtype=torch.float32, device=dev)
        ol = off.cpu().tolist()
        for c in range(nl):
            lo, hi = bh[c], bh[c + 1]
            if hi <= lo or wh[c] == 0:
                continue
            cand = rows[ol[c]:ol[c + 1]][None, :].expand(hi - lo, -1)
            if extra is not None:
                cand = torch.cat([cand, extra[lo:hi, None]], 1)
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")  # (warned once above)
                lg = rerank(model, table, hist_rows[order[lo:hi]], cand.contiguous(), batch_samples=batch_samples)
            flat[oh[lo]:oh[hi]] = lg.reshape(-1)
        path = "per-candidate: " + ", ".join(why)
    rerank.path = path
    out = {"logits": [], "users": [], "path": path}
    for c in range(nl):
        lo, hi = bh[c], bh[c + 1]
        if hi > lo and wh[c] > 0:
            out["logits"].append(flat[oh[lo]:oh[hi]].view(hi - lo, wh[c]))
            out["users"].append(order[lo:hi])
    if last is not None:
        # labels: one-hot at the first occurrence of the last click (its cluster
        # position, else the appended column), BCE over the valid candidates
        # (DIN.py:176-177), NDCG@k with ndcg_at_k's rule, all as segment sums
        has_pos = pos_in >= 0
        pcol = torch.where(has_pos, pos_in, clen if extra is not None else torch.full_like(clen, -1))
        if extra is not None:
            has_pos = has_pos | (extra >= 0)
        # one block per user (nrk_rerank_user_stats): the BCE sum over the
        # finite logits in f64, their count, and the candidates ranked before
        # the positive by the sigmoid probabilities (stable-sort ties)
        from . import _lib

        pos = torch.where(has_pos, oo[:-1] + pcol.clamp_min(0), torch.full_like(pcol, -1)).to(torch.int64).contiguous()
        pr = torch.sigmoid(flat)
        loss_sum = torch.empty(U, dtype=torch.float64, device=dev)
        nval = torch.empty(U, dtype=torch.int64, device=dev)
        before = torch.empty(U, dtype=torch.int64, device=dev)
        _lib.check(_lib.load().nrk_rerank_user_stats(_lib.ptr(flat), _lib.ptr(pr), _lib.ptr(oo), _lib.ptr(pos), U,
                                                     _lib.ptr(loss_sum), _lib.ptr(nval), _lib.ptr(before),
                                                     _lib.stream(dev)), "rerank_user_stats")
        loss = loss_sum / nval.double()
        rank = before + 1
        nd = torch.where(has_pos & (rank <= k), 1.0 / torch.log2(rank.double() + 1.0), torch.zeros_like(loss))
        nd = torch.where(nval > 0, nd, torch.full_like(nd, float("nan")))
        loss_u = torch.empty(U, dtype=torch.float64, device=dev)
        ndcg_u = torch.empty(U, dtype=torch.float64, device=dev)
        loss_u[order] = loss
        ndcg_u[order] = nd
        out["loss"], out["ndcg"] = loss_u, ndcg_u
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

