"""oracle/din_oracle.py — TEST INFRASTRUCTURE ONLY (the checker, never the
product).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import this module.

A float64 numpy restatement of the reference DIN ranker, function by function:

  attention_forward    AttentionLayer.forward           DIN.py:103-111
  din_forward          DIN.forward (+ eval/train BN)    DIN.py:113-133
  bce_with_logits      nn.BCEWithLogitsLoss (mean)      DIN.py:148, 247
  din_backward         loss.backward() for all params   DIN.py:149
  clip_grad_norm       nn.utils.clip_grad_norm_(.., 1)  DIN.py:150
  adam_step            optim.Adam(lr, weight_decay)     DIN.py:151, 245
  ndcg_single          evaluate()'s per-user NDCG@k     DIN.py:181-189

Pinned against tests/golden/din_*.npz, which tests/golden/make_golden.py
produced by running the reference's own DIN.py (see test_oracle_din.py).

Parameters use the reference's state_dict names (DIN.py:97-101,117-122):
  attn.attn.0.weight (A, 2d)  attn.attn.0.bias (A)  attn.attn.2.weight (1, A)  attn.attn.2.bias (1)
  fc.0 BN(2d)  fc.1 Linear(2d, F)  fc.4 BN(F)  fc.5 Linear(F, F/2)  fc.8 BN(F/2)  fc.9 Linear(F/2, 1)
"""
from __future__ import annotations

import numpy as np

BN_EPS = 1e-5
LINEARS = ("fc.1", "fc.5", "fc.9")
BNS = ("fc.0", "fc.4", "fc.8")


def _f64(p: dict) -> dict:
    return {k: np.asarray(v, dtype=np.float64) for k, v in p.items()}


def attention_forward(query, keys, W1, b1, W2, b2):
    """DIN.py:103-111.  s_j = W2 relu(W1 [q; k_j] + b1) + b2 over ALL L slots
    (zero padding rows included: no mask, DIN.py:108), alpha = softmax_j(s),
    out = sum_j alpha_j k_j.  Returns (out, alpha, cache)."""
    q = np.asarray(query, np.float64)
    k = np.asarray(keys, np.float64)
    b, L, d = k.shape
    W1 = np.asarray(W1, np.float64)
    z = (q @ W1[:, :d].T)[:, None, :] + k @ W1[:, d:].T + np.asarray(b1, np.float64)  # (b, L, A)
    h = np.maximum(z, 0.0)
    s = h @ np.asarray(W2, np.float64).reshape(-1) + float(np.asarray(b2).reshape(-1)[0])  # (b, L)
    s = s - s.max(axis=1, keepdims=True)
    e = np.exp(s)
    alpha = e / e.sum(axis=1, keepdims=True)
    out = np.einsum("bl,bld->bd", alpha, k)
    return out, alpha, (q, k, z, h, alpha)


def attention_backward(dout, cache, W1, W2):
    """Gradients of AttentionLayer w.r.t. its parameters (inputs are frozen
    embeddings in the reference, so no input gradient is needed)."""
    q, k, z, h, alpha = cache
    d = k.shape[2]
    w2 = np.asarray(W2, np.float64).reshape(-1)
    dalpha = np.einsum("bd,bld->bl", dout, k)
    ds = alpha * (dalpha - (alpha * dalpha).sum(axis=1, keepdims=True))
    dW2 = np.einsum("bl,bla->a", ds, h)[None, :]
    db2 = np.array([ds.sum()])
    dz = ds[..., None] * w2 * (z > 0)
    dW1k = np.einsum("bla,bld->ad", dz, k)
    dU = dz.sum(axis=1)
    dW1q = dU.T @ q
    db1 = dU.sum(axis=0)
    dW1 = np.concatenate([dW1q, dW1k], axis=1)
    return {"attn.attn.0.weight": dW1, "attn.attn.0.bias": db1, "attn.attn.2.weight": dW2,
            "attn.attn.2.bias": db2}, dU, dW1k


def _bn_forward(x, p, name, train):
    g, beta = p[f"{name}.weight"], p[f"{name}.bias"]
    if train:
        mu = x.mean(axis=0)
        var = x.var(axis=0)  # biased, used for normalisation (torch BatchNorm1d)
    else:
        mu, var = p[f"{name}.running_mean"], p[f"{name}.running_var"]
    inv = 1.0 / np.sqrt(var + BN_EPS)
    xh = (x - mu) * inv
    return xh * g + beta, (xh, inv, g)


def _bn_backward(dy, cache, train):
    xh, inv, g = cache
    dg = (dy * xh).sum(axis=0)
    db = dy.sum(axis=0)
    dxh = dy * g
    if not train:
        return dxh * inv, dg, db
    n = dy.shape[0]
    dx = inv / n * (n * dxh - dxh.sum(axis=0) - xh * (dxh * xh).sum(axis=0))
    return dx, dg, db


def din_forward(p, query, history, train=False):
    """DIN.py:130-133: fc(cat[q, attn(q, h)]).  Dropout is identity in eval mode
    and must be p=0 in train mode for a deterministic restatement."""
    p = _f64(p)
    pooled, alpha, acache = attention_forward(query, history, p["attn.attn.0.weight"], p["attn.attn.0.bias"],
                                              p["attn.attn.2.weight"], p["attn.attn.2.bias"])
    x = np.concatenate([np.asarray(query, np.float64), pooled], axis=1)
    caches = {"attn": acache}
    y, caches["fc.0"] = _bn_forward(x, p, "fc.0", train)
    caches["in.fc.1"] = y
    y = y @ p["fc.1.weight"].T + p["fc.1.bias"]
    caches["pre.relu1"] = y
    y = np.maximum(y, 0.0)
    y, caches["fc.4"] = _bn_forward(y, p, "fc.4", train)
    caches["in.fc.5"] = y
    y = y @ p["fc.5.weight"].T + p["fc.5.bias"]
    caches["pre.relu2"] = y
    y = np.maximum(y, 0.0)
    y, caches["fc.8"] = _bn_forward(y, p, "fc.8", train)
    caches["in.fc.9"] = y
    logits = y @ p["fc.9.weight"].T + p["fc.9.bias"]
    return logits, pooled, alpha, caches


def bce_with_logits(logits, labels):
    """Mean binary cross-entropy with logits (numerically stable form)."""
    x = np.asarray(logits, np.float64)
    y = np.asarray(labels, np.float64)
    return float(np.mean(np.maximum(x, 0) - x * y + np.log1p(np.exp(-np.abs(x)))))


def din_backward(p, caches, logits, labels, train=True):
    """Gradients of mean BCE w.r.t. every DIN parameter (DIN.py:148-149)."""
    p = _f64(p)
    x = np.asarray(logits, np.float64)
    y = np.asarray(labels, np.float64)
    g = {}
    dl = (1.0 / (1.0 + np.exp(-x)) - y) / x.size
    g["fc.9.weight"] = dl.T @ caches["in.fc.9"]
    g["fc.9.bias"] = dl.sum(axis=0)
    dy = dl @ p["fc.9.weight"]
    dy, g["fc.8.weight"], g["fc.8.bias"] = _bn_backward(dy, caches["fc.8"], train)
    dy = dy * (caches["pre.relu2"] > 0)
    g["fc.5.weight"] = dy.T @ caches["in.fc.5"]
    g["fc.5.bias"] = dy.sum(axis=0)
    dy = dy @ p["fc.5.weight"]
    dy, g["fc.4.weight"], g["fc.4.bias"] = _bn_backward(dy, caches["fc.4"], train)
    dy = dy * (caches["pre.relu1"] > 0)
    g["fc.1.weight"] = dy.T @ caches["in.fc.1"]
    g["fc.1.bias"] = dy.sum(axis=0)
    dy = dy @ p["fc.1.weight"]
    dy, g["fc.0.weight"], g["fc.0.bias"] = _bn_backward(dy, caches["fc.0"], train)
    d = caches["attn"][1].shape[2]
    ag, _, _ = attention_backward(dy[:, d:], caches["attn"], p["attn.attn.0.weight"], p["attn.attn.2.weight"])
    g.update(ag)
    return g


def clip_grad_norm(grads: dict, max_norm=1.0):
    """torch.nn.utils.clip_grad_norm_ (DIN.py:150): total 2-norm over all
    parameter grads, scale by min(1, max_norm / (norm + 1e-6))."""
    total = np.sqrt(sum(float((v * v).sum()) for v in grads.values()))
    coef = min(1.0, max_norm / (total + 1e-6))
    return {k: v * coef for k, v in grads.items()}, total


def adam_step(params: dict, grads: dict, state: dict, lr, weight_decay, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.Adam with L2 weight decay (NOT AdamW), DIN.py:245."""
    b1, b2 = betas
    t = state.get("step", 0) + 1
    state["step"] = t
    out = {}
    for k, pv in params.items():
        gk = grads[k] + weight_decay * pv
        m = state.setdefault(f"m.{k}", np.zeros_like(pv))
        v = state.setdefault(f"v.{k}", np.zeros_like(pv))
        m[...] = b1 * m + (1 - b1) * gk
        v[...] = b2 * v + (1 - b2) * gk * gk
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        out[k] = pv - (lr / bc1) * m / (np.sqrt(v) / np.sqrt(bc2) + eps)
    return out


def ndcg_single(probs, labels, k=5):
    """DIN.py:181-189: rank candidates by prob descending, NDCG of the single
    positive = 1/log2(rank+1) if within the top k, else 0.  numpy's default
    argsort (DIN.py:183) is not stable; this restatement breaks exact ties by
    candidate position (stable) — exact-tie parity is unpinned."""
    order = np.argsort(-np.asarray(probs, np.float64), kind="stable")[:k]
    for rank, idx in enumerate(order, start=1):
        if labels[idx] == 1:
            return 1.0 / np.log2(rank + 1)
    return 0.0
