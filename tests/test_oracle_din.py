"""CPU: pin the numpy DIN oracle against the golden fixtures produced by
running the reference's own DIN.py (tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

from oracle import din_oracle as o
from tests.conftest import GOLDEN


def _load(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"))


def _params(z, prefix="sd::"):
    return {k[len(prefix):]: z[k].astype(np.float64) for k in z.files
            if k.startswith(prefix) and "num_batches" not in k}


def _keys(table, idx):
    return np.where(idx[..., None] >= 0, table[np.maximum(idx, 0)], 0.0).astype(np.float32)


@pytest.mark.parametrize("name", ["din_fwd_c1", "din_fwd_c3"])
def test_forward_eval(name):
    z = _load(name)
    keys = _keys(z["table"], z["hist_idx"])
    logits, pooled, alpha, _ = o.din_forward(_params(z), z["query"], keys, train=False)
    np.testing.assert_allclose(logits, z["logits"], atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(pooled, z["pooled"], atol=1e-6, rtol=1e-5)
    np.testing.assert_allclose(alpha, z["alpha"], atol=1e-7, rtol=1e-5)
    # a fully padded history attends uniformly over the L zero rows (no mask, DIN.py:108)
    np.testing.assert_allclose(alpha[0], 1.0 / alpha.shape[1], rtol=1e-6)


@pytest.mark.parametrize("name", ["din_train_c1", "din_train_c3"])
def test_backward_and_adam(name):
    z = _load(name)
    p = _params(z)
    params = {k: v for k, v in p.items() if "running" not in k}
    state, losses = {}, []
    for s in range(2):
        keys = _keys(z["table"], z[f"hist_idx{s}"])
        q = z["table"][z[f"tgt_idx{s}"]]
        full = dict(p)
        full.update(params)
        logits, _, _, cache = o.din_forward(full, q, keys, train=True)
        losses.append(o.bce_with_logits(logits, z[f"label{s}"]))
        g = o.din_backward(full, cache, logits, z[f"label{s}"])
        if s == 0:
            assert abs(losses[0] - z["loss0"]) < 1e-6
            for k, v in g.items():
                ref = z[f"grad::{k}"]
                np.testing.assert_allclose(v, ref, atol=2e-7 + 1e-5 * np.abs(ref).max(), err_msg=k)
        g, _ = o.clip_grad_norm(g, 1.0)
        params = o.adam_step(params, g, state, 1.62e-3, 8.96e-5)
    assert abs(np.mean(losses) - z["mean_loss"]) < 1e-6
    for k, v in params.items():
        # attn.attn.2.bias: its gradient is exactly 0 in exact arithmetic (softmax
        # shift invariance) and fp32 noise in the reference, so Adam moves it by
        # +-lr in a direction set by that noise
        tol = 2 * 1.62e-3 + 1e-6 if k == "attn.attn.2.bias" else 2e-5
        np.testing.assert_allclose(v, z[f"after::{k}"], atol=tol, err_msg=k)


def test_evaluate_ndcg():
    z = _load("din_dataset")
    logits = z["ev_logits"]
    lens = z["ev_cand_len"]
    labs = z["ev_lab"]
    offs = np.concatenate([[0], np.cumsum(lens)])
    nd, ls = [], []
    for u in range(len(lens)):
        lg = logits[offs[u]:offs[u + 1]].astype(np.float64)
        lb = labs[offs[u]:offs[u + 1]]
        probs = (1 / (1 + np.exp(-lg))).astype(np.float32)
        nd.append(o.ndcg_single(probs, lb, 5))
        ls.append(o.bce_with_logits(lg, lb))
    assert abs(np.mean(nd) - z["ev_ndcg"]) < 1e-9
    assert abs(np.mean(ls) - z["ev_loss"]) < 1e-6


@pytest.mark.parametrize("name", ["din_train_c1", "din_train_c3"])
def test_torch_cpu_restatement_pinned(name):
    """oracle/din_torch_ref (the PyTorch-CPU baseline the bench times) equals
    the reference's own two train() steps (DIN.py:139-153)."""
    import torch

    from oracle.din_torch_ref import TorchDIN, train_step

    z = _load(name)
    m = TorchDIN(int(z["d"]), int(z["A"]), int(z["F"]), 0.0)
    m.load_state_dict({k[4:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd::")})
    opt = torch.optim.Adam(m.parameters(), lr=1.62e-3, weight_decay=8.96e-5)
    crit = torch.nn.BCEWithLogitsLoss()
    m.train()
    losses = []
    for s in range(2):
        keys = torch.from_numpy(_keys(z["table"], z[f"hist_idx{s}"]))
        q = torch.from_numpy(z["table"][z[f"tgt_idx{s}"]].astype(np.float32))
        losses.append(train_step(m, opt, crit, q, keys, torch.from_numpy(z[f"label{s}"])).item())
    assert abs(losses[0] - float(z["loss0"])) < 1e-6
    assert abs(np.mean(losses) - float(z["mean_loss"])) < 1e-6
    for k, v in m.state_dict().items():
        if f"after::{k}" in z.files and "num_batches" not in k:
            # b2's gradient is 0 up to rounding (softmax shift invariance): Adam moves it by +-lr
            tol = 2 * 1.62e-3 if k == "attn.attn.2.bias" else 5e-5
            np.testing.assert_allclose(v.numpy(), z[f"after::{k}"], atol=tol, err_msg=k)


def test_cpu_baseline_ports_agree_with_exact_oracle():
    """oracle/cpu_baselines (the faiss-cpu stand-ins the bench times) return
    the exact oracle's neighbours on well-separated data."""
    import torch

    from oracle import cpu_baselines as cb, ivf_oracle as io, knn_oracle as ko

    rng = np.random.default_rng(0)
    c = rng.standard_normal((20, 24)).astype(np.float32) * 3
    xb = (c[rng.integers(0, 20, 3000)] + rng.standard_normal((3000, 24))).astype(np.float32)
    xq = (c[rng.integers(0, 20, 50)] + rng.standard_normal((50, 24))).astype(np.float32)
    for metric in (ko.METRIC_IP, ko.METRIC_L2):
        _, I = cb.flat_search(torch.from_numpy(xq), torch.from_numpy(xb), 5, metric, block=700)
        _, Io, _ = ko.exact_search(xq, xb, 5, metric)
        assert (I.numpy() == Io).mean() > 0.99
    cent = xb[:16].copy()
    assign, _ = io.assign_nearest(xb, cent)
    lists = cb.IvfLists(xb, assign, cent)
    for metric in (ko.METRIC_IP, ko.METRIC_L2):
        _, I = cb.ivf_search(torch.from_numpy(xq), lists, 4, 5, metric)
        _, Io, _, _ = io.ivf_search(xq, xb, cent, assign, 4, 5, metric)
        assert (I.numpy() == Io).mean() > 0.99
