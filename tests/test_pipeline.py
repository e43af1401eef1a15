"""Retrieval -> DIN re-rank (SURVEY §8f rank 1, configs[4]).  CPU: candidate
list semantics of Retrieval.py:28-34 / finialize_retrieval.py.  GPU: the
batched re-rank reproduces the reference's per-user evaluate() (logits and
NDCG@5 from the golden fixture made by DIN.py itself), and the end-to-end
retrieve+rerank equals the oracle composition."""
import os

import numpy as np
import pytest
import torch

from tests.conftest import GOLDEN


def test_finalize_candidates_appends_missing_ground_truth():
    from newsrecommend_amd.pipeline import finalize_candidates

    recs = {1: np.array([5, 6, 7]), 2: np.array([8, 9]), 3: np.arange(500)}
    out = finalize_candidates(recs, {1: 6, 2: 4})
    assert out[1].tolist() == [5, 6, 7] and out[2].tolist() == [8, 9, 4]
    assert len(out[3]) == 500  # the reference's 400-cap line has no effect (its result is discarded)


def test_pad_candidates():
    from newsrecommend_amd.pipeline import pad_candidates

    rows, mask = pad_candidates([[10, 11], [12], []], {10: 0, 11: 1, 12: 2})
    assert rows.tolist() == [[0, 1], [2, -1], [-1, -1]]
    assert mask.sum().item() == 3


def test_folded_eval_head_equals_module():
    """The re-rank head with each eval-mode BatchNorm folded into the next
    Linear equals DIN.fc (DIN.py:200-204) in eval mode."""
    from newsrecommend_amd.din import DIN
    from newsrecommend_amd.pipeline import _fold_eval_head

    torch.manual_seed(0)
    m = DIN(32, 16, 32, 0.36).eval()
    with torch.no_grad():
        for bn in (m.fc[0], m.fc[4], m.fc[8]):
            bn.running_mean.uniform_(-0.3, 0.3)
            bn.running_var.uniform_(0.5, 1.5)
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.2, 0.2)
        x = torch.randn(257, 64)
        (H1, c1), (H2, c2), (H3, c3) = _fold_eval_head(m.fc)
        h = torch.relu(x[:, :32] @ H1[:, :32].t() + x[:, 32:] @ H1[:, 32:].t() + c1)
        y = torch.relu(h @ H2.t() + c2) @ H3.t() + c3
        torch.testing.assert_close(y, m.fc(x), atol=1e-5, rtol=1e-5)


def _eval_world():
    from newsrecommend_amd.din import DIN

    z = np.load(os.path.join(GOLDEN, "din_dataset.npz"))
    row = {int(a): i for i, a in enumerate(z["item_ids"])}
    hist = np.vectorize(lambda a: row.get(int(a), -1))(z["ev_hist"]).astype(np.int32)
    cands, o = [], 0
    for n in z["ev_cand_len"]:
        cands.append(z["ev_cand"][o:o + n])
        o += n
    m = DIN(int(z["d"]), 32, 32, 0.36)
    m.load_state_dict({k[4:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd::")})
    return z, row, hist, cands, m


@pytest.mark.gpu
def test_rerank_matches_reference_evaluate(gpu):
    from newsrecommend_amd.pipeline import ndcg_at_k, pad_candidates, rerank

    z, row, hist, cands, m = _eval_world()
    m = m.cuda()
    table = torch.from_numpy(z["table"]).cuda()
    crow, mask = pad_candidates(cands, row, device="cuda")
    logits = rerank(m, table, torch.from_numpy(hist).cuda(), crow)
    flat = logits[mask].cpu().numpy()
    np.testing.assert_allclose(flat, z["ev_logits"], atol=1e-4)
    labs, o = torch.zeros_like(logits), 0
    for i, n in enumerate(z["ev_cand_len"]):
        labs[i, :n] = torch.from_numpy(z["ev_lab"][o:o + n].astype(np.float32))
        o += n
    nd = ndcg_at_k(logits, labs, 5)
    assert abs(nd.mean().item() - float(z["ev_ndcg"])) < 1e-9


@pytest.mark.gpu
def test_retrieve_and_rerank_end_to_end(gpu):
    from newsrecommend_amd import faiss as nf
    from newsrecommend_amd.din import DIN
    from newsrecommend_amd.pipeline import retrieve_and_rerank
    from oracle import knn_oracle as ko

    rng = np.random.default_rng(3)
    n_items, d, U, L = 30_000, 64, 40, 12
    table = (rng.standard_normal((n_items, d)) * 0.5).astype(np.float32)
    hist = rng.integers(0, n_items, (U, L)).astype(np.int32)
    hist[:, 9:] = -1
    profiles = table[np.maximum(hist, 0)].mean(1).astype(np.float32)
    gt = rng.integers(0, n_items, U).astype(np.int32)
    idx = nf.IndexFlatIP(d)
    idx.add(table)
    torch.manual_seed(0)
    m = DIN(d, 32, 32, 0.0).cuda().eval()
    T = torch.from_numpy(table).cuda()
    top, logits, cand, nd = retrieve_and_rerank(idx, m, T, torch.from_numpy(profiles).cuda(),
                                                torch.from_numpy(hist).cuda(), 50, 5, torch.from_numpy(gt).cuda())
    _, Io, _ = ko.exact_search(profiles, table, 50, ko.METRIC_IP)
    np.testing.assert_array_equal(cand[:, :50].cpu().numpy(), Io)
    for u in range(U):  # appended ground truth only when missing
        assert (cand[u] == gt[u]).sum().item() == 1
    # logits equal a plain per-user DIN forward
    with torch.no_grad():
        for u in (0, 17):
            c = cand[u][cand[u] >= 0].long()
            keys = torch.where(torch.from_numpy(hist[u]).cuda()[None, :, None] >= 0,
                               T[torch.from_numpy(np.maximum(hist[u], 0)).cuda().long()][None], 0.0)
            ref = m(T[c], keys.expand(len(c), -1, -1)).view(-1)
            torch.testing.assert_close(logits[u][cand[u] >= 0], ref, atol=1e-5, rtol=1e-5)
    assert nd.shape == (U,) and top.shape == (U, 5)


@pytest.mark.gpu
@pytest.mark.parametrize("d,L,C", [(256, 50, 201), (64, 20, 37), (128, 64, 70)])
def test_rerank_shared_history_matches_per_candidate(d, L, C):
    """nrk_din_rerank_attn (P = K W1k^T once per user) == every candidate as
    its own DIN sample (the generic attention kernel), eval mode, bf16 table;
    padded histories and padded candidates included."""
    from newsrecommend_amd.din import DIN
    from newsrecommend_amd.pipeline import rerank

    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(5)
    N, U = 5000, 37
    table = (torch.randn((N, d), generator=g, device=dev) * 0.5).to(torch.bfloat16)
    hist = torch.randint(0, N, (U, L), generator=g, device=dev, dtype=torch.int32)
    lens = torch.randint(1, L + 1, (U,), generator=g, device=dev)
    hist = torch.where(torch.arange(L, device=dev)[None] < lens[:, None], hist, torch.full_like(hist, -1))
    cand = torch.randint(0, N, (U, C), generator=g, device=dev, dtype=torch.int32)
    cand[:, -3:] = -1
    torch.manual_seed(0)
    model = DIN(d, 128, 32, 0.0).to(dev).eval()
    with torch.no_grad():  # non-trivial BN statistics
        for bn in (model.fc[0], model.fc[4], model.fc[8]):
            bn.running_mean.uniform_(-0.2, 0.2)
            bn.running_var.uniform_(0.5, 1.5)
    a = rerank(model, table, hist, cand, shared=True)
    b = rerank(model, table, hist, cand, shared=False)
    fin = torch.isfinite(b)
    assert torch.equal(fin, torch.isfinite(a))
    err = (a[fin] - b[fin]).abs().max().item()
    assert err < 2e-3 * max(1.0, b[fin].abs().max().item()), err


@pytest.mark.gpu
@pytest.mark.parametrize("d,NO,n", [(256, 160, 1000), (128, 128, 77), (64, 256, 33)])
def test_item_proj_matches_fp64(d, NO, n):
    """nrk_din_item_proj (gathered bf16 rows x W^T + bias, W as bf16 hi + lo)
    vs fp64 on the same rows; invalid ids give the bias."""
    from newsrecommend_amd import _lib
    from newsrecommend_amd.pipeline import _split_bf16

    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(7)
    N = 3000
    table = torch.randn((N, d), generator=g, device=dev).to(torch.bfloat16)
    ids = torch.randint(0, N, (n,), generator=g, device=dev, dtype=torch.int32)
    ids[::7] = -1
    ids[3::11] = N + 5
    W = torch.randn((NO, d), generator=g, device=dev) * 0.1
    b = torch.randn(NO, generator=g, device=dev)
    hi, lo = _split_bf16(W)
    out = torch.empty((n, NO), device=dev)
    _lib.check(_lib.load().nrk_din_item_proj(_lib.ptr(table), N, _lib.NRK_DTYPE_BF16, _lib.ptr(ids), n, d,
                                             _lib.ptr(hi), _lib.ptr(lo), _lib.ptr(b), NO, _lib.ptr(out),
                                             _lib.stream(dev)), "item_proj")
    ok = (ids >= 0) & (ids < N)
    q = torch.where(ok[:, None], table[ids.clamp(0, N - 1).long()].double(), 0.0)
    ref = q @ W.double().t() + b.double()
    bound = (q.abs() @ W.double().abs().t()).max().item() * 2.0 ** -15 + 1e-6
    err = (out.double() - ref).abs().max().item()
    assert err <= bound, (err, bound)
    assert torch.equal(out[~ok], b.expand(int((~ok).sum()), NO))


@pytest.mark.gpu
@pytest.mark.parametrize("d", [256, 64])
def test_rerank_head_matches_fp64(d):
    """nrk_din_rerank_head (pooled H1p on MFMA with hi/lo splits, two small
    layers per lane) vs the fp64 composition; -inf on padded candidates."""
    from newsrecommend_amd import _lib
    from newsrecommend_amd.pipeline import _split_bf16

    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(9)
    n, F, ldq = 301, 32, 160
    pooled = torch.randn((n, d), generator=g, device=dev)
    Q = torch.randn((n, ldq), generator=g, device=dev)
    cand = torch.randint(0, 100, (n,), generator=g, device=dev, dtype=torch.int32)
    cand[::9] = -1
    H1p = torch.randn((F, d), generator=g, device=dev) * 0.1
    c1 = torch.randn(F, generator=g, device=dev) * 0.1
    H2 = torch.randn((F // 2, F), generator=g, device=dev) * 0.3
    c2 = torch.randn(F // 2, generator=g, device=dev) * 0.1
    h3 = torch.randn(F // 2, generator=g, device=dev) * 0.3
    c3 = 0.25
    hi, lo = _split_bf16(H1p)
    lg = torch.empty(n, device=dev)
    off = 128  # Q1 = columns 128..159 of each Q row
    _lib.check(_lib.load().nrk_din_rerank_head(_lib.ptr(pooled), n, d, _lib.ptr(Q) + 4 * off, ldq, _lib.ptr(cand),
                                               _lib.ptr(hi), _lib.ptr(lo), _lib.ptr(c1), F, _lib.ptr(H2),
                                               _lib.ptr(c2), _lib.ptr(h3), c3, _lib.ptr(lg), _lib.stream(dev)),
               "rerank_head")
    p64 = pooled.double()
    h1 = (Q[:, off:off + F].double() + p64 @ H1p.double().t() + c1.double()).relu()
    h2 = (h1 @ H2.double().t() + c2.double()).relu()
    ref = h2 @ h3.double() + c3
    valid = cand >= 0
    assert torch.isneginf(lg[~valid]).all()
    err = (lg[valid].double() - ref[valid]).abs().max().item()
    assert err < 1e-4 * max(1.0, ref.abs().max().item()), err


def test_top_and_ndcg_equal_stable_sort_and_segment_ndcg():
    """CPU: the e2e ranking tail (key top-k + row-sum NDCG) equals a stable
    descending sort and din.ndcg_from_logits's segment formulation, with exact
    ties, -inf padding, +/-0 logits and users without a positive."""
    import torch

    from newsrecommend_amd.din import ndcg_from_logits
    from newsrecommend_amd.pipeline import _top_and_ndcg

    g = torch.Generator().manual_seed(3)
    U, C = 300, 37
    logits = torch.randn((U, C), generator=g)
    logits[:, 5] = logits[:, 2]
    logits[:10, :4] = 0.0
    logits[:10, 4] = -0.0
    logits[::3, -1] = float("-inf")
    cand = torch.randint(0, 1 << 20, (U, C), generator=g, dtype=torch.int32)
    labels = torch.zeros((U, C), dtype=torch.bool)
    labels[torch.arange(U), torch.randint(0, C, (U,), generator=g)] = True
    labels[::5] = False
    top, nd = _top_and_ndcg(logits, cand, labels, 5)
    order = torch.sort(logits, dim=1, descending=True, stable=True).indices[:, :5]
    assert torch.equal(top, torch.gather(cand, 1, order))
    seg = torch.arange(U).repeat_interleave(C)
    ref = ndcg_from_logits(logits.reshape(-1), labels.reshape(-1).float(), seg, U, 5)
    assert torch.equal(nd, ref)
