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


def _din_model(d, A, F, dev, seed=0):
    from newsrecommend_amd.din import DIN

    torch.manual_seed(seed)
    model = DIN(d, A, F, 0.0).to(dev).eval()
    with torch.no_grad():  # non-trivial BN statistics and affines
        for bn in (model.fc[0], model.fc[4], model.fc[8]):
            bn.running_mean.uniform_(-0.2, 0.2)
            bn.running_var.uniform_(0.5, 1.5)
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.1, 0.1)
    return model


def _oracle_logits(model, T, hist_u, cand_u):
    """fp64 DIN eval forward (oracle/din_oracle.py) of one user's candidates."""
    from oracle import din_oracle as o

    p = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in model.state_dict().items()
         if "num_batches" not in k}
    keys = np.where(hist_u[:, None] >= 0, T[np.maximum(hist_u, 0)], 0.0)
    lo, _, _, _ = o.din_forward(p, T[cand_u], np.broadcast_to(keys, (len(cand_u),) + keys.shape), train=False)
    return lo.reshape(-1)


@pytest.mark.gpu
@pytest.mark.parametrize("d,L,C,A,F", [(256, 50, 201, 128, 32), (64, 20, 90, 32, 64), (128, 64, 70, 96, 128),
                                       (256, 64, 130, 64, 96), (128, 33, 37, 128, 32),
                                       # histories past 64 slots (max_history reaches 128, DIN.py:207):
                                       # the lane kernel's 128-row form
                                       (256, 128, 75, 128, 32), (128, 96, 40, 64, 64), (64, 100, 33, 32, 32),
                                       # ... where [P' | R^T] and H2 do not fit the LDS together (R and H2
                                       # read from global memory, the RG form): fc_units 96 / 128 and
                                       # (A, F) = (96, 64), (128, 64)
                                       (256, 128, 75, 128, 128), (256, 96, 70, 96, 64), (128, 100, 40, 128, 64),
                                       (64, 128, 33, 32, 96), (256, 65, 66, 64, 128)])
def test_rerank_fused_vs_oracle_and_per_candidate(d, L, C, A, F):
    """nrk_din_rerank over the reference's hyper-parameter space (Optuna
    DIN.py:203-204: attn_units and fc_units 32..128 step 32) against the fp64
    oracle (<= 1e-4 of the logit scale) and against every candidate as its own
    DIN sample (model.forward_ids: the same logits up to that path's bf16 W1k,
    2e-3); padded histories (an empty one included) and padded candidates.
    Candidate counts that are not multiples of the 32-candidate wave item, and
    histories of 65..128 slots (the 128-row form)."""
    from newsrecommend_amd.pipeline import rerank

    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(5)
    N, U = 5000, 37
    table = (torch.randn((N, d), generator=g, device=dev) * 0.5).to(torch.bfloat16)
    hist = torch.randint(0, N, (U, L), generator=g, device=dev, dtype=torch.int32)
    lens = torch.randint(1, L + 1, (U,), generator=g, device=dev)
    hist = torch.where(torch.arange(L, device=dev)[None] < lens[:, None], hist, torch.full_like(hist, -1))
    hist[1] = -1
    cand = torch.randint(0, N, (U, C), generator=g, device=dev, dtype=torch.int32)
    cand[:, -3:] = -1
    model = _din_model(d, A, F, dev)
    a = rerank(model, table, hist, cand)
    assert rerank.path == "fused", rerank.path
    b = rerank(model, table, hist, cand, shared=False)
    fin = torch.isfinite(b)
    assert torch.equal(fin, torch.isfinite(a))
    scale = max(1.0, b[fin].abs().max().item())
    assert (a[fin] - b[fin]).abs().max().item() < 2e-3 * scale
    T = table.float().cpu().numpy().astype(np.float64)
    H, Cn, A_ = hist.cpu().numpy(), cand.cpu().numpy(), a.cpu().numpy()
    worst = 0.0
    for u in range(0, U, 3):
        v = Cn[u] >= 0
        worst = max(worst, float(np.abs(A_[u][v] - _oracle_logits(model, T, H[u], Cn[u][v])).max()))
    print(f"fused re-rank d={d} A={A} F={F}: max abs err vs fp64 {worst:.3g}")
    assert worst < 1e-4 * scale, worst


@pytest.mark.gpu
@pytest.mark.parametrize("L", [40, 100])
def test_rerank_ragged_shared_lists_extra_and_gaps(L):
    """nrk_din_rerank's ragged form (the flow's): users sharing one candidate
    list (same offset), lists of 0, 1, 63, 64, 65 and 300 candidates, an
    appended extra candidate (-1 = a padded slot, a row past the table = -inf),
    duplicated candidates, out_off with gaps between users; every logit of the
    projected form (nrk_din_rerank_projected) equals the rectangular rerank()
    of the same list bit for bit, and the row-staged kernel (nrk_din_rerank,
    direct=True, L <= 64) agrees within 1e-4.  L = 100 (75 valid slots): the
    lane kernel's 128-row form."""
    from newsrecommend_amd.pipeline import rerank, rerank_ragged

    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(11)
    d, N = 128, 3000
    table = (torch.randn((N, d), generator=g, device=dev) * 0.5).to(torch.bfloat16)
    model = _din_model(d, 128, 32, dev, seed=3)
    pool = torch.randint(0, N, (600,), generator=g, device=dev, dtype=torch.int32)
    pool[10] = pool[11]  # a duplicate
    lists = [(0, 0), (5, 1), (20, 63), (20, 64), (100, 65), (200, 300), (20, 64), (0, 0)]  # (offset, length)
    extra = torch.tensor([7, -1, 12, N + 4, -1, 99, 5, -1], dtype=torch.int32, device=dev)
    U = len(lists)
    hist = torch.randint(0, N, (U, L), generator=g, device=dev, dtype=torch.int32)
    hist[:, (3 * L) // 4:] = -1
    hist[3] = -1
    co = torch.tensor([o for o, _ in lists], dtype=torch.int64, device=dev)
    cl = torch.tensor([n for _, n in lists], dtype=torch.int32, device=dev)
    width = cl.long() + 1
    oo = torch.cumsum(width + 3, 0) - (width + 3)  # gaps of 3 between users
    n_out = int((oo[-1] + width[-1]).item()) + 5
    got = rerank_ragged(model, table, hist, pool, co, cl, extra, oo, n_out, shared=True)  # projected lists
    # the row-staged kernel (nrk_din_rerank, histories <= 64): its own arithmetic
    # order, so equal to the projected form within the re-rank tolerance
    direct = rerank_ragged(model, table, hist, pool, co, cl, extra, oo, n_out, direct=True) if L <= 64 else None
    for u, (o, n) in enumerate(lists):
        lst = torch.cat([pool[o:o + n], extra[u:u + 1]])
        ref = rerank(model, table, hist[u:u + 1], lst[None])[0]
        seg = got[oo[u]:oo[u] + n + 1]
        assert torch.equal(seg, ref), u
        if direct is not None:
            dseg = direct[oo[u]:oo[u] + n + 1]
            fin = torch.isfinite(ref)
            assert torch.equal(torch.isneginf(dseg), torch.isneginf(ref)), u
            scale = max(1.0, ref[fin].abs().max().item()) if fin.any() else 1.0
            assert (dseg[fin] - ref[fin]).abs().max().item() <= 1e-4 * scale if fin.any() else True, u
        if extra[u] < 0 or extra[u] >= N:
            assert torch.isneginf(seg[-1])
    assert torch.equal(got[0:1], rerank(model, table, hist[:1], extra[:1, None])[0])  # list of 0 + extra


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
