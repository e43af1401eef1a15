"""bench.py's CPU-baseline legs for the end-to-end records (host only, tiny sizes).

The legs time the reference's algorithm on the host cores (oracle/cpu_baselines.py,
oracle/din_torch_ref.py); these tests check that they run, report the contract's
fields, and that the per-user re-rank is the reference's per-user forward
(DIN.py:166-173: model(cand_emb, his.expand(C, -1, -1)), zero rows for padded slots)
whatever the candidate chunking.
"""
import types

import pytest
import torch

bench = pytest.importorskip("bench")


def _model(d):
    from newsrecommend_amd.din import DIN

    torch.manual_seed(3)
    return DIN(d, 128, 32, 0.36).eval()


def test_cpu_rerank_user_is_the_reference_forward_in_any_chunking():
    torch.manual_seed(0)
    n, d, L = 500, 64, 12
    xb = torch.randn(n, d)
    h = torch.randint(0, n, (L,))
    h[9:] = -1
    cand = torch.randint(0, n, (37,))
    m = bench._cpu_torch_din(_model(d), d, 128, 32)
    keys = torch.where(h[:, None] >= 0, xb[h.clamp_min(0)], 0.0)
    with torch.no_grad():
        ref = m(xb[cand], keys[None].expand(len(cand), -1, -1)).view(-1)
        for chunk in (1, 8, 1024):
            got = bench._cpu_rerank_user(m, xb, h, cand, chunk=chunk)
            assert torch.allclose(got, ref, atol=1e-5, rtol=1e-5), float((got - ref).abs().max())


def test_cpu_e2e_and_flow_legs_report_the_contract_fields():
    torch.manual_seed(1)
    n, d, U, L = 3000, 64, 24, 10
    table = torch.randn(n, d)
    hist = torch.randint(0, n, (U, L)).int()
    hist[:, 7:] = -1
    prof, gt = torch.randn(U, d), torch.randint(0, n, (U,)).int()
    model = _model(d)
    args = types.SimpleNamespace(cpu_seconds=0.2)
    r = bench._cpu_e2e(args, prof, table, hist, gt, model, 50)
    assert r["unit"] == "users/s" and r["kind"] == "port" and r["value"] > 0 and r["cores"] >= 1
    nl = 8
    assign = torch.randint(0, nl, (n,))
    rows = torch.sort(assign, stable=True).indices.int()
    off = torch.zeros(nl + 1, dtype=torch.int64)
    off[1:] = torch.cumsum(torch.bincount(assign, minlength=nl), 0)
    r = bench._cpu_flow(args, table, torch.randn(nl, d), off, rows, prof, hist.long(), gt.long(), model)
    assert r["unit"] == "users/s" and r["kind"] == "port" and r["value"] > 0 and "sample" in r
