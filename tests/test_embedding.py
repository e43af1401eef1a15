"""Article embedding producer (embedding_generate.py:51-131) against the
golden fixture made by running the reference's own inference()
(tests/golden/make_golden.py:embedding_fixture): same state_dict keys, BN-folded
batched inference within fp32 GEMM reordering tolerance (1e-5 abs), typed
corpus files that Retrieval.py's loader can read (the reference's object
array cannot: fixture flag table_loadable == False)."""
import os
import random

import numpy as np
import pytest
import torch

from tests.conftest import GOLDEN


def _model(z):
    from newsrecommend_amd.embedding import ArticleEmbeddingModel

    m = ArticleEmbeddingModel(253, 512, 256, 0.13)
    m.load_state_dict({k[4:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd::")})
    return m.eval()


def test_state_dict_keys_and_eval_forward_cpu():
    z = np.load(os.path.join(GOLDEN, "embedding_infer.npz"))
    m = _model(z)
    assert set(m.state_dict()) == {k[4:] for k in z.files if k.startswith("sd::")}
    with torch.no_grad():
        y = m(torch.from_numpy(z["feats"])).numpy()
    np.testing.assert_allclose(y, z["emb"], atol=1e-5, rtol=0)


def test_article_table_loader(tmp_path):
    """Retrieval.py:6-9's loader over the typed .npz inference() writes and a
    plain numeric (N, d+1) table; the reference's own object-array table is
    not loadable (fixture flag)."""
    from newsrecommend_amd.embedding import load_article_table

    z = np.load(os.path.join(GOLDEN, "embedding_infer.npz"))
    path = str(tmp_path / "article_table.npz")
    np.savez(path, ids=z["aids"], emb=z["emb"])
    ids, emb = load_article_table(path)
    np.testing.assert_array_equal(ids, z["aids"])
    np.testing.assert_array_equal(emb, z["emb"])
    num = str(tmp_path / "table.npy")
    np.save(num, np.concatenate([z["emb"].astype(np.float64), z["aids"][:, None]], 1))
    ids2, emb2 = load_article_table(num)
    np.testing.assert_array_equal(ids2, z["aids"])
    np.testing.assert_array_equal(emb2, z["emb"])
    assert not bool(z["table_loadable"])  # the reference's own table fails Retrieval.py:6


def test_embed_refuses_host_tensors():
    from newsrecommend_amd._lib import NrkError

    z = np.load(os.path.join(GOLDEN, "embedding_infer.npz"))
    with pytest.raises(NrkError, match="GPU"):
        _model(z).embed(torch.from_numpy(z["feats"]))


@pytest.mark.gpu
def test_typed_inference_and_loader_gpu(gpu, tmp_path):
    """inference() (embedding_generate.py:109-131) through nrk_embed: the
    reference's own output to 1e-5 (measured: the fp32 level), typed .npz
    read back by the loader."""
    from newsrecommend_amd.embedding import inference, load_article_table

    z = np.load(os.path.join(GOLDEN, "embedding_infer.npz"))
    m = _model(z).cuda()
    feats = {int(a): z["feats"][i] for i, a in enumerate(z["aids"])}
    path = str(tmp_path / "article_table.npz")
    ids, emb = inference(m, feats, device=torch.device("cuda"), out_path=path)
    np.testing.assert_array_equal(ids, z["aids"])
    err = float(np.abs(emb - z["emb"]).max())
    print(f"nrk_embed vs the reference's inference(): {err:.3g}")
    assert err < 1e-5, err
    ids2, emb2 = load_article_table(path)
    np.testing.assert_array_equal(ids2, ids)
    np.testing.assert_array_equal(emb2, emb)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 64, 65, 4097])
def test_embed_kernel_vs_fp64_ragged_rows(gpu, n):
    """nrk_embed against the fp64 evaluation of the same folded model on
    random features (row counts around the 64-row tile, a strided x view):
    fp32-level error (<= 2e-6 relative to the output scale)."""
    from newsrecommend_amd.embedding import ArticleEmbeddingModel

    torch.manual_seed(n)
    m = ArticleEmbeddingModel().cuda().eval()
    with torch.no_grad():
        m.fc[3].running_mean.uniform_(-0.2, 0.2)
        m.fc[3].running_var.uniform_(0.5, 1.5)
    big = torch.randn(n, 300, device="cuda") * 2
    x = big[:, 5:258]  # rows 300 floats apart
    y = m.embed(x).double().cpu()
    W1, b1, W2, b2 = (p.detach().double().cpu() for p in m.folded())
    ref = torch.relu(x.double().cpu() @ W1.t() + b1) @ W2.t() + b2
    err = float((y - ref).abs().max())
    assert err <= 2e-6 * max(1.0, float(ref.abs().max())), err


def test_triplet_dataset_semantics():
    from newsrecommend_amd.embedding import ArticleTripletDataset

    clicks = {1: [10, 11, 12], 2: [13], 3: [14, 15]}
    ds = ArticleTripletDataset(clicks, list(range(10, 30)), rng=random.Random(0))
    t = ds.triplets
    assert len(ds) == 3 + 1
    assert [tuple(r[:2]) for r in t] == [(10, 11), (10, 12), (11, 12), (14, 15)]
    assert all(r[2] not in clicks[1] for r in t[:3]) and t[3][2] not in (14, 15)


@pytest.mark.gpu
def test_embed_gpu_and_triplet_step(gpu):
    from newsrecommend_amd.embedding import ArticleEmbeddingModel, train_triplet

    z = np.load(os.path.join(GOLDEN, "embedding_infer.npz"))
    m = _model(z).cuda()
    y = m.embed(torch.from_numpy(z["feats"]).cuda()).cpu().numpy()
    np.testing.assert_allclose(y, z["emb"], atol=1e-5, rtol=0)
    torch.manual_seed(0)
    mt = ArticleEmbeddingModel().cuda()
    feats = torch.randn(40, 253, device="cuda")
    id_to_row = {100 + i: i for i in range(40)}
    trip = np.array([[100 + i, 100 + (i + 1) % 40, 100 + (i + 7) % 40] for i in range(40)])
    opt = torch.optim.Adam(mt.parameters(), lr=1e-3, weight_decay=5e-5)
    l0 = train_triplet(mt, trip, id_to_row, feats, opt, batch_size=8)
    l1 = train_triplet(mt, trip, id_to_row, feats, opt, batch_size=8)
    assert np.isfinite(l0) and l1 < l0


def _fixture_logs(z):
    from newsrecommend_amd.data import ClickLog

    def log(prefix):
        lens = z[f"{prefix}_click_len"]
        off = np.concatenate([[0], np.cumsum(lens)])
        return ClickLog(z[f"{prefix}_users"], off, z[f"{prefix}_clicks"])

    return log("train"), log("test")


def _epoch_losses(z):
    """per-epoch (train, eval) as main() computes them (embedding_generate.py:90-103)"""
    v, rows, tr = z["loss_values"], z["loss_rows"], z["loss_train"]
    out, i = [], 0
    while i < len(v):
        j = i
        while j < len(v) and tr[j]:
            j += 1
        k = j
        while k < len(v) and not tr[k]:
            k += 1
        out.append((float(np.sum(v[i:j] * rows[i:j])) / (j - i), float(np.sum(v[j:k] * rows[j:k])) / (k - j)))
        i = k
    return out


def test_fit_triplet_matches_reference_main(tmp_path):
    """The reference's main() (embedding_generate.py:67-107) run as written on
    a synthetic world (tests/golden/embedding_train.npz): triplets from the
    typed click logs under the same `random` seed, then fit_triplet on the CPU
    under the same torch seed: the same batches, dropout masks and Adam
    steps, so every epoch's train/eval loss and the best-eval-loss checkpoint
    match the reference's."""
    from newsrecommend_amd.embedding import ArticleEmbeddingModel, ArticleTripletDataset, fit_triplet

    z = np.load(os.path.join(GOLDEN, "embedding_train.npz"))
    seed = int(z["seed"])
    tr_log, te_log = _fixture_logs(z)
    rng = random.Random(seed)
    tr = ArticleTripletDataset.from_click_log(tr_log, z["aids"], rng).triplets
    te = ArticleTripletDataset.from_click_log(te_log, z["aids"], rng).triplets
    np.testing.assert_array_equal(tr, z["train_triplets"])
    np.testing.assert_array_equal(te, z["test_triplets"])
    torch.manual_seed(seed)
    m = ArticleEmbeddingModel()
    path = str(tmp_path / "best_eg_model.pth")
    nt = torch.get_num_threads()
    torch.set_num_threads(4)  # as make_golden.py: CPU sgemm blocking follows the thread count
    try:
        hist, best = fit_triplet(m, tr, te, z["aids"], torch.from_numpy(z["feats"]), save_path=path)
    finally:
        torch.set_num_threads(nt)
    np.testing.assert_allclose(np.array(hist), np.array(_epoch_losses(z)), rtol=1e-6, atol=0)
    saved = torch.load(path, weights_only=True)
    for k, v in best.items():
        np.testing.assert_allclose(v.numpy(), z[f"best::{k}"], rtol=0, atol=1e-6, err_msg=k)
        np.testing.assert_array_equal(saved[k].numpy(), v.numpy())


@pytest.mark.gpu
def test_fit_triplet_on_device(gpu):
    """The reference's best checkpoint (embedding_train.npz) evaluated on the
    device reproduces main()'s best eval loss: Σ per-triplet losses / number
    of batches does not depend on the shuffled batch order.  Then fit_triplet
    runs with the features resident on the GPU (dropout masks come from the
    device RNG, so that trajectory is checked for finiteness and the
    best-checkpoint rule only)."""
    from newsrecommend_amd.embedding import ArticleEmbeddingModel, _triplet_rows, fit_triplet

    z = np.load(os.path.join(GOLDEN, "embedding_train.npz"))
    feats = torch.from_numpy(z["feats"]).to(gpu)
    m = ArticleEmbeddingModel().to(gpu)
    m.load_state_dict({k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("best::")})
    m.eval()
    r = _triplet_rows(z["test_triplets"], z["aids"], gpu)
    with torch.no_grad():
        per = torch.nn.TripletMarginLoss(margin=1.0, p=2, reduction="none")(*(m(feats[r[:, c]]) for c in range(3)))
    n_batches = -(-len(r) // 64)
    best_eval = min(e for _, e in _epoch_losses(z))
    np.testing.assert_allclose(per.double().sum().item() / n_batches, best_eval, rtol=1e-5)
    hist, best = fit_triplet(m, z["train_triplets"], z["test_triplets"], z["aids"], feats, epochs=2)
    assert np.all(np.isfinite(np.array(hist)))
    ev = [e for _, e in hist]
    assert best is not None and len(hist) == 2 and min(ev) <= ev[-1]
