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


def test_typed_inference_and_loader(tmp_path):
    from newsrecommend_amd.embedding import inference, load_article_table

    z = np.load(os.path.join(GOLDEN, "embedding_infer.npz"))
    m = _model(z)
    feats = {int(a): z["feats"][i] for i, a in enumerate(z["aids"])}
    path = str(tmp_path / "article_table.npz")
    ids, emb = inference(m, feats, device=torch.device("cpu"), out_path=path, batch=7)
    np.testing.assert_array_equal(ids, z["aids"])
    np.testing.assert_allclose(emb, z["emb"], atol=1e-5, rtol=0)
    ids2, emb2 = load_article_table(path)
    np.testing.assert_array_equal(ids2, ids)
    np.testing.assert_array_equal(emb2, emb)
    assert not bool(z["table_loadable"])  # the reference's own table fails Retrieval.py:6


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
    y = m.embed(torch.from_numpy(z["feats"]).cuda(), batch=16).cpu().numpy()
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
