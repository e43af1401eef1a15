"""CPU: the k-NN oracle (oracle/knn_exact.c) against an independent numpy
float64 restatement, on the edge cases the faiss contract has (ties, k > ntotal,
empty corpus, shard merge).  faiss itself is absent offline: parity unpinned."""
import numpy as np
import pytest

from oracle import knn_oracle as ko


def _data(nb, nq, d, seed=0, dups=True):
    rng = np.random.default_rng(seed)
    xb = rng.standard_normal((nb, d)).astype(np.float32)
    xq = rng.standard_normal((nq, d)).astype(np.float32)
    if dups and nb > 50:
        xb[40] = xb[3]
        xb[nb - 1] = xb[3]
        xq[0] = xb[3]
    return xq, xb


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
@pytest.mark.parametrize("k", [1, 5, 17])
def test_exact_matches_numpy(metric, k):
    xq, xb = _data(2000, 40, 24, seed=k)
    D, I, S = ko.exact_search(xq, xb, k, metric)
    S2, I2 = ko.numpy_search(xq, xb, k, metric)
    np.testing.assert_array_equal(I, I2)
    np.testing.assert_allclose(S, S2, rtol=1e-12, atol=1e-9)
    np.testing.assert_array_equal(D, S.astype(np.float32))


def test_ties_break_to_lower_id():
    xq, xb = _data(500, 3, 8)
    _, I, _ = ko.exact_search(xq, xb, 3, ko.METRIC_L2)
    assert I[0].tolist() == [3, 40, 499]


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
def test_k_larger_than_ntotal_pads(metric):
    xq, xb = _data(4, 2, 8, dups=False)
    D, I, _ = ko.exact_search(xq, xb, 7, metric)
    assert (I[:, 4:] == -1).all()
    pad = -np.finfo(np.float32).max if metric == ko.METRIC_IP else np.finfo(np.float32).max
    assert (D[:, 4:] == pad).all()
    D0, I0, _ = ko.exact_search(xq, xb[:0], 2, metric)
    assert (I0 == -1).all()


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
def test_shard_merge_equals_single_search(metric):
    xq, xb = _data(3001, 30, 16, seed=5)
    k = 9
    D, I, S = ko.exact_search(xq, xb, k, metric)
    bounds = [0, 700, 1500, 1501, 3001]
    parts = [ko.exact_search(xq, xb[a:b], k, metric, id_offset=a) for a, b in zip(bounds[:-1], bounds[1:])]
    Dm, Im, Sm = ko.merge(np.stack([p[2] for p in parts]), np.stack([p[1] for p in parts]), k, metric)
    np.testing.assert_array_equal(Im, I)
    np.testing.assert_array_equal(Sm, S)


def test_faiss_port_recall():
    xq, xb = _data(5000, 64, 32, seed=9, dups=False)
    _, I, _ = ko.exact_search(xq, xb, 5, ko.METRIC_IP)
    _, Ip = ko.faiss_port(xq, xb, 5, ko.METRIC_IP)
    assert np.mean([len(set(a) & set(b)) / 5 for a, b in zip(I, Ip)]) > 0.99
