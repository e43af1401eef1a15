"""CPU: the IVF / k-means oracle (oracle/ivf_oracle.py) against pure-Python
loop restatements on small cases.  faiss is absent offline, so the oracle is
pinned to faiss's published algorithm only (parity unpinned vs faiss itself;
DESIGN.md)."""
import numpy as np
import pytest

from oracle import ivf_oracle as io
from oracle import knn_oracle as ko


def test_group_by_list_stable_and_empty_lists():
    rng = np.random.default_rng(0)
    assign = rng.integers(0, 7, 1000)
    assign[assign == 3] = 4  # list 3 empty
    off, pos2id = io.group_by_list(assign, 9)
    assert off[0] == 0 and off[-1] == 1000 and off[4] == off[3]
    for l in range(9):
        ids = pos2id[off[l]:off[l + 1]].tolist()
        assert ids == [i for i in range(1000) if assign[i] == l]


def test_update_centroids_sequential_fp64_mean():
    rng = np.random.default_rng(1)
    x = rng.standard_normal((300, 5)).astype(np.float32)
    labels = rng.integers(0, 4, 300)
    labels[labels == 2] = 1
    prev = np.full((4, 5), 7.0, np.float32)
    c, counts = io.update_centroids(x, labels, prev)
    for j in range(4):
        members = [i for i in range(300) if labels[i] == j]
        assert counts[j] == len(members)
        if not members:
            assert (c[j] == 7.0).all()  # empty: untouched
            continue
        for t in range(5):
            acc = 0.0
            for i in members:
                acc += float(x[i, t])
            assert c[j, t] == np.float32(acc / len(members))


def test_split_refills_every_empty_cluster():
    c = np.arange(12, dtype=np.float32).reshape(4, 3) + 1
    counts = np.array([0, 10, 0, 6])
    out, nsplit = io.split_clusters(c.copy(), counts, 16)
    assert nsplit == 2
    # each refilled centroid is a +-1/1024 perturbation of a donor with members
    for ci in (0, 2):
        donors = [j for j in (1, 3) if np.allclose(out[ci], c[j], rtol=2e-3)]
        assert donors


def test_kmeans_objective_decreases_and_recovers_centres():
    rng = np.random.default_rng(2)
    centres = rng.standard_normal((8, 16)).astype(np.float32) * 4
    x = (centres[rng.integers(0, 8, 4000)] + 0.1 * rng.standard_normal((4000, 16))).astype(np.float32)
    cent, obj = io.kmeans(x, 8, niter=15, seed=1234, max_points_per_centroid=10_000)
    assert all(b <= a * (1 + 1e-9) for a, b in zip(obj, obj[1:]))
    d2 = ((cent[:, None, :] - centres[None]) ** 2).sum(-1)
    assert (d2.min(0) < 0.1).sum() >= 4  # k-means from a random init: local optima allowed


def test_kmeans_subsample_size():
    x = np.random.default_rng(3).standard_normal((5000, 4)).astype(np.float32)
    xs = io.subsample(x, 10, 39, seed=1234)
    assert xs.shape == (390, 4)
    assert len({tuple(r) for r in xs.tolist()}) == 390


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
def test_ivf_search_matches_python_loop(metric):
    rng = np.random.default_rng(4)
    xb = rng.standard_normal((400, 6)).astype(np.float32)
    xq = rng.standard_normal((7, 6)).astype(np.float32)
    cent = xb[:5].copy()
    assign, _ = io.assign_nearest(xb, cent)
    D, I, S, probe = io.ivf_search(xq, xb, cent, assign, 2, 4, metric)
    for q in range(7):
        # coarse: 2 nearest centroids (squared L2, ties lower id)
        dc = [(sum((float(xq[q, t]) - float(cent[c, t])) ** 2 for t in range(6)), c) for c in range(5)]
        probed = [c for _, c in sorted(dc)[:2]]
        assert sorted(probed) == sorted(probe[q].tolist())
        cand = []
        for i in range(400):
            if assign[i] in probed:
                if metric == ko.METRIC_IP:
                    s = sum(float(xq[q, t]) * float(xb[i, t]) for t in range(6))
                    cand.append((-s, i))
                else:
                    s = sum((float(xq[q, t]) - float(xb[i, t])) ** 2 for t in range(6))
                    cand.append((s, i))
        top = [i for _, i in sorted(cand)[:4]]
        assert I[q].tolist() == top


def test_ivf_search_all_lists_equals_flat():
    rng = np.random.default_rng(5)
    xb = rng.standard_normal((600, 8)).astype(np.float32)
    xq = rng.standard_normal((10, 8)).astype(np.float32)
    cent = xb[::60].copy()
    assign, _ = io.assign_nearest(xb, cent)
    D, I, S, _ = io.ivf_search(xq, xb, cent, assign, cent.shape[0], 5, ko.METRIC_L2)
    Df, If, Sf = ko.exact_search(xq, xb, 5, ko.METRIC_L2)
    np.testing.assert_array_equal(I, If)
    np.testing.assert_array_equal(D, Df)
