"""GPU parity for the index-building half of retrieval (Retrieval.py:11-23)
and IVF-Flat search (BASELINE configs[3]) against oracle/ivf_oracle.py:
grouping by list and k-means centroids bit-exact, IVF indices bit-exact and D
equal to the fp32 rounding of the same fp64 scores."""
import numpy as np
import pytest
import torch

from oracle import ivf_oracle as io
from oracle import knn_oracle as ko

pytestmark = pytest.mark.gpu


def _mixture(nb, nq, d, seed, centers=64, sigma=0.35):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((centers, d)).astype(np.float32)
    xb = (c[rng.integers(0, centers, nb)] + sigma * rng.standard_normal((nb, d))).astype(np.float32)
    xq = (c[rng.integers(0, centers, nq)] + sigma * rng.standard_normal((nq, d))).astype(np.float32)
    return xq, xb


@pytest.mark.parametrize("n,nlist", [(1, 3), (4095, 5), (4096 * 3 + 17, 300), (50_000, 5000)])
def test_group_by_list(gpu, n, nlist):
    from newsrecommend_amd import _lib

    rng = np.random.default_rng(n)
    assign = rng.integers(0, nlist, n).astype(np.int64)
    if nlist > 4:
        assign[assign == 2] = 1  # an empty list
    L = _lib.load()
    a = torch.from_numpy(assign).cuda()
    off = torch.empty(nlist + 1, dtype=torch.int64, device="cuda")
    p2i = torch.empty(n, dtype=torch.int64, device="cuda")
    p2l = torch.empty(n, dtype=torch.int32, device="cuda")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")
    sz = _lib.c_size(0)
    _lib.check(L.nrk_group_by_list_workspace(n, nlist, sz))
    ws = torch.empty(sz.value, dtype=torch.uint8, device="cuda")
    _lib.check(L.nrk_group_by_list(_lib.ptr(a), n, nlist, _lib.ptr(off), _lib.ptr(p2i), _lib.ptr(p2l), _lib.ptr(bad),
                                   _lib.ptr(ws), ws.numel(), _lib.stream()))
    o_off, o_p2i = io.group_by_list(assign, nlist)
    np.testing.assert_array_equal(off.cpu().numpy(), o_off)
    np.testing.assert_array_equal(p2i.cpu().numpy(), o_p2i)
    np.testing.assert_array_equal(p2l.cpu().numpy(), assign[o_p2i])
    assert bad.item() == 0


@pytest.mark.parametrize("metric", [ko.METRIC_L2, ko.METRIC_IP])
def test_clustering_matches_oracle(gpu, metric):
    """faiss.Clustering semantics incl. subsampling (n > k * max_points) and
    the empty-cluster split (duplicated rows make the init pick twins)."""
    from newsrecommend_amd import faiss as nf

    _, x = _mixture(9000, 1, 32, seed=21, centers=20)
    x[1::7] = x[0]  # many exact duplicates -> twin centroids -> empty clusters
    k = 40
    cl = nf.Clustering(32, k)
    cl.niter = 6
    cl.max_points_per_centroid = 200  # 9000 > 40 * 200: subsample path
    idx = nf.IndexFlat(32, metric)
    cl.train(x, idx)
    cent, obj = io.kmeans(x, k, niter=6, seed=1234, max_points_per_centroid=200, metric=metric)
    np.testing.assert_array_equal(cl.centroids.cpu().numpy(), cent)
    np.testing.assert_allclose(cl.obj, obj, rtol=1e-9)
    assert sum(s["nsplit"] for s in cl.iteration_stats) > 0
    assert idx.ntotal == k  # the assignment index ends holding the centroids (faiss)


def _ivf(xb, nlist, metric, seed=0):
    from newsrecommend_amd import faiss as nf

    q = nf.IndexFlatL2(xb.shape[1])
    ivf = nf.IndexIVFFlat(q, xb.shape[1], nlist, metric)
    ivf.cp.niter = 4
    ivf.train(xb)
    ivf.add(xb)
    return ivf


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
@pytest.mark.parametrize("d,k,nprobe", [(64, 5, 8), (128, 10, 4), (96, 40, 16), (256, 5, 3), (128, 1, 1)])
def test_ivf_search_matches_oracle(gpu, metric, d, k, nprobe):
    xq, xb = _mixture(40_000, 300, d, seed=d + k)
    ivf = _ivf(xb, 50, metric)
    ivf.nprobe = nprobe
    D, I = ivf.search(xq, k)
    cent = ivf.quantizer._xb[:50].cpu().numpy()
    assign = ivf._assign.cpu().numpy()
    Do, Io, So, probe = io.ivf_search(xq, xb, cent, assign, nprobe, k, metric)
    np.testing.assert_array_equal(I, Io)
    np.testing.assert_array_equal(D, Do)
    assert ivf.max_list == int(np.bincount(assign, minlength=50).max())


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
@pytest.mark.parametrize("form", ["0", "1"])
def test_ivf_collect_forms(gpu, monkeypatch, metric, form):
    """Both phase-B collect kernels give the oracle's result: the 16x16x32
    screen16_collect_kernel (d = 128, k <= 8; the default) and the 32x32x16
    screen MODE 3 (NRK_SCREEN16=0, a test hook)."""
    monkeypatch.setenv("NRK_SCREEN16", form)
    xq, xb = _mixture(60_000, 700, 128, seed=77 + int(form))
    ivf = _ivf(xb, 40, metric)
    ivf.nprobe = 8
    D, I = ivf.search(xq, 5)
    cent = ivf.quantizer._xb[:40].cpu().numpy()
    assign = ivf._assign.cpu().numpy()
    Do, Io, _, _ = io.ivf_search(xq, xb, cent, assign, 8, 5, metric)
    np.testing.assert_array_equal(I, Io)
    np.testing.assert_array_equal(D, Do)


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
@pytest.mark.parametrize("force", ["0", "1"])
def test_ivf_collect16_small_lists(gpu, monkeypatch, metric, force):
    """The 16x16x32 collect (d = 128, k <= 8) on lists of a few dozen rows (one
    partial 64-row tile per chunk), a few probing queries per list (work items
    with 1-3 active half-tiles) and, with NRK_FORCE_FALLBACK=1, every query's
    candidate buffer overflowed into the IVF-aware fallback."""
    monkeypatch.setenv("NRK_FORCE_FALLBACK", force)
    xq, xb = _mixture(3_000, 50, 128, seed=91, centers=16)
    ivf = _ivf(xb, 40, metric)
    ivf.nprobe = 3
    D, I = ivf.search(xq, 5)
    Do, Io, _, _ = io.ivf_search(xq, xb, ivf.quantizer._xb[:40].cpu().numpy(), ivf._assign.cpu().numpy(), 3, 5,
                                 metric)
    np.testing.assert_array_equal(I, Io)
    np.testing.assert_array_equal(D, Do)
    if force == "1":
        assert int(ivf.last_fallback.item()) == 50


def test_ivf_all_lists_equals_flat_and_list_ids(gpu):
    from newsrecommend_amd import faiss as nf

    xq, xb = _mixture(30_000, 100, 64, seed=5)
    xb[20_000] = xb[11]
    xq[0] = xb[11]
    ivf = _ivf(xb, 20, ko.METRIC_L2)
    ivf.nprobe = 20
    D, I = ivf.search(xq, 7)
    Df, If, _ = ko.exact_search(xq, xb, 7, ko.METRIC_L2)
    np.testing.assert_array_equal(I, If)
    np.testing.assert_array_equal(D, Df)
    assign = ivf._assign.cpu().numpy()
    for l in (0, 7, 19):
        np.testing.assert_array_equal(ivf.list_ids(l), np.nonzero(assign == l)[0])
    flat = nf.IndexFlatL2(64)
    flat.add(xb)
    Dg, Ig = flat.search(xq, 7)
    np.testing.assert_array_equal(Ig, I)


@pytest.mark.parametrize("cap", [None, "3"])
def test_ivf_forced_fallback(gpu, monkeypatch, cap):
    monkeypatch.setenv("NRK_FORCE_FALLBACK", "1")
    if cap:
        monkeypatch.setenv("NRK_FB_CAP", cap)
    xq, xb = _mixture(20_000, 64, 64, seed=6)
    for metric in (ko.METRIC_IP, ko.METRIC_L2):
        ivf = _ivf(xb, 30, metric)
        ivf.nprobe = 5
        D, I = ivf.search(xq, 6)
        Do, Io, _, _ = io.ivf_search(xq, xb, ivf.quantizer._xb[:30].cpu().numpy(), ivf._assign.cpu().numpy(), 5, 6,
                                     metric)
        np.testing.assert_array_equal(I, Io)
        np.testing.assert_array_equal(D, Do)
        assert int(ivf.last_fallback.item()) == 64
        # n_fallback[1]: the queries whose tiled-scan buffer overflowed too (the
        # block-per-query scan); a 3-candidate buffer cannot hold k = 6
        nscan = int(ivf.last_exact_scan.item())
        assert 0 <= nscan <= 64
        if cap:
            assert nscan > 0, nscan


def test_ivf_k_exceeds_probed_items_pads(gpu):
    from newsrecommend_amd import faiss as nf

    xq, xb = _mixture(200, 5, 32, seed=7, centers=4)
    ivf = _ivf(xb, 40, ko.METRIC_L2)
    ivf.nprobe = 1
    D, I = ivf.search(xq, 64)
    Do, Io, _, _ = io.ivf_search(xq, xb, ivf.quantizer._xb[:40].cpu().numpy(), ivf._assign.cpu().numpy(), 1, 64,
                                 ko.METRIC_L2)
    np.testing.assert_array_equal(I, Io)
    assert (I == -1).any()


def test_retrieval_py_flow(gpu):
    """Retrieval.py:11-34 end to end: Clustering with an IndexHNSWFlat
    assignment index, index.search(xb, 1), cluster_to_articles, then the
    centroid IndexFlatL2 search per user profile."""
    from newsrecommend_amd import faiss as nf

    _, xb = _mixture(12_000, 1, 256, seed=8, centers=40)
    ids = np.arange(10**6, 10**6 + 12_000)
    clustering = nf.Clustering(256, 30)
    clustering.niter = 5
    index = nf.IndexHNSWFlat(256, 32)
    clustering.train(xb, index)
    centroids = nf.vector_float_to_array(clustering.centroids).reshape(30, 256)
    _, assign = index.search(xb, 1)
    cluster_to_articles = {i: ids[assign.ravel() == i] for i in range(30)}
    cent_o, _ = io.kmeans(xb, 30, niter=5, seed=1234, max_points_per_centroid=256)
    np.testing.assert_array_equal(centroids, cent_o)
    lab_o, _ = io.assign_nearest(xb, cent_o)
    np.testing.assert_array_equal(assign.ravel(), lab_o)
    centroid_index = nf.IndexFlatL2(256)
    centroid_index.add(centroids)
    profile = xb[:5].mean(0, keepdims=True)
    _, I = centroid_index.search(profile, 1)
    assert I[0, 0] == io.assign_nearest(profile, cent_o)[0][0]
    assert sum(len(v) for v in cluster_to_articles.values()) == 12_000


@pytest.mark.parametrize("metric", [ko.METRIC_L2, ko.METRIC_IP])
def test_ivf_c4_geometry_unbalanced_lists_and_collect_overflow(gpu, metric):
    """configs[3]'s index geometry at test scale: nlist = 300, nprobe = 32,
    faiss's IVF training defaults (niter 10; spherical for IP), a clustered
    300k x 128 corpus from 1024 centres (lists of very different sizes), k = 5.
    A block of 3001 exact duplicates of query 0 overflows its 2048-entry
    collect buffer, so the IVF-aware fallback must finish that query (ties ->
    lower ids)."""
    from newsrecommend_amd import faiss as nf

    xq, xb = _mixture(300_000, 256, 128, seed=41, centers=1024)
    xb[1000:4000] = xb[999]
    xq[0] = xb[999]
    ivf = nf.IndexIVFFlat(nf.IndexFlatL2(128), 128, 300, metric)
    assert ivf.cp.niter == 10 and ivf.cp.spherical == (metric == ko.METRIC_IP)
    ivf.train(xb)
    ivf.add(xb)
    ivf.nprobe = 32
    D, I = ivf.search(xq, 5)
    cent = ivf.quantizer._xb[:300].cpu().numpy()
    assign = ivf._assign.cpu().numpy()
    sizes = np.bincount(assign, minlength=300)
    assert sizes.max() > 2 * sizes.mean()  # unbalanced lists
    Do, Io, _, _ = io.ivf_search(xq, xb, cent, assign, 32, 5, metric)
    np.testing.assert_array_equal(I, Io)
    np.testing.assert_array_equal(D, Do)
    if metric == ko.METRIC_L2:
        assert I[0].tolist() == [999, 1000, 1001, 1002, 1003]
    assert int(ivf.last_fallback.item()) >= 1


def test_ivf_configs3_full_size_repeated_searches(gpu):
    """configs[3] at FULL size, as bench.py's `ivf` record runs it (the record
    that faulted in round 5's driver bench): bench's clustered 10M x 128 corpus
    and 4096 queries, nlist 300, nprobe 32, k-means niter 20, k 5, L2; 5
    warm-up + 20 timed-loop searches on one index (a 213K-row max list, 2048-
    block persistent grids with per-XCD tickets, 4096-row phase-A chunks).
    Every search: index guards clear, ids in [0, n) and unique per query,
    distances ascending, results identical to the first search's; a query
    sample against oracle/ivf_oracle.ivf_search over the full corpus."""
    from newsrecommend_amd import faiss as nf
    from newsrecommend_amd.data import clustered_corpus

    n, d, nlist, nprobe, k, nq = 10_000_000, 128, 300, 32, 5, 4096
    xb = clustered_corpus(n, d, seed=1234, device="cuda")
    xq = clustered_corpus(nq, d, seed=4321, device="cuda")
    ivf = nf.IndexIVFFlat(nf.IndexFlatL2(d), d, nlist, nf.METRIC_L2)
    ivf.cp.niter = 20
    ivf.train(xb)
    ivf.add(xb)
    ivf.nprobe = nprobe
    assert ivf.max_list > 100_000
    D0 = I0 = None
    for s in range(25):
        D, I = ivf.search_device(xq, k, check=True)
        if D0 is None:
            D0, I0 = D.clone(), I.clone()
            assert bool(((I >= 0) & (I < n)).all())
            assert bool((D[:, 1:] >= D[:, :-1]).all())
            srt = torch.sort(I, 1).values
            assert bool((srt[:, 1:] != srt[:, :-1]).all())
        else:
            assert torch.equal(I, I0) and torch.equal(D, D0), f"search {s} differs from search 0"
    assert int(ivf.last_fallback.item()) == 0
    sample = np.arange(0, nq, nq // 8)
    Do, Io, _, _ = io.ivf_search(xq[sample].cpu().numpy(), xb.cpu().numpy(), ivf.quantizer._xb[:nlist].cpu().numpy(),
                                 ivf._assign.cpu().numpy(), nprobe, k, ko.METRIC_L2)
    np.testing.assert_array_equal(I0[sample].cpu().numpy(), Io)
    np.testing.assert_array_equal(D0[sample].cpu().numpy(), Do)


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
@pytest.mark.parametrize("nq", [1, 3, 257])
def test_ivf_odd_query_batches(gpu, metric, nq):
    """Batches that fill no query tile (1, 3) or spill one row into the next
    (257): the grouping pads every list segment to the tile, the collect's
    waves skip the padding half-tiles; results equal the oracle's."""
    xq, xb = _mixture(25_000, nq, 128, seed=300 + nq, centers=32)
    ivf = _ivf(xb, 24, metric)
    ivf.nprobe = 6
    D, I = ivf.search(xq, 5)
    Do, Io, _, _ = io.ivf_search(xq, xb, ivf.quantizer._xb[:24].cpu().numpy(), ivf._assign.cpu().numpy(), 6, 5,
                                 metric)
    np.testing.assert_array_equal(I, Io)
    np.testing.assert_array_equal(D, Do)
    ivf.check_guards()


def test_ivf_incremental_add_continues_ids(gpu):
    """faiss IndexIVF.add twice: the second batch's ids continue from ntotal and
    the inverted lists are rebuilt over both (same result as one add)."""
    xq, xb = _mixture(30_000, 200, 64, seed=41, centers=24)
    one = _ivf(xb, 16, ko.METRIC_L2)
    from newsrecommend_amd import faiss as nf

    q = nf.IndexFlatL2(64)
    two = nf.IndexIVFFlat(q, 64, 16, ko.METRIC_L2)
    two.cp.niter = 4
    two.train(xb)
    two.add(xb[:12_345])
    two.add(xb[12_345:])
    assert two.ntotal == one.ntotal == 30_000
    for ivf in (one, two):
        ivf.nprobe = 4
    D1, I1 = one.search(xq, 8)
    D2, I2 = two.search(xq, 8)
    np.testing.assert_array_equal(I1, I2)
    np.testing.assert_array_equal(D1, D2)
    Do, Io, _, _ = io.ivf_search(xq, xb, two.quantizer._xb[:16].cpu().numpy(), two._assign.cpu().numpy(), 4, 8,
                                 ko.METRIC_L2)
    np.testing.assert_array_equal(I2, Io)
