"""GPU parity: libnrk flat search (through the faiss-compatible wrapper and the
C-ABI) against the oracle — indices bit-exact, D bit-exact (the fp32 rounding
of the same fp64 scores)."""
import numpy as np
import pytest
import torch

from oracle import knn_oracle as ko

pytestmark = pytest.mark.gpu


def _mixture(nb, nq, d, seed, centers=64, sigma=0.35):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((centers, d)).astype(np.float32)
    xb = (c[rng.integers(0, centers, nb)] + sigma * rng.standard_normal((nb, d))).astype(np.float32)
    xq = (c[rng.integers(0, centers, nq)] + sigma * rng.standard_normal((nq, d))).astype(np.float32)
    return xq, xb


def _check(xq, xb, k, metric, gpu, exact_below=None, monkeypatch=None):
    from newsrecommend_amd import faiss as nf

    idx = nf.IndexFlat(xb.shape[1], metric)
    idx.add(xb)
    D, I = idx.search(xq, k)
    Do, Io, So = ko.exact_search(xq, xb, k, metric)
    np.testing.assert_array_equal(I, Io)
    np.testing.assert_array_equal(D, Do)
    return idx


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
def test_c1_shape(gpu, metric):
    """configs[0]: 10k x 64, 1k queries, k=5 (below 16384 rows: the fp64 exact
    path; the screened path is covered by the larger tests)."""
    xq, xb = _mixture(10_000, 1000, 64, seed=1)
    _check(xq, xb, 5, metric, gpu)


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
@pytest.mark.parametrize("d,k", [(128, 5), (64, 10), (100, 32), (256, 5), (32, 1), (128, 100), (256, 200)])
def test_screened_path(gpu, metric, d, k):
    xq, xb = _mixture(60_001, 300, d, seed=d + k)
    idx = _check(xq, xb, k, metric, gpu)
    assert idx.last_fallback is not None


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
@pytest.mark.parametrize("d,k", [(128, 5), (64, 10), (100, 32), (256, 5), (32, 1)])
def test_screen_partial_chunk_tiles(gpu, metric, d, k):
    """A corpus size whose chunks end in partial tiles (the deferred epilogue
    masks the last sub-tile's rows after the loop) gives the oracle's results."""
    xq, xb = _mixture(70_003, 300, d, seed=d + k + 1)
    _check(xq, xb, k, metric, gpu)


@pytest.mark.parametrize("form", ["0", "1"])
@pytest.mark.parametrize("d,n,k", [(128, 60_001, 5), (128, 70_003, 5), (256, 60_001, 5), (256, 70_003, 5),
                                   (256, 60_001, 200), (256, 70_003, 200)])
def test_screen_main_pass_forms(gpu, monkeypatch, form, d, n, k):
    """The inner-product main pass runs on the 16x16x32 kernel (screen16.h) by
    default at k <= 8 for d 128 / 256 and at k = 200 for d 256 (its 2-step
    fragment ring over three LDS buffers) (=1); the 32x32x16 kernel
    (NRK_SCREEN16=0, the one every other form runs) gives the oracle's results
    too, with and without partial last tiles."""
    monkeypatch.setenv("NRK_SCREEN16", form)
    xq, xb = _mixture(n, 300, d, seed=d + n % 7)
    _check(xq, xb, k, ko.METRIC_IP, gpu)


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
def test_collect_pass_dense_neighbourhoods(gpu, metric):
    """Few, dense clusters (8 centres, 400k rows): neighbours closer together
    than the bf16 screening error bound, so the certificate leaves queries
    uncovered; the collect pass (one more screen for those queries, every item
    within the bound of the merge's exact k-th, exact rescoring) answers them
    without the fp64 corpus scan, bit-exact vs the oracle."""
    xq, xb = _mixture(400_000, 256, 128, seed=21, centers=8, sigma=0.2)
    idx = _check(xq, xb, 10, metric, gpu)
    nfb, nscan = int(idx.last_fallback.item()), int(idx.last_exact_scan.item())
    print(f"uncertified {nfb}, fp64 scan {nscan}")
    if metric == ko.METRIC_L2:
        assert nfb > 0
    assert nscan == 0


def test_gaussian_unstructured(gpu):
    rng = np.random.default_rng(7)
    xb = rng.standard_normal((50_000, 128)).astype(np.float32)
    xq = rng.standard_normal((257, 128)).astype(np.float32)
    for metric in (ko.METRIC_IP, ko.METRIC_L2):
        _check(xq, xb, 10, metric, gpu)


def test_duplicates_and_ties_take_lower_id(gpu):
    """Exact duplicates straddling chunks and lanes: the certificate cannot
    separate them, so these queries go through the fp64 fallback, which must
    return the lower ids first."""
    xq, xb = _mixture(40_000, 64, 64, seed=3)
    for j in (5, 17_000, 39_999, 20_001):
        xb[j] = xb[3]
    xq[0] = xb[3]
    xq[1] = xb[3] * 2
    for metric in (ko.METRIC_IP, ko.METRIC_L2):
        idx = _check(xq, xb, 4, metric, gpu)
    _, I = idx.search(xq[:1], 4)
    assert I[0].tolist() == [3, 5, 17000, 20001]


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
@pytest.mark.parametrize("d", [64, 256])
def test_k200_tied_block_at_the_selection_cut(gpu, metric, d):
    """k = 200 (the merge SELECTS its 400 rescoring candidates by score keys):
    900 exact copies of one row spread over the corpus tie at the cut, so the
    tie rule (ascending id) decides which copies are rescored; results equal
    the oracle's (d 256: the 16x16x32 main pass's lane lists)."""
    xq, xb = _mixture(60_001, 64, d, seed=11)
    rng = np.random.default_rng(5)
    dup = np.sort(rng.choice(np.arange(1, 60_001), 900, replace=False))
    xb[dup] = xb[0]
    xq[:8] = xb[0] * np.float32(1.5)
    _check(xq, xb, 200, metric, gpu)


def test_k_exceeds_ntotal_and_empty(gpu):
    from newsrecommend_amd import faiss as nf

    xq, xb = _mixture(5, 3, 16, seed=4)
    for metric in (ko.METRIC_IP, ko.METRIC_L2):
        idx = nf.IndexFlat(16, metric)
        idx.add(xb)
        D, I = idx.search(xq, 8)
        Do, Io, _ = ko.exact_search(xq, xb, 8, metric)
        np.testing.assert_array_equal(I, Io)
        np.testing.assert_array_equal(D, Do)
        empty = nf.IndexFlat(16, metric)
        D, I = empty.search(xq, 2)
        assert (I == -1).all()


def test_incremental_add_and_torch_io(gpu):
    from newsrecommend_amd import faiss as nf

    xq, xb = _mixture(30_000, 100, 128, seed=8)
    idx = nf.IndexFlatIP(128)
    for lo in range(0, 30_000, 7_000):
        idx.add(xb[lo:lo + 7_000])
    assert idx.ntotal == 30_000
    D, I = idx.search(torch.from_numpy(xq).cuda(), 5)
    assert D.is_cuda and I.dtype == torch.int64
    _, Io, _ = ko.exact_search(xq, xb, 5, ko.METRIC_IP)
    np.testing.assert_array_equal(I.cpu().numpy(), Io)


def test_retrieval_centroid_search(gpu):
    """Retrieval.py:25-34 shape: IndexFlatL2 over 300 centroids, nq=1 searches."""
    from newsrecommend_amd import faiss as nf

    xq, xb = _mixture(300, 50, 256, seed=9)
    idx = nf.IndexFlatL2(256)
    idx.add(xb)
    _, Io, _ = ko.exact_search(xq, xb, 1, ko.METRIC_L2)
    for i in range(0, 50, 7):
        _, I = idx.search(xq[i].reshape(1, 256), 1)
        assert I[0, 0] == Io[i, 0]


def test_shard_merge_kernel(gpu):
    from newsrecommend_amd import faiss as nf

    xq, xb = _mixture(20_000, 64, 64, seed=10)
    xb[15_000] = xb[2]
    xq[0] = xb[2]
    for metric in (ko.METRIC_IP, ko.METRIC_L2):
        parts_S, parts_I = [], []
        for lo, hi in ((0, 6_000), (6_000, 6_001), (6_001, 20_000)):
            D, I, S = nf.knn_exact(torch.from_numpy(xq).cuda(), torch.from_numpy(xb[lo:hi]).cuda(), 7, metric,
                                   id_offset=lo)
            parts_S.append(S)
            parts_I.append(I)
        Dm, Im, Sm = nf.topk_merge(torch.stack(parts_S), torch.stack(parts_I), 7, metric)
        Do, Io, So = ko.exact_search(xq, xb, 7, metric)
        np.testing.assert_array_equal(Im.cpu().numpy(), Io)
        np.testing.assert_array_equal(Sm.cpu().numpy(), So)


def test_full_size_properties(gpu):
    """configs[1] size (1M x 128, nq=4096, k=5): size-independent properties —
    every returned score equals an fp64 recomputation, lists are sorted with
    ids ascending on ties, and a sample of queries equals the oracle."""
    from newsrecommend_amd import faiss as nf
    from newsrecommend_amd.data import clustered_corpus

    xb = clustered_corpus(1_000_000, 128, seed=1234, device="cuda")
    xq = clustered_corpus(4096, 128, seed=4321, device="cuda")
    idx = nf.IndexFlatIP(128)
    idx.add(xb)
    D, I, S = idx.search_device(xq, 5, exact_scores=True)
    assert (I >= 0).all()
    rows = xb[I.view(-1)].double().view(4096, 5, 128)
    s64 = (rows * xq.double()[:, None, :]).sum(-1)
    assert torch.allclose(s64, S, rtol=0, atol=1e-9)
    assert (S[:, :-1] >= S[:, 1:]).all()
    sample = torch.arange(0, 4096, 97)
    _, Io, So = ko.exact_search(xq[sample].cpu().numpy(), xb.cpu().numpy(), 5, ko.METRIC_IP)
    np.testing.assert_array_equal(I[sample].cpu().numpy(), Io)
    assert int(idx.last_fallback.item()) <= 41  # certificate covers (nearly) every query


@pytest.mark.parametrize("force,cap", [("1", None), ("2", None), ("2", "6")])
def test_forced_fallback_paths(gpu, monkeypatch, force, cap):
    """Every query uncertified (NRK_FORCE_FALLBACK=1): the collect pass must
    reproduce the oracle; with every collect buffer overflowed (=2) the tiled
    fp64 fallback (scan + select) must; with a tiny candidate cap the overflow
    path (block-per-query exact kernel) must too."""
    monkeypatch.setenv("NRK_FORCE_FALLBACK", force)
    if cap:
        monkeypatch.setenv("NRK_FB_CAP", cap)
    xq, xb = _mixture(50_000, 200, 96, seed=11)
    xb[40_000] = xb[7]
    xq[3] = xb[7]
    for metric in (ko.METRIC_IP, ko.METRIC_L2):
        for k in (1, 5, 40):
            idx = _check(xq, xb, k, metric, gpu)
            assert int(idx.last_fallback.item()) == 200
            assert int(idx.last_exact_scan.item()) == (200 if force == "2" else 0)


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
def test_collect_rounds_beyond_the_slot_budget(gpu, monkeypatch, metric):
    """more uncertified queries than collect slots (20,000
    > FB_SLOTS_MAX = 16,384, every query uncertified by NRK_FORCE_FALLBACK=1, as
    an 8-GPU shard searched by 8 x 4096 queries can leave them at L2): the
    collect pass runs in two rounds over the same storage and answers every
    query -- results equal the oracle and NO query takes the fp64 scan."""
    monkeypatch.setenv("NRK_FORCE_FALLBACK", "1")
    xq, xb = _mixture(30_000, 20_000, 64, seed=21)
    idx = _check(xq, xb, 5, metric, gpu)
    assert int(idx.last_fallback.item()) == 20_000
    assert int(idx.last_exact_scan.item()) == 0


@pytest.mark.parametrize("metric", [ko.METRIC_IP, ko.METRIC_L2])
@pytest.mark.parametrize("nb,nq,d,k", [(300, 4100, 128, 32), (300, 777, 256, 1), (1, 70, 32, 3), (63, 65, 100, 63),
                                       (4096, 5000, 32, 10), (2048, 300, 300, 200), (500, 129, 64, 700),
                                       (512, 1000, 256, 64), (257, 33, 36, 17), (64, 16, 4, 64),
                                       (300, 1, 256, 1), (3000, 63, 100, 1), (1000, 5, 99, 40)])
def test_small_corpus_exact_path(gpu, metric, nb, nq, d, k):
    """nb <= 4096 (the coarse quantizer, k-means assignment, IndexIVFFlat.add):
    the fp64 tile-GEMM path (k = 1: fused arg-best; k > 1: goodness chunks +
    per-query select, several chunks at nb = 4096) equals the oracle bit for
    bit, including k > nb padding, d > 256 and exact duplicates.  Fewer than 64
    queries take a thread per (query, item) (small_rows_kernel, also at k = 1
    and for d not a multiple of 4)."""
    xq, xb = _mixture(nb, nq, d, seed=nb + nq + d + k)
    if nb > 10:
        xb[nb // 2] = xb[3]
        xq[0] = xb[3]
    from newsrecommend_amd import faiss as nf

    idx = nf.IndexFlat(d, metric)
    idx.add(xb)
    D, I, S = idx.search_device(torch.from_numpy(xq).cuda(), k, exact_scores=True)
    Do, Io, So = ko.exact_search(xq, xb, k, metric)
    np.testing.assert_array_equal(I.cpu().numpy(), Io)
    np.testing.assert_array_equal(D.cpu().numpy(), Do)
    np.testing.assert_array_equal(S.cpu().numpy(), So)
    assert int(idx.last_fallback.item()) == 0


def test_small_corpus_assignment_at_scale(gpu):
    """IndexIVFFlat.add's assignment shape: 200k rows x 300 centroids, k = 1."""
    from newsrecommend_amd import faiss as nf

    xq, xb = _mixture(300, 200_000, 128, seed=77)
    idx = nf.IndexFlatL2(128)
    idx.add(xb)
    D, I = idx.search(xq, 1)
    Do, Io, _ = ko.exact_search(xq, xb, 1, ko.METRIC_L2)
    np.testing.assert_array_equal(I, Io)
    np.testing.assert_array_equal(D, Do)


def test_search_device_input_checks(gpu):
    """search_device converts bf16 / strided queries and refuses host tensors
    and wrong widths; probes are normalised to int64."""
    from newsrecommend_amd import _lib, faiss as nf

    xq, xb = _mixture(20_000, 64, 64, seed=12)
    idx = nf.IndexFlatIP(64)
    idx.add(xb)
    q = torch.from_numpy(xq).cuda()
    _, I_ref = idx.search_device(q, 5)
    wide = torch.zeros((64, 128), device="cuda")
    wide[:, ::2] = q
    _, I_view = idx.search_device(wide[:, ::2], 5)  # non-contiguous view
    assert torch.equal(I_view, I_ref)
    _, I_bf = idx.search_device(q.to(torch.bfloat16), 5)  # converted to f32 (bf16 values)
    _, I_bf_ref = idx.search_device(q.to(torch.bfloat16).float(), 5)
    assert torch.equal(I_bf, I_bf_ref)
    with pytest.raises(_lib.NrkError):
        idx.search_device(q.cpu(), 5)
    with pytest.raises(AssertionError):
        idx.search_device(q[:, :32], 5)
    ivf = nf.IndexIVFFlat(nf.IndexFlatL2(64), 64, 16, nf.METRIC_L2)
    ivf.cp.niter = 2
    ivf.train(xb)
    ivf.add(xb)
    ivf.nprobe = 4
    _, probe = ivf.quantizer.search_device(q, 4)
    _, I1 = ivf.search_device(q, 5, probe=probe)
    _, I2 = ivf.search_device(q, 5, probe=probe.to(torch.int32))
    assert torch.equal(I1, I2)
    with pytest.raises(AssertionError):
        ivf.search_device(q, 5, probe=probe[:, :2])


def test_numpy_search_one_query_at_a_time(gpu):
    """The reference's per-user loop (Retrieval.py:28-34: centroid_index.search
    (profile, 1) for each profile): the numpy path (pinned staging, one sync)
    returns fresh arrays equal to one batched device search, call after call."""
    from newsrecommend_amd import faiss as nf

    xq, xb = _mixture(300, 40, 256, seed=5)
    idx = nf.IndexFlatL2(256)
    idx.add(xb)
    Db, Ib = idx.search_device(torch.from_numpy(xq).cuda(), 1)
    got = [idx.search(xq[i:i + 1], 1) for i in range(len(xq))]
    np.testing.assert_array_equal(np.concatenate([g[1] for g in got]), Ib.cpu().numpy())
    np.testing.assert_array_equal(np.concatenate([g[0] for g in got]), Db.cpu().numpy())
    D2, I2 = idx.search(xq, 3)  # a larger call grows the staging; earlier results stay intact
    np.testing.assert_array_equal(I2[:, :1], Ib.cpu().numpy())
    np.testing.assert_array_equal(np.concatenate([g[1] for g in got]), Ib.cpu().numpy())
