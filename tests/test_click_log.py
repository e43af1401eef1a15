"""CPU: typed click logs and libnrk's host row builders (nrk_train_samples,
nrk_triplet_samples) against the reference's TrainDataset fixture
(tests/golden/din_dataset.npz, made by running DIN.py:66-76 under
random.seed(42)) and against the Python restatements of DIN.py:66-76 and
embedding_generate.py:25-39 on ragged logs (empty, single-click and duplicate
clicks, histories longer than max_history).  Host memory only: no GPU."""
import os
import random

import numpy as np
import pytest

from tests.conftest import GOLDEN
from tests.test_host import _world


def _random_log(seed, n_users, n_items, max_clicks, dup=True):
    rng = np.random.default_rng(seed)
    ids = rng.choice(np.arange(10, 10 + 20 * n_items), size=n_items, replace=False)
    emb = {int(a): np.full(4, i, np.float32) for i, a in enumerate(ids)}
    clicks = {}
    for u in range(n_users):
        n = int(rng.integers(0, max_clicks + 1))
        c = rng.choice(ids, size=n, replace=dup and n > 3)
        clicks[1000 + 3 * u] = [int(x) for x in c]
    return emb, clicks


def test_train_rows_match_reference_fixture():
    from newsrecommend_amd.data import ArticleTable, ClickLog, train_rows

    z = np.load(os.path.join(GOLDEN, "din_dataset.npz"))
    emb, trc, _, _ = _world(z)
    table = ArticleTable.from_dict(emb)
    rng = random.Random(42)  # as DIN.py:228
    r = train_rows(int(z["L"]), ClickLog.from_dict(trc), table, rng)
    np.testing.assert_array_equal(r.uid, z["tr_uid"])
    np.testing.assert_array_equal(table.ids[r.target], z["tr_target"])
    np.testing.assert_array_equal(r.label[:, 0], z["tr_label"].astype(np.float32))
    np.testing.assert_array_equal(r.hist, table.rows(z["tr_hist"]))


@pytest.mark.parametrize("seed,L", [(0, 3), (1, 8), (2, 50)])
def test_train_rows_match_python_loop(seed, L):
    from newsrecommend_amd.data import ArticleTable, ClickLog, TrainDataset, train_rows

    emb, clicks = _random_log(seed, 40, 60, 14)
    table = ArticleTable.from_dict(emb)
    r_py, r_nat = random.Random(seed), random.Random(seed)
    ds = TrainDataset(L, clicks, emb, rng=r_py)
    rows = train_rows(L, ClickLog.from_dict(clicks), table, r_nat)
    h, t, lab = ds.id_arrays(table)
    np.testing.assert_array_equal(rows.hist, h)
    np.testing.assert_array_equal(rows.target, t)
    np.testing.assert_array_equal(rows.label, lab)
    np.testing.assert_array_equal(rows.uid, [s["uid"] for s in ds.samples])
    assert r_py.getstate() == r_nat.getstate()  # the `random` stream continues identically


def test_train_rows_module_random_and_state_wraparound():
    """A long run crosses several 624-word twists; `random` itself (the
    module) is accepted as the rng, as the reference uses it."""
    from newsrecommend_amd.data import ArticleTable, ClickLog, TrainDataset, train_rows

    emb, clicks = _random_log(5, 300, 97, 20)
    table = ArticleTable.from_dict(emb)
    random.seed(7)
    st = random.getstate()
    rows = train_rows(6, ClickLog.from_dict(clicks), table)
    after = random.getstate()
    random.setstate(st)
    ds = TrainDataset(6, clicks, emb)
    assert random.getstate() == after
    np.testing.assert_array_equal(rows.target, ds.id_arrays(table)[1])


def test_triplets_match_python_loop():
    from newsrecommend_amd.data import ClickLog
    from newsrecommend_amd.embedding import ArticleTripletDataset

    emb, clicks = _random_log(3, 30, 50, 9)
    ids = list(emb.keys())
    r_py, r_nat = random.Random(11), random.Random(11)
    a = ArticleTripletDataset(clicks, ids, rng=r_py)
    b = ArticleTripletDataset.from_click_log(ClickLog.from_dict(clicks), ids, rng=r_nat)
    np.testing.assert_array_equal(a.triplets, b.triplets)
    assert r_py.getstate() == r_nat.getstate()


def test_empty_and_degenerate_logs():
    from newsrecommend_amd import _lib
    from newsrecommend_amd.data import ArticleTable, ClickLog, train_rows

    emb = {5: np.zeros(2, np.float32), 9: np.ones(2, np.float32)}
    table = ArticleTable.from_dict(emb)
    r = train_rows(4, ClickLog.from_dict({1: [], 2: [5]}), table, random.Random(0))
    assert len(r) == 0 and r.hist.shape == (0, 4)
    with pytest.raises(_lib.NrkError, match="clicked every item"):  # the reference would loop forever
        train_rows(4, ClickLog.from_dict({1: [5, 9]}), table, random.Random(0))
    with pytest.raises(KeyError):
        train_rows(4, ClickLog.from_dict({1: [5, 77]}), table, random.Random(0))


def test_click_log_roundtrip(tmp_path):
    from newsrecommend_amd.data import ClickLog

    _, clicks = _random_log(4, 25, 40, 7)
    log = ClickLog.from_dict(clicks)
    assert log.to_dict() == clicks
    p = str(tmp_path / "clicks.npz")
    log.save(p)
    back = ClickLog.load(p)
    assert back.to_dict() == clicks
    with pytest.raises(ValueError):
        ClickLog(log.users, log.offsets[:-1], log.clicks)


def test_row_builder_c_abi_rejects_bad_input():
    """The host builders through the raw C-ABI (include/nrk.h): wrong sample
    counts, non-monotone offsets, out-of-range rows and a bad Mersenne Twister
    position are NRK_EINVAL (-1) with a message in nrk_last_error()."""
    from newsrecommend_amd import _lib

    L = _lib.load()
    off = np.array([0, 3, 5], np.int64)
    rows = np.array([0, 1, 2, 3, 4], np.int32)
    st = np.array(random.Random(1).getstate()[1], np.uint32)
    n = 2 * (2 + 1)
    u, t, lab = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.float32)

    def call(off_, rows_, n_items, st_, n_):
        return L.nrk_train_samples(off_.ctypes.data, len(off_) - 1, rows_.ctypes.data, n_items, 4, st_.ctypes.data,
                                   n_, u.ctypes.data, t.ctypes.data, lab.ctypes.data, None)

    assert call(off, rows, 10, st.copy(), n) == 0
    assert call(off, rows, 10, st.copy(), n + 2) == -1 and b"yields" in L.nrk_last_error()
    assert call(np.array([0, 3, 2], np.int64), rows, 10, st.copy(), n) == -1
    assert call(off, rows, 4, st.copy(), n) == -1 and b"outside" in L.nrk_last_error()
    bad = st.copy()
    bad[624] = 1000
    assert call(off, rows, 10, bad, n) == -1 and b"position" in L.nrk_last_error()
    trip = np.empty((4, 3), np.int32)
    assert L.nrk_triplet_samples(off.ctypes.data, 2, rows.ctypes.data, 10, st.copy().ctypes.data, 4,
                                 trip.ctypes.data) == 0
    assert L.nrk_triplet_samples(off.ctypes.data, 2, rows.ctypes.data, 10, st.copy().ctypes.data, 5,
                                 trip.ctypes.data) == -1
