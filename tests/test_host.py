"""CPU: host-side logic — dataset restatements vs the reference fixtures,
the DIN module's state_dict/init parity, the C-ABI library exports."""
import ctypes
import os
import random
import re

import numpy as np
import pytest
import torch

from tests.conftest import GOLDEN, ROOT


def _world(z):
    def dict_of(users, lens, flat):
        out, o = {}, 0
        for u, n in zip(users, lens):
            out[int(u)] = [int(x) for x in flat[o:o + n]]
            o += n
        return out

    emb = {int(a): z["table"][i] for i, a in enumerate(z["item_ids"])}
    trc = dict_of(z["train_users"], z["train_click_len"], z["train_clicks"])
    tec = dict_of(z["test_users"], z["test_click_len"], z["test_clicks"])
    recs, o = {}, 0
    for u, n in zip(z["rec_users"], z["rec_len"]):
        recs[int(u)] = z["recs"][o:o + n].astype(np.int64)
        o += n
    return emb, trc, tec, recs


def test_train_dataset_matches_reference():
    from newsrecommend_amd.data import ArticleTable, TrainDataset

    z = np.load(os.path.join(GOLDEN, "din_dataset.npz"))
    emb, trc, _, _ = _world(z)
    random.seed(42)  # as DIN.py:228
    ds = TrainDataset(int(z["L"]), trc, emb)
    assert len(ds) == len(z["tr_uid"])
    np.testing.assert_array_equal([s["uid"] for s in ds.samples], z["tr_uid"])
    np.testing.assert_array_equal([s["target"] for s in ds.samples], z["tr_target"])
    np.testing.assert_array_equal([s["label"] for s in ds.samples], z["tr_label"])
    item = ds[3]
    np.testing.assert_array_equal(item["history_emb"].numpy(), z["item3_hist"])
    np.testing.assert_array_equal(item["target_emb"].numpy(), z["item3_target"])
    table = ArticleTable.from_dict(emb)
    hist_rows, tgt_rows, lab = ds.id_arrays(table)
    expect = table.rows(z["tr_hist"])
    np.testing.assert_array_equal(hist_rows, expect)
    np.testing.assert_array_equal(table.table[tgt_rows], np.stack([emb[int(t)] for t in z["tr_target"]]))


def test_eval_dataset_matches_reference():
    from newsrecommend_amd.data import EvalDataset

    z = np.load(os.path.join(GOLDEN, "din_dataset.npz"))
    emb, _, tec, recs = _world(z)
    ds = EvalDataset(int(z["L"]), tec, recs, emb)
    np.testing.assert_array_equal([s["uid"] for s in ds.data], z["ev_uid"])
    np.testing.assert_array_equal([len(s["candidates"]) for s in ds.data], z["ev_cand_len"])
    np.testing.assert_array_equal(np.concatenate([s["labels"] for s in ds.data]), z["ev_lab"])


@pytest.mark.parametrize("name", ["din_fwd_c1", "din_fwd_c3"])
def test_din_state_dict_and_init_parity(name):
    from newsrecommend_amd.din import DIN

    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    torch.manual_seed({"din_fwd_c1": 11, "din_fwd_c3": 12}[name])
    m = DIN(int(z["d"]), int(z["A"]), int(z["F"]), 0.36)
    sd = m.state_dict()
    ref_keys = sorted(k[len("init_sd::"):] for k in z.files if k.startswith("init_sd::"))
    assert sorted(sd.keys()) == ref_keys
    for k in ref_keys:  # same init order and RNG consumption -> identical parameters
        np.testing.assert_array_equal(sd[k].numpy(), z[f"init_sd::{k}"], err_msg=k)
    m.load_state_dict({k[4:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd::")})


def test_cpu_tensors_raise():
    from newsrecommend_amd import _lib
    from newsrecommend_amd.din import DIN

    m = DIN(64, 32, 32, 0.0)
    with pytest.raises((_lib.NrkError, RuntimeError)):
        m(torch.zeros(2, 64), torch.zeros(2, 5, 64))


def _header_symbols():
    text = open(os.path.join(ROOT, "include", "nrk.h")).read()
    return sorted(set(re.findall(r"\b(nrk_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    from newsrecommend_amd import _lib

    syms = _header_symbols()
    assert len(syms) >= 10
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in syms:
        assert hasattr(lib, s), f"libnrk.so does not export {s}"
    assert set(syms) == set(_lib.SIGNATURES), "ctypes SIGNATURES out of sync with include/nrk.h"
    L = _lib.load()
    assert L.nrk_version() == 1
    assert L.nrk_padded_dim(100) == 128
    sz = _lib.c_size(0)
    assert L.nrk_knn_flat_workspace(4096, 1_000_000, 128, 5, sz) == 0 and sz.value > 0
    assert L.nrk_knn_flat_workspace(-1, 10, 8, 5, sz) != 0
    assert b"bad arguments" in L.nrk_last_error()


def test_rerank_max_history_query():
    """nrk_din_rerank_max_history (host only): 128 history slots for every
    (A, F) of the reference's Optuna grid (DIN.py:203-207; the lane kernel's
    128-row form, R and H2 from global memory where they do not fit its LDS);
    an unsupported (A, F) is an error."""
    from newsrecommend_amd import _lib
    from newsrecommend_amd.pipeline import rerank_max_history

    for A in (32, 64, 96, 128):
        for F in (32, 64, 96, 128):
            assert rerank_max_history(A, F) == 128, (A, F)
    v = ctypes.c_int32(0)
    assert _lib.load().nrk_din_rerank_max_history(48, 32, ctypes.byref(v)) != 0


def test_shard_ranges_cover():
    from newsrecommend_amd.dist import shard_range

    for n in (0, 7, 1000, 1_000_003):
        for w in (1, 2, 3, 8):
            r = [shard_range(n, i, w) for i in range(w)]
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(r[:-1], r[1:]))
            assert max(b - a for a, b in r) - min(b - a for a, b in r) <= 1
