"""Host-side data plumbing for the DIN path and synthetic workloads.

Restates the reference's dataset classes over explicit inputs instead of the
module-level `news/*.npy` globals (DIN.py:14-19):

  TrainDataset   DIN.py:66-92   (same sample order and the same `random`
                                 negative draws given the same seed)
  EvalDataset    DIN.py:21-57
  custom_collate_fn DIN.py:59-64

plus `ArticleTable`, a typed device-ready layout of the {article_id: vector}
dict (ids int64 + table float32 (N, d)) — the typed format SURVEY.md §8f asks
for — and `to_id_batch` helpers for the id-based fast path.  Synthetic
generators follow SURVEY.md §8d (clustered corpus, Zipf click logs).
"""
from __future__ import annotations

import random

import numpy as np
import torch
from torch.utils.data import Dataset


class ArticleTable:
    """{article_id: vector} -> ids (N,) int64 (dict order) + table (N, d) f32."""

    def __init__(self, ids: np.ndarray, table: np.ndarray):
        self.ids = np.asarray(ids, dtype=np.int64)
        self.table = np.ascontiguousarray(table, dtype=np.float32)
        order = np.argsort(self.ids, kind="stable")
        self._sorted_ids = self.ids[order]
        self._sorted_rows = order

    @classmethod
    def from_dict(cls, article_emb: dict) -> "ArticleTable":
        ids = np.fromiter(article_emb.keys(), dtype=np.int64, count=len(article_emb))
        table = np.stack([np.asarray(v, dtype=np.float32) for v in article_emb.values()]) if ids.size else \
            np.zeros((0, 0), np.float32)
        return cls(ids, table)

    @property
    def dim(self) -> int:
        return self.table.shape[1]

    def rows(self, article_ids) -> np.ndarray:
        """article ids -> row indices (int32); -1 stays -1 (padding)."""
        a = np.asarray(article_ids, dtype=np.int64)
        pos = np.searchsorted(self._sorted_ids, np.where(a < 0, 0, a))
        pos = np.clip(pos, 0, max(len(self._sorted_ids) - 1, 0))
        ok = (a >= 0) & (self._sorted_ids[pos] == a) if len(self._sorted_ids) else np.zeros(a.shape, bool)
        if np.any((a >= 0) & ~ok):
            raise KeyError("unknown article id in input")
        return np.where(a < 0, -1, self._sorted_rows[pos]).astype(np.int32)


class ClickLog:
    """Typed click log in place of the reference's
    {uid: [article ids]} dicts (DIN.py:17-18, embedding_generate.py:21-22):
    users int64 (U,) in dict order, CSR offsets int64 (U+1,), clicks int64
    (nnz,) article ids oldest -> newest.  `save`/`load` use a plain .npz
    (no pickles)."""

    def __init__(self, users, offsets, clicks):
        self.users = np.ascontiguousarray(users, dtype=np.int64)
        self.offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        self.clicks = np.ascontiguousarray(clicks, dtype=np.int64)
        if self.offsets.shape != (len(self.users) + 1,) or self.offsets[0] != 0 or \
                self.offsets[-1] != len(self.clicks) or np.any(np.diff(self.offsets) < 0):
            raise ValueError("ClickLog: offsets must be a non-decreasing (U+1,) CSR index over the clicks")

    @classmethod
    def from_dict(cls, user_clicks: dict) -> "ClickLog":
        users = np.fromiter(user_clicks.keys(), dtype=np.int64, count=len(user_clicks))
        lens = np.fromiter((len(v) for v in user_clicks.values()), dtype=np.int64, count=len(user_clicks))
        off = np.zeros(len(users) + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        clicks = np.fromiter((int(a) for v in user_clicks.values() for a in v), dtype=np.int64, count=int(off[-1]))
        return cls(users, off, clicks)

    def to_dict(self) -> dict:
        return {int(u): self.clicks[self.offsets[i]:self.offsets[i + 1]].tolist() for i, u in enumerate(self.users)}

    def __len__(self):
        return len(self.users)

    def save(self, path: str) -> None:
        np.savez(path, users=self.users, offsets=self.offsets, clicks=self.clicks)

    @classmethod
    def load(cls, path: str) -> "ClickLog":
        z = np.load(path)
        return cls(z["users"], z["offsets"], z["clicks"])


def _rng_words(rng):
    st = rng.getstate()
    if st[0] != 3 or len(st[1]) != 625:
        raise ValueError("expected a CPython Mersenne Twister state (version 3, 625 words)")
    return st, np.array(st[1], dtype=np.uint32)


def _rng_restore(rng, st, words):
    rng.setstate((st[0], tuple(int(w) for w in words), st[2]))


class TrainRows:
    """Typed TrainDataset rows: uid int64 (n,), hist int32 (n, L) table rows
    (-1 padded), target int32 (n,) table rows, label f32 (n, 1).  The id-based
    DIN path (FusedTrainStep / nrk_din_batch) consumes these directly."""

    def __init__(self, uid, hist, target, label):
        self.uid, self.hist, self.target, self.label = uid, hist, target, label

    def __len__(self):
        return len(self.target)


def train_rows(max_history: int, log: ClickLog, table: "ArticleTable", rng=random) -> TrainRows:
    """TrainDataset.__init__ (DIN.py:66-76) over a typed click log, built by
    libnrk's host builder (nrk_train_samples): the same rows as the Python loop
    and the same `random` draws, `rng` left advanced exactly as the loop would
    leave it.  Negatives index `table`'s row order (= list(article_emb.keys()))."""
    from . import _lib

    rows = table.rows(log.clicks)
    lens = np.diff(log.offsets)
    n = int(2 * np.maximum(lens - 1, 0).sum())
    L = int(max_history)
    uidx = np.empty(n, np.int32)
    tgt = np.empty(n, np.int32)
    lab = np.empty(n, np.float32)
    hist = np.empty((n, L), np.int32)
    st, words = _rng_words(rng)
    rc = _lib.load().nrk_train_samples(log.offsets.ctypes.data, len(log), rows.ctypes.data, len(table.ids), L,
                                       words.ctypes.data, n, uidx.ctypes.data, tgt.ctypes.data, lab.ctypes.data,
                                       hist.ctypes.data)
    _rng_restore(rng, st, words)
    _lib.check(rc, "train_rows")
    return TrainRows(log.users[uidx], hist, tgt, lab.reshape(n, 1))


class TrainDataset(Dataset):
    """DIN.py:66-92.  For each user (dict order) and click i >= 1: history =
    clicks[:i][-max_history:], one positive (target clicks[i], label 1) and one
    negative drawn with `random.choice(article_ids)` until not clicked (label 0).
    Pass the same `rng` state as the reference (it seeds `random` with 42,
    DIN.py:228) to get the identical sample list."""

    def __init__(self, max_history, train_user_clicks: dict, article_emb: dict, rng=random):
        self.max_history = max_history
        self.article_emb = article_emb
        article_ids = list(article_emb.keys())
        self.samples = []
        for uid, clicks in train_user_clicks.items():
            clicked = clicks  # membership test on the list, as the reference does
            for i in range(1, len(clicks)):
                hist = clicks[:i][-max_history:]
                self.samples.append({"uid": uid, "history": hist, "target": clicks[i], "label": 1})
                neg = rng.choice(article_ids)
                while neg in clicked:
                    neg = rng.choice(article_ids)
                self.samples.append({"uid": uid, "history": hist, "target": neg, "label": 0})
        self.dim = len(next(iter(article_emb.values()))) if article_emb else 0

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, idx):
        s = self.samples[idx]
        hist = np.zeros((self.max_history, self.dim), dtype=np.float32)
        for i, aid in enumerate(s["history"]):
            hist[i] = self.article_emb[aid]
        return {
            "uid": s["uid"],
            "history_emb": torch.from_numpy(hist),
            "target_emb": torch.as_tensor(np.asarray(self.article_emb[s["target"]], dtype=np.float32)),
            "label": torch.tensor([float(s["label"])], dtype=torch.float32),
        }

    def id_arrays(self, table: ArticleTable):
        """(hist_rows (n, L) int32 with -1 padding, target_rows (n,) int32, labels (n, 1) f32)."""
        n, L = len(self.samples), self.max_history
        hist = np.full((n, L), -1, dtype=np.int64)
        for j, s in enumerate(self.samples):
            h = s["history"]
            hist[j, : len(h)] = h
        tgt = np.array([s["target"] for s in self.samples], dtype=np.int64)
        lab = np.array([[float(s["label"])] for s in self.samples], dtype=np.float32).reshape(n, 1)
        return table.rows(hist), table.rows(tgt), lab


class EvalDataset(Dataset):
    """DIN.py:21-57: test users with >1 click; history = clicks[:-1][-L:];
    candidates = the retrieval output; labels one-hot at the FIRST candidate
    equal to the last click."""

    def __init__(self, max_history, test_user_clicks: dict, test_user_recs: dict, article_emb: dict):
        self.max_history = max_history
        self.article_emb = article_emb
        self.dim = len(next(iter(article_emb.values()))) if article_emb else 0
        self.data = []
        for uid, clicks in test_user_clicks.items():
            if len(clicks) <= 1:
                continue
            recs = test_user_recs[uid]
            labels = [0] * len(recs)
            for i, aid in enumerate(recs):
                if int(aid) == int(clicks[-1]):
                    labels[i] = 1
                    break
            self.data.append({"uid": uid, "history": clicks[:-1][-max_history:], "candidates": recs,
                              "labels": labels})

    def __len__(self):
        return len(self.data)

    def __getitem__(self, idx):
        s = self.data[idx]
        hist = np.zeros((self.max_history, self.dim), dtype=np.float32)
        for i, aid in enumerate(s["history"]):
            hist[i] = self.article_emb[aid]
        cand = np.array([self.article_emb[a] for a in s["candidates"]], dtype=np.float32).reshape(-1, self.dim)
        return {
            "uid": s["uid"],
            "history_emb": torch.from_numpy(hist),
            "cand_embs": torch.from_numpy(cand),
            "labels": torch.tensor(s["labels"], dtype=torch.float32),
        }


def custom_collate_fn(batch):
    """DIN.py:59-64: stack histories, keep candidates/labels as ragged lists."""
    return {
        "uid": [b["uid"] for b in batch],
        "history_emb": torch.stack([b["history_emb"] for b in batch], 0),
        "cand_embs": [b["cand_embs"] for b in batch],
        "labels": [b["labels"] for b in batch],
    }


# ------------------------------------------------------------- synthetic --
def clustered_corpus(n: int, d: int, n_centers: int = 1024, sigma: float = 0.35, seed: int = 1234,
                     device=None, center_seed: int = 1234) -> torch.Tensor:
    """item = centre[z] + sigma * N(0, I), centres ~ N(0, I)
    (drawn from `center_seed`, so corpus and queries share one mixture),
    z uniform; float32 (n, d).  Generated on `device` (GPU for large n)."""
    gc = torch.Generator(device=device or "cpu").manual_seed(center_seed)
    centers = torch.randn((n_centers, d), generator=gc, device=device)
    g = torch.Generator(device=device or "cpu").manual_seed(seed + 7919)
    out = torch.empty((n, d), dtype=torch.float32, device=device)
    step = 1 << 20
    for lo in range(0, n, step):
        hi = min(n, lo + step)
        z = torch.randint(0, n_centers, (hi - lo,), generator=g, device=device)
        out[lo:hi] = centers[z] + sigma * torch.randn((hi - lo, d), generator=g, device=device)
    return out


def zipf_ids(n: int, n_items: int, s: float = 1.1, generator=None, device=None) -> torch.Tensor:
    """n draws from a Zipf(s) popularity over n_items (rank r has mass ~ r^-s), int32."""
    ranks = torch.arange(1, n_items + 1, dtype=torch.float64, device=device)
    cdf = torch.cumsum(ranks.pow(-s), 0)
    cdf /= cdf[-1].clone()
    u = torch.rand(n, generator=generator, device=device, dtype=torch.float64)
    return torch.searchsorted(cdf, u).clamp_(max=n_items - 1).to(torch.int32)


def synthetic_click_rows(n_rows: int, n_items: int, L: int, seed: int = 7, device=None):
    """SURVEY.md §8d click log for the DIN train config: per row a history of
    uniform length 1..L (oldest->newest, tail padded with -1 as DIN.py:84-86
    zero-fills), Zipf(1.1) item popularity, target = a Zipf draw with label 1
    or a uniform draw with label 0 (50/50).  Returns (hist (n, L) int32,
    target (n,) int32, label (n, 1) f32) on `device`."""
    g = torch.Generator(device=device or "cpu").manual_seed(seed)
    hist = torch.empty((n_rows, L), dtype=torch.int32, device=device)
    step = 1 << 18
    ar = torch.arange(L, device=device)[None, :]
    for lo in range(0, n_rows, step):
        hi = min(n_rows, lo + step)
        ln = torch.randint(1, L + 1, (hi - lo, 1), generator=g, device=device)
        ids = zipf_ids((hi - lo) * L, n_items, generator=g, device=device).view(hi - lo, L)
        hist[lo:hi] = torch.where(ar < ln, ids, torch.full_like(ids, -1))
    label = (torch.rand((n_rows, 1), generator=g, device=device) < 0.5).float()
    pos = zipf_ids(n_rows, n_items, generator=g, device=device)
    neg = torch.randint(0, n_items, (n_rows,), generator=g, device=device, dtype=torch.int32)
    target = torch.where(label.view(-1) > 0.5, pos, neg)
    return hist, target, label
