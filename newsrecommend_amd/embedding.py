"""Article embedding model and corpus producer (embedding_generate.py:51-131),
the producer side of the retrieval path.

  ArticleEmbeddingModel   same layers, init order and state_dict keys as
                          embedding_generate.py:51-65 (fc.0 Linear(253,512),
                          fc.1 ReLU, fc.2 Dropout, fc.3 BatchNorm1d(512),
                          fc.4 Linear(512,256)); a reference checkpoint
                          (best_eg_model.pth) loads with weights_only=True
  ArticleEmbeddingModel.embed   eval-mode inference for a whole corpus: the
                          BatchNorm is folded into fc.4 (W' = W diag(s),
                          b' = b + W t) and both layers run in ONE hand-written
                          kernel (libnrk nrk_embed, csrc/embed.hip: h stays on
                          chip, fp32-exact products from three-plane bf16 MFMAs)
                          instead of the reference's 364,047 batch-1 forwards
                          (embedding_generate.py:118-121)
  inference               embedding_generate.py:109-131 with typed outputs:
                          ids int64 (N,) + embeddings float32 (N, 256) in one
                          .npz instead of the pickled dict / object array
                          (the object array cannot be read back by
                          Retrieval.py:6 with allow_pickle=False)
  load_article_table      Retrieval.py:6-9 for both the typed .npz and a plain
                          numeric (N, d+1) table (ids in the last column)
  ArticleTripletDataset / train_triplet   embedding_generate.py:25-49,67-107
                          (TripletMarginLoss(margin=1, p=2), Adam with L2
                          weight decay), features gathered on the device;
                          .from_click_log builds the triplets natively
  fit_triplet             main() (embedding_generate.py:67-107): shuffled
                          train/eval loaders, per-epoch losses, best-eval-loss
                          checkpoint; pinned to the reference's own main() run
                          (tests/golden/embedding_train.npz)
"""
from __future__ import annotations

import random

import numpy as np
import torch
import torch.nn as nn

NUM_FEATURE = 253
FC_DIM = 512
EMBEDDING_DIM = 256
DROPOUT = 0.13
MARGIN = 1.0
LR = 1e-3
WEIGHT_DECAY = 5e-5


class ArticleEmbeddingModel(nn.Module):
    def __init__(self, input_dim=NUM_FEATURE, fc_dim=FC_DIM, embedding_dim=EMBEDDING_DIM, dropout_rate=DROPOUT):
        super().__init__()
        self.fc = nn.Sequential(
            nn.Linear(input_dim, fc_dim),
            nn.ReLU(),
            nn.Dropout(dropout_rate),
            nn.BatchNorm1d(fc_dim),
            nn.Linear(fc_dim, embedding_dim),
        )

    def forward(self, x):
        return self.fc(x)

    def folded(self):
        """(W1, b1, W2', b2') with the eval-mode BatchNorm folded into fc.4."""
        l1, bn, l2 = self.fc[0], self.fc[3], self.fc[4]
        s = bn.weight / torch.sqrt(bn.running_var + bn.eps)
        t = bn.bias - bn.running_mean * s
        return l1.weight, l1.bias, l2.weight * s[None, :], l2.bias + l2.weight @ t

    @torch.no_grad()
    def embed(self, x: torch.Tensor, batch: int | None = None) -> torch.Tensor:
        """Eval-mode embeddings of x (n, input_dim) -> (n, embedding_dim) f32 on
        x's device, in ONE launch of libnrk's nrk_embed (the hidden layer stays
        on chip; fp32-exact products from bf16 MFMAs).  `batch` is accepted for
        the older call form and ignored.  There is no CPU path: host tensors
        raise (the module's own forward is the reference's arithmetic)."""
        from . import _lib

        dev = _lib.require_device(x, what="ArticleEmbeddingModel.embed")
        W1, b1, W2, b2 = (p.detach().float().contiguous() for p in self.folded())
        if W1.device != dev:
            raise _lib.NrkError(f"ArticleEmbeddingModel.embed: input on {dev}, model on {W1.device}")
        x = x.float()
        if x.dim() != 2 or x.shape[1] != W1.shape[1]:  # the reference's forward raises here too
            raise RuntimeError(f"ArticleEmbeddingModel.embed: expected (n, {W1.shape[1]}) input, got "
                               f"{tuple(x.shape)}")
        if x.stride(-1) != 1:
            x = x.contiguous()
        n, in_dim = x.shape
        hid, out_dim = W1.shape[0], W2.shape[0]
        if not embed_supported(in_dim, hid, out_dim):
            # a non-default architecture (nrk_embed: in_dim <= 256, hidden a multiple
            # of 128, out_dim 256): the folded layers as two GPU GEMMs, said loudly
            import warnings

            warnings.warn(f"ArticleEmbeddingModel.embed: dims {in_dim} -> {hid} -> {out_dim} outside nrk_embed's "
                          f"(<= 256, k*128, 256): two torch GEMMs on {dev}")
            self.embed_path = "torch-gemm"
            return torch.addmm(b2, torch.relu(torch.addmm(b1, x, W1.t())), W2.t())
        self.embed_path = "nrk_embed"
        out = torch.empty((n, out_dim), dtype=torch.float32, device=dev)
        lib = _lib.load()
        sz = _lib.c_size(0)
        _lib.check(lib.nrk_embed_workspace(in_dim, hid, out_dim, sz), "embed_workspace")
        ws = torch.empty(sz.value, dtype=torch.uint8, device=dev)
        _lib.check(lib.nrk_embed(_lib.ptr(x), n, x.stride(0), in_dim, _lib.ptr(W1), _lib.ptr(b1), hid, _lib.ptr(W2),
                                 _lib.ptr(b2), out_dim, _lib.ptr(out), _lib.ptr(ws), ws.numel(), _lib.stream(dev)),
                   "embed")
        return out


def embed_supported(in_dim: int, hidden: int, out_dim: int) -> bool:
    """Shapes nrk_embed runs (csrc/embed.hip: KP = 256 input columns, HC = 128
    hidden units per chunk, OD = 256 outputs); the reference's 253 -> 512 -> 256."""
    return 1 <= in_dim <= 256 and hidden >= 128 and hidden % 128 == 0 and out_dim == 256


def inference(model: ArticleEmbeddingModel, article_features, device=None, out_path: str | None = None,
              batch: int = 65536):
    """embedding_generate.py:109-131.  `article_features` is the reference's
    {article_id: feature(253)} dict or an (ids, features) pair.  Returns
    (ids int64 (N,), emb float32 (N, 256)); with out_path, also writes them as
    a typed .npz (keys "ids", "emb")."""
    if isinstance(article_features, dict):
        ids = np.fromiter(article_features.keys(), dtype=np.int64, count=len(article_features))
        feats = np.stack([np.asarray(article_features[int(a)], dtype=np.float32) for a in ids])
    else:
        ids, feats = article_features
        ids = np.asarray(ids, dtype=np.int64)
        feats = np.ascontiguousarray(feats, dtype=np.float32)
    if device is None:
        # the model's device, or the GPU for a model loaded on the host (a
        # checkpoint read with map_location="cpu"): embed() runs on the GPU only
        device = next(model.parameters()).device
        if device.type != "cuda" and torch.cuda.is_available():
            device = torch.device("cuda", torch.cuda.current_device())
    model = model.to(device).eval()
    x = torch.from_numpy(feats).to(device)
    emb = model.embed(x, batch=batch).cpu().numpy()
    if out_path is not None:
        np.savez(out_path, ids=ids, emb=emb)
    return ids, emb


def load_article_table(path: str):
    """Retrieval.py:6-9 -> (ids int64 (N,), embeddings float32 (N, d))."""
    if path.endswith(".npz"):
        z = np.load(path)
        return z["ids"].astype(np.int64), np.ascontiguousarray(z["emb"], dtype=np.float32)
    table = np.load(path)  # numeric (N, d+1) table; object arrays are refused (allow_pickle=False)
    return table[:, -1].astype(np.int64), np.ascontiguousarray(table[:, :-1], dtype=np.float32)


class ArticleTripletDataset(torch.utils.data.Dataset):
    """embedding_generate.py:25-49: for every user and every ordered pair of
    clicks (i < j): (anchor = click i, positive = click j, negative = a random
    article the user never clicked).  Items are ids; features are gathered on
    the device by train_triplet."""

    def __init__(self, user_clicks: dict, all_article_ids, rng=random):
        all_ids = list(all_article_ids)
        trip = []
        for _, clicked_articles in user_clicks.items():
            clicked = set(clicked_articles)
            if len(clicked_articles) < 2:
                continue
            for i in range(len(clicked_articles) - 1):
                for j in range(i + 1, len(clicked_articles)):
                    neg = rng.choice(all_ids)
                    while neg in clicked:
                        neg = rng.choice(all_ids)
                    trip.append((clicked_articles[i], clicked_articles[j], neg))
        self.triplets = np.asarray(trip, dtype=np.int64).reshape(-1, 3)

    @classmethod
    def from_click_log(cls, log, all_article_ids, rng=random) -> "ArticleTripletDataset":
        """The same triplets (and `random` draws) from a typed data.ClickLog,
        built by libnrk's host builder (nrk_triplet_samples) instead of the
        per-pair Python loop."""
        from . import _lib
        from .data import ArticleTable, _rng_restore, _rng_words

        ids = np.asarray(list(all_article_ids), dtype=np.int64)
        rows = ArticleTable(ids, np.zeros((len(ids), 0), np.float32)).rows(log.clicks)
        lens = np.diff(log.offsets)
        n = int((lens * (lens - 1) // 2)[lens >= 2].sum())
        out = np.empty((n, 3), np.int32)
        st, words = _rng_words(rng)
        rc = _lib.load().nrk_triplet_samples(log.offsets.ctypes.data, len(log), rows.ctypes.data, len(ids),
                                             words.ctypes.data, n, out.ctypes.data)
        _rng_restore(rng, st, words)
        _lib.check(rc, "ArticleTripletDataset.from_click_log")
        self = cls.__new__(cls)
        self.triplets = ids[out]
        return self

    def __len__(self):
        return len(self.triplets)

    def __getitem__(self, idx):
        return self.triplets[idx]


def train_triplet(model, triplets: np.ndarray, id_to_row: dict, features: torch.Tensor, optimizer,
                  batch_size: int = 64, margin: float = MARGIN, shuffle_seed: int | None = 0):
    """One epoch of embedding_generate.py:88-100 over id triplets; features
    (N, 253) live on the device, rows looked up by id.  Returns the mean of
    loss * batch rows, as the reference's running_loss / len(loader)."""
    dev = features.device
    rows = torch.from_numpy(np.vectorize(id_to_row.__getitem__)(triplets).astype(np.int64)).to(dev)
    crit = nn.TripletMarginLoss(margin=margin, p=2)
    order = np.arange(len(rows))
    if shuffle_seed is not None:
        np.random.default_rng(shuffle_seed).shuffle(order)
    order = torch.from_numpy(order).to(dev)
    model.train()
    running = torch.zeros((), dtype=torch.float64, device=dev)
    nb = 0
    for lo in range(0, len(order), batch_size):
        r = rows[order[lo:lo + batch_size]]
        optimizer.zero_grad()
        a, p, n = (model(features[r[:, c]]) for c in range(3))
        loss = crit(a, p, n)
        loss.backward()
        optimizer.step()
        running += loss.detach() * r.shape[0]
        nb += 1
    return (running / max(nb, 1)).item()


def _triplet_rows(triplets, ids: np.ndarray, device) -> torch.Tensor:
    from .data import ArticleTable

    rows = ArticleTable(ids, np.zeros((len(ids), 0), np.float32)).rows(np.asarray(triplets, np.int64))
    return torch.from_numpy(rows.astype(np.int64)).to(device)


def fit_triplet(model, train_triplets, test_triplets, article_ids, features: torch.Tensor, epochs: int = 3,
                batch_size: int = 64, lr: float = LR, weight_decay: float = WEIGHT_DECAY, margin: float = MARGIN,
                save_path: str | None = None):
    """embedding_generate.py:67-107 (main()) over id triplets, features
    (N, 253) resident on the device in `article_ids` order.

    Same loop as the reference: shuffled DataLoaders over the train and test
    triplets (same sampler, so the same torch RNG draws and batch order),
    TripletMarginLoss(margin, p=2), Adam(lr, weight_decay); per epoch
    train_loss = Σ loss·rows / number of batches (running_loss /
    len(trainDataloader), :92) and the same for the eval pass (:103); the
    state_dict with the lowest eval loss is kept (:105-107) and saved to
    `save_path` if given.  The rows are gathered from `features` on the device
    by index batches instead of per-item dict lookups (:45-49).
    Returns (history [(train_loss, eval_loss)], best_state_dict)."""
    dev = features.device
    ids = np.asarray(article_ids, np.int64)
    tr_rows = _triplet_rows(train_triplets, ids, dev).reshape(-1, 3)
    te_rows = _triplet_rows(test_triplets, ids, dev).reshape(-1, 3)
    loader = lambda n: torch.utils.data.DataLoader(range(n), batch_size=batch_size, shuffle=True)  # noqa: E731
    tr_loader, te_loader = loader(len(tr_rows)), loader(len(te_rows))
    crit = nn.TripletMarginLoss(margin=margin, p=2)
    opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay)
    best_loss, best_sd, history = float("inf"), None, []
    for _ in range(epochs):
        model.train()
        running = 0.0
        for idx in tr_loader:
            r = tr_rows[idx.to(dev)]
            opt.zero_grad()
            a, p, n = (model(features[r[:, c]]) for c in range(3))
            loss = crit(a, p, n)
            loss.backward()
            opt.step()
            running += loss.item() * r.shape[0]
        train_loss = running / len(tr_loader)
        running = 0.0
        model.eval()
        with torch.no_grad():
            for idx in te_loader:
                r = te_rows[idx.to(dev)]
                a, p, n = (model(features[r[:, c]]) for c in range(3))
                running += crit(a, p, n).item() * r.shape[0]
        eval_loss = running / len(te_loader)
        history.append((train_loss, eval_loss))
        if eval_loss < best_loss:
            best_loss = eval_loss
            best_sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
            if save_path is not None:
                torch.save(model.state_dict(), save_path)
    return history, best_sd
