"""Generate the golden fixtures under tests/golden/ by RUNNING THE REFERENCE.

Build-container tool only: it imports /root/reference/DIN.py and
/root/reference/embedding_generate.py (read-only, no bytecode written), feeds
them small synthetic inputs and records inputs + outputs as .npz data.  Nothing
of the reference's source is copied; the GPU box only ever sees the .npz files.

Import recipe: DIN.py imports `optuna` (DIN.py:9, used only by
the disabled `objective`, DIN.py:195-223,260-262) -> a stub module; both files
np.load() their data from `news/` at import time (DIN.py:14-19,
embedding_generate.py:20-22) -> we chdir into a temp dir holding synthetic
`news/*.npy` dict-pickles that THIS script writes.

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import importlib.util
import os
import random
import sys
import tempfile
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_ref(name: str, workdir: str):
    sys.dont_write_bytecode = True
    sys.modules.setdefault("optuna", types.ModuleType("optuna"))
    cwd = os.getcwd()
    os.chdir(workdir)
    try:
        spec = importlib.util.spec_from_file_location(f"ref_{name}", os.path.join(REF, f"{name}.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        os.chdir(cwd)
    return mod


def _sd(model) -> dict:
    return {f"sd::{k}": v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}


def _write_news(workdir, article_emb, train_clicks, test_clicks, test_recs, extra=None):
    os.makedirs(os.path.join(workdir, "news"), exist_ok=True)
    p = lambda n: os.path.join(workdir, "news", n)  # noqa: E731
    np.save(p("article_dict.npy"), article_emb, allow_pickle=True)
    np.save(p("train_user_clicked_article_ids.npy"), train_clicks, allow_pickle=True)
    np.save(p("test_user_clicked_article_ids.npy"), test_clicks, allow_pickle=True)
    np.save(p("test_user_recommendations.npy"), test_recs, allow_pickle=True)
    for k, v in (extra or {}).items():
        np.save(p(k), v, allow_pickle=True)


def _synthetic_world(seed, n_items, d, n_train_users, n_test_users, max_clicks, n_cand):
    rng = np.random.default_rng(seed)
    ids = rng.choice(np.arange(1000, 1000 + 10 * n_items), size=n_items, replace=False)
    table = rng.standard_normal((n_items, d)).astype(np.float32) * 0.5
    article_emb = {int(a): table[i] for i, a in enumerate(ids)}
    train_clicks = {}
    for u in range(n_train_users):
        n = int(rng.integers(1, max_clicks + 1))
        train_clicks[100 + u] = [int(x) for x in rng.choice(ids, size=n, replace=False)]
    test_clicks, test_recs = {}, {}
    for u in range(n_test_users):
        n = int(rng.integers(1, max_clicks + 1))
        clicks = [int(x) for x in rng.choice(ids, size=n, replace=False)]
        uid = 5000 + u
        test_clicks[uid] = clicks
        c = int(rng.integers(n_cand // 2, n_cand + 1))
        cands = rng.choice(ids, size=c, replace=False).astype(np.int64)
        if rng.random() < 0.7 and clicks[-1] not in set(cands.tolist()):
            cands[int(rng.integers(0, c))] = clicks[-1]
        test_recs[uid] = cands
    return ids, table, article_emb, train_clicks, test_clicks, test_recs


def _pad_hist(hist_lists, L):
    out = np.full((len(hist_lists), L), -1, dtype=np.int64)
    for i, h in enumerate(hist_lists):
        out[i, : len(h)] = h
    return out


def _random_bn_stats(model, gen):
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm1d):
            m.running_mean.copy_(torch.randn(m.num_features, generator=gen) * 0.3)
            m.running_var.copy_(torch.rand(m.num_features, generator=gen) * 1.5 + 0.25)
            m.weight.data.copy_(torch.rand(m.num_features, generator=gen) + 0.5)
            m.bias.data.copy_(torch.randn(m.num_features, generator=gen) * 0.1)


def din_forward_fixture(name, d, A, F, B, L, n_items, seed):
    """Eval-mode DIN + AttentionLayer outputs (DIN.py:94-137)."""
    with tempfile.TemporaryDirectory() as wd:
        ids, table, emb, trc, tec, ter = _synthetic_world(seed, n_items, d, 4, 4, 6, 10)
        _write_news(wd, emb, trc, tec, ter)
        ref = _import_ref("DIN", wd)
        torch.manual_seed(seed)
        model = ref.DIN(d, A, F, 0.36)
        init_sd = _sd(model)  # right after the reference init (xavier_normal_, DIN.py:124-128)
        gen = torch.Generator().manual_seed(seed + 1)
        _random_bn_stats(model, gen)
        model.eval()
        rng = np.random.default_rng(seed + 2)
        hist_len = rng.integers(0, L + 1, size=B)
        hist_len[0], hist_len[1] = 0, L  # empty and full histories (all-padding / no padding)
        rows = rng.integers(0, n_items, size=(B, L))
        hist_idx = np.where(np.arange(L)[None, :] < hist_len[:, None], rows, -1)
        tgt_idx = rng.integers(0, n_items, size=B)
        keys = np.where(hist_idx[..., None] >= 0, table[np.maximum(hist_idx, 0)], 0.0).astype(np.float32)
        query = table[tgt_idx].astype(np.float32)
        with torch.no_grad():
            q = torch.from_numpy(query)
            k = torch.from_numpy(keys)
            pooled = model.attn(q, k).numpy()
            # attention weights through the reference's own sub-module (DIN.py:105-108)
            attn_in = torch.cat([q.unsqueeze(1).repeat(1, L, 1), k], dim=2).view(-1, 2 * d)
            alpha = torch.softmax(model.attn.attn(attn_in).view(B, L), dim=1).numpy()
            logits = model(q, k).numpy()
            probs = model.predict(q, k).numpy()
        np.savez_compressed(
            os.path.join(OUT, f"{name}.npz"),
            d=d, A=A, F=F, B=B, L=L, table=table, hist_idx=hist_idx.astype(np.int32),
            tgt_idx=tgt_idx.astype(np.int32), query=query, pooled=pooled, alpha=alpha,
            logits=logits, probs=probs, **_sd(model), **{f"init_{k}": v for k, v in init_sd.items()},
        )


def din_train_fixture(name, d, A, F, B, L, n_items, seed):
    """Two reference train() steps (DIN.py:139-153) with dropout 0 (dropout RNG
    cannot be matched across devices), Adam(lr=1.62e-3, wd=8.96e-5) and
    BCEWithLogitsLoss exactly as main() (DIN.py:231-247)."""
    with tempfile.TemporaryDirectory() as wd:
        ids, table, emb, trc, tec, ter = _synthetic_world(seed, n_items, d, 4, 4, 6, 10)
        _write_news(wd, emb, trc, tec, ter)
        ref = _import_ref("DIN", wd)
        torch.manual_seed(seed)
        model = ref.DIN(d, A, F, 0.0)
        sd0 = _sd(model)
        rng = np.random.default_rng(seed + 3)
        batches = []
        arrays = {}
        for s in range(2):
            hist_len = rng.integers(1, L + 1, size=B)
            rows = rng.integers(0, n_items, size=(B, L))
            hist_idx = np.where(np.arange(L)[None, :] < hist_len[:, None], rows, -1)
            tgt_idx = rng.integers(0, n_items, size=B)
            label = (rng.random(B) < 0.5).astype(np.float32)[:, None]
            keys = np.where(hist_idx[..., None] >= 0, table[np.maximum(hist_idx, 0)], 0.0).astype(np.float32)
            batches.append({
                "uid": list(range(B)),
                "history_emb": torch.from_numpy(keys),
                "target_emb": torch.from_numpy(table[tgt_idx].astype(np.float32)),
                "label": torch.from_numpy(label),
            })
            arrays[f"hist_idx{s}"] = hist_idx.astype(np.int32)
            arrays[f"tgt_idx{s}"] = tgt_idx.astype(np.int32)
            arrays[f"label{s}"] = label
        crit = torch.nn.BCEWithLogitsLoss()
        # unclipped gradients of batch 0 (what train() computes before clip_grad_norm_)
        model.train()
        loss0 = crit(model(batches[0]["target_emb"], batches[0]["history_emb"]), batches[0]["label"])
        loss0.backward()
        grads0 = {f"grad::{n}": p.grad.detach().numpy().copy() for n, p in model.named_parameters()}
        model.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in sd0.items()})
        model.zero_grad()
        opt = torch.optim.Adam(model.parameters(), lr=1.62e-3, weight_decay=8.96e-5)
        mean_loss = ref.train(model, batches, opt, crit, torch.device("cpu"))
        sd_after = {f"after::{k[4:]}": v for k, v in _sd(model).items()}
        np.savez_compressed(
            os.path.join(OUT, f"{name}.npz"),
            d=d, A=A, F=F, B=B, L=L, table=table, loss0=np.float64(loss0.item()),
            mean_loss=np.float64(mean_loss), **arrays, **sd0, **grads0, **sd_after,
        )


def din_dataset_fixture(name, seed):
    """TrainDataset / EvalDataset / evaluate() (DIN.py:21-92,155-193)."""
    with tempfile.TemporaryDirectory() as wd:
        d, L = 16, 8
        ids, table, emb, trc, tec, ter = _synthetic_world(seed, 200, d, 30, 25, 12, 40)
        _write_news(wd, emb, trc, tec, ter)
        ref = _import_ref("DIN", wd)
        random.seed(42)  # as main(), DIN.py:228
        tr = ref.TrainDataset(L)
        uid = np.array([s["uid"] for s in tr.samples], np.int64)
        tgt = np.array([s["target"] for s in tr.samples], np.int64)
        lab = np.array([s["label"] for s in tr.samples], np.int64)
        hist = _pad_hist([s["history"] for s in tr.samples], L)
        item0 = tr[3]
        ev = ref.EvalDataset(L)
        ev_uid = np.array([s["uid"] for s in ev.data], np.int64)
        ev_hist = _pad_hist([s["history"] for s in ev.data], L)
        ev_cand_len = np.array([len(s["candidates"]) for s in ev.data], np.int64)
        ev_cand = np.concatenate([np.asarray(s["candidates"], np.int64) for s in ev.data])
        ev_lab = np.concatenate([np.asarray(s["labels"], np.int64) for s in ev.data])
        torch.manual_seed(seed)
        model = ref.DIN(d, 32, 32, 0.36)
        gen = torch.Generator().manual_seed(seed + 1)
        _random_bn_stats(model, gen)
        loader = torch.utils.data.DataLoader(ev, batch_size=8, shuffle=False, num_workers=0,
                                             collate_fn=ref.custom_collate_fn)
        crit = torch.nn.BCEWithLogitsLoss()
        ev_loss, ev_ndcg = ref.evaluate(model, loader, crit, torch.device("cpu"), 5)
        # per-user logits via the reference model for the same pairs (DIN.py:168-175)
        per_user = []
        model.eval()
        with torch.no_grad():
            for b in loader:
                for i in range(len(b["uid"])):
                    c = b["cand_embs"][i]
                    per_user.append(model(c, b["history_emb"][i].unsqueeze(0).expand(c.size(0), -1, -1)).view(-1).numpy())
        np.savez_compressed(
            os.path.join(OUT, f"{name}.npz"),
            d=d, L=L, item_ids=ids.astype(np.int64), table=table,
            train_users=np.array(list(trc.keys()), np.int64),
            train_click_len=np.array([len(v) for v in trc.values()], np.int64),
            train_clicks=np.concatenate([np.asarray(v, np.int64) for v in trc.values()]),
            test_users=np.array(list(tec.keys()), np.int64),
            test_click_len=np.array([len(v) for v in tec.values()], np.int64),
            test_clicks=np.concatenate([np.asarray(v, np.int64) for v in tec.values()]),
            rec_users=np.array(list(ter.keys()), np.int64),
            rec_len=np.array([len(v) for v in ter.values()], np.int64),
            recs=np.concatenate([np.asarray(v, np.int64) for v in ter.values()]),
            tr_uid=uid, tr_hist=hist, tr_target=tgt, tr_label=lab,
            item3_hist=item0["history_emb"].numpy(), item3_target=item0["target_emb"].numpy(),
            item3_label=item0["label"].numpy(),
            ev_uid=ev_uid, ev_hist=ev_hist, ev_cand_len=ev_cand_len, ev_cand=ev_cand, ev_lab=ev_lab,
            ev_loss=np.float64(ev_loss), ev_ndcg=np.float64(ev_ndcg),
            ev_logits=np.concatenate(per_user), **_sd(model),
        )


def din_rerank_fixture(name, seed, d=256, L=50, n_users=24, n_cand=201, n_items=1200, bf16_exact=True):
    """configs[4]'s re-rank shape through the reference's own EvalDataset +
    evaluate() (DIN.py:21-57,155-193): d = 256, L = 50, 201 candidates per
    user, DIN(256, 128, 32, 0.36) in eval mode with non-trivial BN statistics.
    bf16_exact: the item table is rounded to bf16-representable values so the
    same numbers feed the reference's fp32 forward and the bf16-table GPU path;
    otherwise it is a plain fp32 table, as embedding_generate.py produces (the
    bf16-table path then sees each embedding rounded once)."""
    with tempfile.TemporaryDirectory() as wd:
        rng = np.random.default_rng(seed)
        ids = rng.choice(np.arange(1000, 1000 + 10 * n_items), size=n_items, replace=False)
        table = torch.from_numpy(rng.standard_normal((n_items, d)).astype(np.float32) * 0.5)
        table = table.to(torch.bfloat16).float().numpy() if bf16_exact else table.numpy()
        emb = {int(a): table[i] for i, a in enumerate(ids)}
        test_clicks, test_recs = {}, {}
        for u in range(n_users):
            n = int(rng.integers(2, L + 12))  # histories of 1..L+10 clicks: short, full and truncated
            clicks = [int(x) for x in rng.choice(ids, size=n, replace=False)]
            cands = rng.choice(ids, size=n_cand, replace=False).astype(np.int64)
            if u % 4 != 3 and clicks[-1] not in set(cands.tolist()):
                cands[int(rng.integers(0, n_cand))] = clicks[-1]
            test_clicks[7000 + u] = clicks
            test_recs[7000 + u] = cands
        _write_news(wd, emb, {1: [int(ids[0]), int(ids[1])]}, test_clicks, test_recs)
        ref = _import_ref("DIN", wd)
        torch.manual_seed(seed)
        model = ref.DIN(d, 128, 32, 0.36)
        _random_bn_stats(model, torch.Generator().manual_seed(seed + 1))
        ev = ref.EvalDataset(L)
        loader = torch.utils.data.DataLoader(ev, batch_size=8, shuffle=False, num_workers=0,
                                             collate_fn=ref.custom_collate_fn)
        ev_loss, ev_ndcg = ref.evaluate(model, loader, torch.nn.BCEWithLogitsLoss(), torch.device("cpu"), 5)
        per_logits, per_ndcg = [], []
        model.eval()
        with torch.no_grad():
            for b in loader:
                for i in range(len(b["uid"])):
                    c = b["cand_embs"][i]
                    lg = model(c, b["history_emb"][i].unsqueeze(0).expand(c.size(0), -1, -1)).view(-1)
                    per_logits.append(lg.numpy())
                    probs = torch.sigmoid(lg).numpy()
                    labs = b["labels"][i].numpy()
                    nd = 0.0
                    for rank, idx in enumerate(np.argsort(-probs)[:5], start=1):  # DIN.py:183-188
                        if labs[idx] == 1:
                            nd = 1 / np.log2(rank + 1)
                            break
                    per_ndcg.append(nd)
        assert abs(float(np.mean(per_ndcg)) - ev_ndcg) < 1e-12
        np.savez_compressed(
            os.path.join(OUT, f"{name}.npz"),
            d=d, L=L, A=128, F=32, item_ids=ids.astype(np.int64), table=table,
            ev_uid=np.array([s["uid"] for s in ev.data], np.int64),
            ev_hist=_pad_hist([s["history"] for s in ev.data], L),
            ev_cand=np.stack([np.asarray(s["candidates"], np.int64) for s in ev.data]),
            ev_lab=np.stack([np.asarray(s["labels"], np.int64) for s in ev.data]),
            ev_loss=np.float64(ev_loss), ev_ndcg=np.float64(ev_ndcg),
            ev_logits=np.stack(per_logits), ev_ndcg_user=np.array(per_ndcg, np.float64), **_sd(model),
        )


def din_rerank_cluster_fixture(name, seed, d=256, L=64, n_users=12, sizes=(403, 1187, 4410)):
    """The candidate geometry the reference actually scores: Retrieval.py:28-34
    hands each user the WHOLE nearest cluster (400-4,974 ragged candidates per
    user, readme.md:20), scored by the reference's own EvalDataset + evaluate()
    (DIN.py:21-57,155-193) at main()'s max_history L = 64 (DIN.py:237) and the
    256-d corpus (embedding_generate.py:14).  Items are split into clusters
    (member lists in corpus row order, as `ids[assign == i]` keeps them); user
    u gets cluster u % len(sizes); for 3 of every 4 users the last click is a
    member of that cluster (labelled), otherwise every label is 0.  The table
    is bf16-representable (stored as bf16 bits) so the same numbers feed the
    reference's fp32 forward and the bf16-table GPU path."""
    with tempfile.TemporaryDirectory() as wd:
        rng = np.random.default_rng(seed)
        n_items = int(sum(sizes))
        ids = rng.choice(np.arange(1000, 1000 + 10 * n_items), size=n_items, replace=False)
        table = torch.from_numpy(rng.standard_normal((n_items, d)).astype(np.float32) * 0.5).to(torch.bfloat16)
        table_bits = table.view(torch.int16).numpy().view(np.uint16).copy()
        table = table.float().numpy()
        emb = {int(a): table[i] for i, a in enumerate(ids)}
        assign = np.repeat(np.arange(len(sizes)), sizes)
        rng.shuffle(assign)
        members = [np.nonzero(assign == c)[0] for c in range(len(sizes))]  # corpus row order
        test_clicks, test_recs, user_cluster = {}, {}, []
        for u in range(n_users):
            c = u % len(sizes)
            n = int(rng.integers(2, L + 12))  # 1..L+10 history clicks: short, full and truncated
            rows = [int(x) for x in rng.choice(n_items, size=n, replace=False)]
            if u % 4 != 3:
                last = int(rng.choice(members[c]))
                rows = [r for r in rows if r != last][: n - 1] + [last]
            else:
                rows = [r for r in rows if assign[r] != c] or [int(np.nonzero(assign != c)[0][0])] * 2
            test_clicks[9000 + u] = [int(ids[r]) for r in rows]
            test_recs[9000 + u] = ids[members[c]].astype(np.int64)
            user_cluster.append(c)
        _write_news(wd, emb, {1: [int(ids[0]), int(ids[1])]}, test_clicks, test_recs)
        ref = _import_ref("DIN", wd)
        torch.manual_seed(seed)
        model = ref.DIN(d, 128, 32, 0.36)
        _random_bn_stats(model, torch.Generator().manual_seed(seed + 1))
        ev = ref.EvalDataset(L)
        loader = torch.utils.data.DataLoader(ev, batch_size=8, shuffle=False, num_workers=0,
                                             collate_fn=ref.custom_collate_fn)
        ev_loss, ev_ndcg = ref.evaluate(model, loader, torch.nn.BCEWithLogitsLoss(), torch.device("cpu"), 5)
        per_logits, per_ndcg = [], []
        model.eval()
        with torch.no_grad():
            for b in loader:
                for i in range(len(b["uid"])):
                    c = b["cand_embs"][i]
                    lg = model(c, b["history_emb"][i].unsqueeze(0).expand(c.size(0), -1, -1)).view(-1)
                    per_logits.append(lg.numpy())
                    probs = torch.sigmoid(lg).numpy()
                    labs = b["labels"][i].numpy()
                    nd = 0.0
                    for rank, idx in enumerate(np.argsort(-probs)[:5], start=1):  # DIN.py:183-188
                        if labs[idx] == 1:
                            nd = 1 / np.log2(rank + 1)
                            break
                    per_ndcg.append(nd)
        assert abs(float(np.mean(per_ndcg)) - ev_ndcg) < 1e-12
        row_of = {int(a): i for i, a in enumerate(ids)}
        np.savez_compressed(
            os.path.join(OUT, f"{name}.npz"),
            d=d, L=L, A=128, F=32, item_ids=ids.astype(np.int64), table_bf16=table_bits,
            cluster_sizes=np.asarray(sizes, np.int64), cluster_rows=np.concatenate(members).astype(np.int32),
            user_cluster=np.asarray([user_cluster[s["uid"] - 9000] for s in ev.data], np.int64),
            ev_uid=np.array([s["uid"] for s in ev.data], np.int64),
            ev_hist_rows=_pad_hist([[row_of[int(a)] for a in s["history"]] for s in ev.data], L).astype(np.int32),
            ev_cand_len=np.array([len(s["candidates"]) for s in ev.data], np.int64),
            ev_lab=np.concatenate([np.asarray(s["labels"], np.int8) for s in ev.data]),
            ev_loss=np.float64(ev_loss), ev_ndcg=np.float64(ev_ndcg),
            ev_logits=np.concatenate(per_logits), ev_ndcg_user=np.array(per_ndcg, np.float64), **_sd(model),
        )


def embedding_fixture(name, seed, n_articles=48):
    """ArticleEmbeddingModel + inference() (embedding_generate.py:51-65,109-131)."""
    with tempfile.TemporaryDirectory() as wd:
        rng = np.random.default_rng(seed)
        aids = rng.choice(np.arange(10, 10 * n_articles + 10), size=n_articles, replace=False)
        feats = rng.standard_normal((n_articles, 253)).astype(np.float32)
        a2f = {int(a): feats[i] for i, a in enumerate(aids)}
        clicks = {1: [int(aids[0]), int(aids[1])]}
        _write_news(wd, {0: np.zeros(4, np.float32)}, clicks, clicks, {}, {
            "article_embedding_dict.npy": a2f})
        ref = _import_ref("embedding_generate", wd)
        torch.manual_seed(seed)
        m = ref.ArticleEmbeddingModel(253, 512, 256, 0.13)
        gen = torch.Generator().manual_seed(seed + 1)
        _random_bn_stats(m, gen)
        torch.save(m.state_dict(), os.path.join(wd, "news", "best_eg_model.pth"))
        cwd = os.getcwd()
        os.chdir(wd)
        try:
            ref.inference()
            out = np.load("article_dict.npy", allow_pickle=True).item()  # file written by the reference run above
            try:
                np.load("article_table.npy")  # how Retrieval.py:6 loads it
                table_loadable = True
            except ValueError:
                table_loadable = False
        finally:
            os.chdir(cwd)
        emb = np.stack([out[int(a)] for a in aids]).astype(np.float32)
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), aids=aids.astype(np.int64), feats=feats,
                            emb=emb, table_loadable=np.bool_(table_loadable), **_sd(m))


def embedding_train_fixture(name, seed, n_articles=120, n_train=16, n_test=9, max_clicks=8):
    """The reference's triplet training main() (embedding_generate.py:67-107),
    run as written (3 epochs, batch 64, shuffled loaders, dropout 0.13, Adam
    with weight decay, best-eval-loss checkpoint) on a small synthetic world.
    Every TripletMarginLoss value main() computes is recorded by handing the
    module a loss subclass that logs (value, batch rows, train/eval)."""
    with tempfile.TemporaryDirectory() as wd:
        rng = np.random.default_rng(seed)
        aids = rng.choice(np.arange(10, 10 * n_articles + 10), size=n_articles, replace=False)
        feats = rng.standard_normal((n_articles, 253)).astype(np.float32)
        a2f = {int(a): feats[i] for i, a in enumerate(aids)}

        def clicks(n_users, base):
            return {base + u: [int(x) for x in rng.choice(aids, size=int(rng.integers(1, max_clicks + 1)),
                                                          replace=False)] for u in range(n_users)}

        trc, tec = clicks(n_train, 100), clicks(n_test, 900)
        _write_news(wd, {0: np.zeros(4, np.float32)}, trc, tec, {}, {"article_embedding_dict.npy": a2f})
        ref = _import_ref("embedding_generate", wd)
        log = []

        class RecordingLoss(torch.nn.TripletMarginLoss):
            def forward(self, a, p, n):
                out = super().forward(a, p, n)
                log.append((float(out.detach()), a.shape[0], torch.is_grad_enabled()))
                return out

        class NNProxy:  # the module's `nn` with TripletMarginLoss swapped for the recorder
            TripletMarginLoss = RecordingLoss

            def __getattr__(self, k):
                return getattr(torch.nn, k)

        ref.nn = NNProxy()
        ref.tqdm = lambda it, desc=None: it
        random.seed(seed)
        torch.manual_seed(seed)
        cwd = os.getcwd()
        os.chdir(wd)
        try:
            ref.main()
            best = torch.load(os.path.join("news", "best_eg_model.pth"), weights_only=True)  # written by main() above
        finally:
            os.chdir(cwd)
        random.seed(seed)  # the triplets main() built (the datasets are its first `random` consumers)
        tr = np.asarray(ref.ArticleTripletDataset(True).triplets, np.int64)
        te = np.asarray(ref.ArticleTripletDataset(False).triplets, np.int64)
        np.savez_compressed(
            os.path.join(OUT, f"{name}.npz"), seed=np.int64(seed), aids=aids.astype(np.int64), feats=feats,
            train_users=np.array(list(trc.keys()), np.int64),
            train_click_len=np.array([len(v) for v in trc.values()], np.int64),
            train_clicks=np.concatenate([np.asarray(v, np.int64) for v in trc.values()]),
            test_users=np.array(list(tec.keys()), np.int64),
            test_click_len=np.array([len(v) for v in tec.values()], np.int64),
            test_clicks=np.concatenate([np.asarray(v, np.int64) for v in tec.values()]),
            train_triplets=tr, test_triplets=te,
            loss_values=np.array([v for v, _, _ in log], np.float64),
            loss_rows=np.array([b for _, b, _ in log], np.int64),
            loss_train=np.array([g for _, _, g in log], np.bool_),
            **{f"best::{k}": v.numpy() for k, v in best.items()})


def main():
    torch.set_num_threads(4)
    if sys.argv[1:] == ["embedding_train"]:  # regenerate only the triplet-training fixture
        embedding_train_fixture("embedding_train", seed=18)
        return
    if sys.argv[1:] == ["din_rerank_cluster"]:  # regenerate only the whole-cluster re-rank fixture
        din_rerank_cluster_fixture("din_rerank_cluster", seed=19)
        return
    if sys.argv[1:] == ["din_rerank_f32"]:  # regenerate only the fp32-table re-rank fixture
        din_rerank_fixture("din_rerank_f32", seed=20, n_users=16, bf16_exact=False)
        return
    din_forward_fixture("din_fwd_c1", d=64, A=32, F=32, B=64, L=20, n_items=300, seed=11)
    din_forward_fixture("din_fwd_c3", d=128, A=128, F=32, B=96, L=50, n_items=600, seed=12)
    din_train_fixture("din_train_c1", d=64, A=32, F=32, B=48, L=20, n_items=300, seed=13)
    din_train_fixture("din_train_c3", d=128, A=128, F=32, B=32, L=50, n_items=400, seed=14)
    din_dataset_fixture("din_dataset", seed=15)
    embedding_fixture("embedding_infer", seed=16)
    din_rerank_fixture("din_rerank_c5", seed=17)
    embedding_train_fixture("embedding_train", seed=18)
    din_rerank_cluster_fixture("din_rerank_cluster", seed=19)
    din_rerank_fixture("din_rerank_f32", seed=20, n_users=16, bf16_exact=False)
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
