"""DIN ranker on MI355X — drop-in for the reference's DIN.py call surface.

Same names, constructor arguments, forward signatures and state_dict keys as
the reference (DIN.py:94-137), so `news/DIN_model.pth` checkpoints load both
ways.  The attention layer's arithmetic (DIN.py:103-111) runs in libnrk's HIP
kernels (K-LAU-POOL fwd/bwd, with the history gather fused in); the small
BN/MLP head (DIN.py:117-122, ~1% of the flops) stays in torch.

Two ways in:
  * `DIN.forward(query, history)` — the reference's dense form: query (b, d),
    history (b, L, d) (fp32 gives the fp32 parity path; bf16 the bf16 path).
  * `DIN.forward_ids(table, target_ids, hist_ids)` — the id form: a device-
    resident embedding table (N, d) (fp32 or bf16) plus int32 ids, padding
    id -1 meaning an all-zero row (as DIN.py:84-86 zero-fills).  This removes
    the CPU gather and host->device copy of TrainDataset.__getitem__.

There is no CPU path: CPU tensors raise (use oracle/din_oracle.py, a test-only
restatement, for CPU checks).
"""
from __future__ import annotations

import ctypes
import os
import warnings

import torch
import torch.nn as nn
import torch.nn.functional as F  # noqa: F401  (parity with the reference's imports)

from . import _lib


def _dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return _lib.NRK_DTYPE_F32
    if t.dtype == torch.bfloat16:
        return _lib.NRK_DTYPE_BF16
    raise TypeError(f"DIN attention supports float32 / bfloat16 embeddings, got {t.dtype}")


_KERNEL_DIMS = (32, 64, 128, 256)


def _kernel_dim(d: int) -> int:
    """Embedding widths with a compiled kernel; other widths are zero-padded
    (zero columns change neither z, alpha nor the pooled sum)."""
    for k in _KERNEL_DIMS:
        if d <= k:
            return k
    raise ValueError(f"DIN attention: emb_dim {d} > 256 is not supported")


def _pad_last(t: torch.Tensor, width: int) -> torch.Tensor:
    return t if t.shape[-1] == width else torch.nn.functional.pad(t, (0, width - t.shape[-1]))


class KernelTimer:
    """Bench hook: while active, brackets each kernel launch that marks itself
    (the attention kernels: "fwd" / "bwd"; the fused re-rank: "rerank") with
    torch.cuda.Event pairs on the launch stream (the current stream)."""

    active = None

    def __init__(self):
        self.ev = {}

    def __enter__(self):
        KernelTimer.active = self
        return self

    def __exit__(self, *exc):
        KernelTimer.active = None

    @staticmethod
    def mark(kind):
        t = KernelTimer.active
        if t is None:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    @staticmethod
    def push(kind, start):
        t = KernelTimer.active
        if t is None or start is None:
            return
        end = torch.cuda.Event(enable_timing=True)
        end.record()
        t.ev.setdefault(kind, []).append((start, end))

    def mean_ms(self, kind, skip=0):
        ev = self.ev.get(kind, [])[skip:]
        return sum(a.elapsed_time(b) for a, b in ev) / max(len(ev), 1)


class _LauPool(torch.autograd.Function):
    """AttentionLayer forward/backward through nrk_din_attn_fwd/bwd.

    keys_src is either dense keys (B, L, d) (hist_ids None) or a table (N, d)
    addressed by hist_ids (B, L) int32.  Gradients flow to W1, b1, W2, b2 and
    the query; the keys/table are frozen inputs as in the reference."""

    @staticmethod
    def forward(ctx, query, W1, b1, W2, b2, keys_src, hist_ids, L):
        dev = _lib.require_device(query, W1, keys_src, hist_ids, what="DIN attention")
        B, d = query.shape
        A = W1.shape[0]
        dtype = _dtype_code(keys_src)
        Dk = _kernel_dim(d)
        keys_src = _pad_last(keys_src, Dk).contiguous()
        U = torch.addmm(b1, query, W1[:, :d].t()).contiguous()  # (B, A) f32: the query half of W1 [q; k] + b1
        W1k = _pad_last(W1[:, d:], Dk).contiguous()
        W1k_k = W1k if dtype == _lib.NRK_DTYPE_F32 else W1k.to(torch.bfloat16)
        w2 = W2.reshape(-1).contiguous()
        pooled = torch.empty((B, Dk), dtype=torch.float32, device=dev)
        alpha = torch.empty((B, L), dtype=torch.float32, device=dev)
        n_table = keys_src.shape[0] if hist_ids is not None else 0
        # softmax is shift-invariant (DIN.py:108): b2 never changes alpha or the
        # pooled output, so it is not sent (reading it would need a host sync).
        t0 = KernelTimer.mark("fwd")
        _lib.check(_lib.load().nrk_din_attn_fwd(
            _lib.ptr(keys_src), _lib.ptr(hist_ids), n_table, dtype, _lib.ptr(U), _lib.ptr(W1k_k), _lib.ptr(w2), 0.0,
            B, L, Dk, A, _lib.ptr(pooled), _lib.ptr(alpha), _lib.stream(dev)), "din_attn_fwd")
        KernelTimer.push("fwd", t0)
        ctx.save_for_backward(query, W1, U, W1k_k, w2, alpha, keys_src, hist_ids)
        ctx.meta = (B, L, d, Dk, A, dtype, n_table)
        return pooled if Dk == d else pooled[:, :d]

    @staticmethod
    def backward(ctx, dpooled):
        query, W1, U, W1k_k, w2, alpha, keys_src, hist_ids = ctx.saved_tensors
        B, L, d, Dk, A, dtype, n_table = ctx.meta
        dev = query.device
        dpooled = _pad_last(dpooled.float(), Dk).contiguous()
        dU = torch.empty((B, A), dtype=torch.float32, device=dev)
        dW1k = torch.empty((A, Dk), dtype=torch.float32, device=dev)
        dw2 = torch.empty((A,), dtype=torch.float32, device=dev)
        db2 = torch.empty((1,), dtype=torch.float32, device=dev)
        L_ = _lib.load()
        sz = _lib.c_size(0)
        _lib.check(L_.nrk_din_attn_bwd_workspace(B, Dk, A, sz), "din_attn_bwd_workspace")
        ws = torch.empty(max(sz.value // 4, 1), dtype=torch.float32, device=dev)
        t0 = KernelTimer.mark("bwd")
        _lib.check(L_.nrk_din_attn_bwd(
            _lib.ptr(keys_src), _lib.ptr(hist_ids), n_table, dtype, _lib.ptr(U), _lib.ptr(W1k_k), _lib.ptr(w2), 0.0,
            B, L, Dk, A, _lib.ptr(dpooled), _lib.ptr(alpha), _lib.ptr(dU), _lib.ptr(dW1k), _lib.ptr(dw2), _lib.ptr(db2),
            _lib.ptr(ws), ws.numel() * 4, _lib.stream(dev)), "din_attn_bwd")
        KernelTimer.push("bwd", t0)
        dW1 = torch.cat([dU.t() @ query, dW1k[:, :d]], dim=1)
        db1 = dU.sum(dim=0)
        dquery = dU @ W1[:, :d] if ctx.needs_input_grad[0] else None
        return dquery, dW1, db1, dw2.view(1, A), db2, None, None, None


class AttentionLayer(nn.Module):
    """DIN.py:94-111.  attn = Sequential(Linear(2d, A), ReLU, Linear(A, 1))."""

    def __init__(self, emb_dim, attn_units):
        super().__init__()
        self.attn = nn.Sequential(
            nn.Linear(emb_dim * 2, attn_units),
            nn.ReLU(),
            nn.Linear(attn_units, 1),
        )

    def _params(self):
        return self.attn[0].weight, self.attn[0].bias, self.attn[2].weight, self.attn[2].bias

    def forward(self, query, keys):  # (b, d), (b, L, d) -> (b, d)
        b, L, d = keys.shape
        W1, b1, W2, b2 = self._params()
        return _LauPool.apply(query.float(), W1, b1, W2, b2, keys, None, L)

    def forward_ids(self, query, table, hist_ids):
        """query (b, d) f32; table (N, d) f32/bf16 on device; hist_ids (b, L) int32 (-1 = zero row)."""
        if hist_ids.dtype != torch.int32:
            hist_ids = hist_ids.to(torch.int32)
        W1, b1, W2, b2 = self._params()
        return _LauPool.apply(query.float(), W1, b1, W2, b2, table, hist_ids.contiguous(), hist_ids.shape[1])


def gather_rows(table: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """table[ids] as f32 (ids < 0 -> zero rows) through nrk_gather_rows."""
    dev = _lib.require_device(table, ids, what="gather_rows")
    ids = ids.to(torch.int32).contiguous()
    n = ids.numel()
    d = table.shape[1]
    out = torch.empty((n, d), dtype=torch.float32, device=dev)
    _lib.check(_lib.load().nrk_gather_rows(_lib.ptr(table.contiguous()), table.shape[0], _dtype_code(table),
                                           _lib.ptr(ids), n, d, _lib.ptr(out), _lib.stream(dev)), "gather_rows")
    return out.view(*ids.shape, d)


class DIN(nn.Module):
    """DIN.py:113-137 — same submodules, init and state_dict keys."""

    def __init__(self, emb_dim, attn_units, fc_units, dropout_rate):
        super().__init__()
        self.attn = AttentionLayer(emb_dim, attn_units)
        self.fc = nn.Sequential(
            nn.BatchNorm1d(emb_dim * 2),
            nn.Linear(emb_dim * 2, fc_units), nn.ReLU(), nn.Dropout(dropout_rate), nn.BatchNorm1d(fc_units),
            nn.Linear(fc_units, fc_units // 2), nn.ReLU(), nn.Dropout(dropout_rate), nn.BatchNorm1d(fc_units // 2),
            nn.Linear(fc_units // 2, 1),
        )
        self.sigmoid = nn.Sigmoid()
        for m in self.modules():  # same init order as DIN.py:124-128 -> same params under one seed
            if isinstance(m, nn.Linear):
                nn.init.xavier_normal_(m.weight)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    def forward(self, query, history):
        weighted = self.attn(query, history)
        return self.fc(torch.cat([query.float(), weighted], dim=1))

    def predict(self, target, history):
        return self.sigmoid(self(target, history))

    def forward_ids(self, table, target_ids, hist_ids):
        query = gather_rows(table, target_ids)
        weighted = self.attn.forward_ids(query, table, hist_ids)
        return self.fc(torch.cat([query, weighted], dim=1))


# ----------------------------------------------------------------- loops --
def _batch_logits(model, batch, device):
    if "history_ids" in batch:  # id form: batch carries ids, the model's table lives on the device
        table = batch["table"]
        return model.forward_ids(table, batch["target_ids"].to(device, non_blocking=True),
                                 batch["history_ids"].to(device, non_blocking=True))
    return model(batch["target_emb"].to(device, non_blocking=True), batch["history_emb"].to(device, non_blocking=True))


def train(model, loader, optimizer, criterion, device, clip=1.0):
    """DIN.py:139-153: one epoch of BCE + clip_grad_norm_(clip) + optimizer
    step; returns the mean of the per-batch losses.  The losses are summed on
    the device and read back once (the reference syncs every step, DIN.py:152)."""
    model.train()
    total = torch.zeros((), dtype=torch.float64, device=device)
    n = 0
    for batch in loader:
        label = batch["label"].to(device, non_blocking=True)
        optimizer.zero_grad()
        loss = criterion(_batch_logits(model, batch, device), label)
        loss.backward()
        nn.utils.clip_grad_norm_(model.parameters(), clip)
        optimizer.step()
        total += loss.detach()
        n += 1
    return (total / max(n, 1)).item()


def ndcg_from_logits(logits: torch.Tensor, labels: torch.Tensor, seg: torch.Tensor, nseg: int, k: int):
    """Per-segment NDCG@k with one relevant item (DIN.py:181-189), on device.
    Rank of the positive = 1 + #{p_j > p_pos} + #{j before pos with p_j == p_pos}
    (a stable descending order; the reference's np.argsort is unstable on exact
    ties, which this cannot reproduce)."""
    probs = torch.sigmoid(logits)
    dev = logits.device
    pos_mask = labels > 0.5
    idx = torch.arange(logits.numel(), device=dev)
    # position of the first positive per segment (reference labels one-hot at the first match)
    big = torch.full((nseg,), logits.numel(), dtype=torch.long, device=dev)
    first_pos = big.scatter_reduce(0, seg[pos_mask], idx[pos_mask], reduce="amin", include_self=True)
    has_pos = first_pos < logits.numel()
    fp = first_pos.clamp(max=logits.numel() - 1)
    p_pos = probs[fp][seg]
    before = (probs > p_pos) | ((probs == p_pos) & (idx < fp[seg]))
    rank = torch.zeros(nseg, dtype=torch.long, device=dev).index_add_(0, seg, before.long()) + 1
    nd = torch.where(has_pos & (rank <= k), 1.0 / torch.log2(rank.double() + 1.0), torch.zeros_like(rank,
                                                                                                   dtype=torch.double))
    return nd


def evaluate(model, loader, criterion, device, k):
    """DIN.py:155-193: per-user BCE and NDCG@k over ragged candidate lists.
    All users of a batch are scored in ONE forward (BN in eval mode is row-
    independent, so this equals the reference's per-user loop); per-user
    loss/NDCG are segment reductions on the device, read back once."""
    model.eval()
    loss_sum = torch.zeros((), dtype=torch.float64, device=device)
    ndcg_sum = torch.zeros((), dtype=torch.float64, device=device)
    users = 0
    with torch.no_grad():
        for batch in loader:
            hist = batch["history_emb"].to(device, non_blocking=True).float()
            cands = batch["cand_embs"]
            labs = batch["labels"]
            nu, L, d = hist.shape
            counts = torch.tensor([c.shape[0] for c in cands], device=device)
            seg = torch.repeat_interleave(torch.arange(nu, device=device), counts)
            cand = torch.cat([c.to(device, non_blocking=True).float() for c in cands], 0)
            lab = torch.cat([x.to(device, non_blocking=True).float() for x in labs], 0)
            # candidate row i attends over its user's history: address the
            # (nu*L, d) history as a table with per-row ids seg*L + j
            hid = (seg[:, None] * L + torch.arange(L, device=device)[None, :]).to(torch.int32)
            logits = model.fc(torch.cat([cand, model.attn.forward_ids(cand, hist.reshape(nu * L, d), hid)], 1)).view(-1)
            per = nn.functional.binary_cross_entropy_with_logits(logits, lab, reduction="none")
            seg_loss = torch.zeros(nu, dtype=torch.float64, device=device).index_add_(0, seg, per.double())
            loss_sum += (seg_loss / counts.double()).sum()
            ndcg_sum += ndcg_from_logits(logits, lab, seg, nu, k).sum()
            users += nu
    return (loss_sum / users).item(), (ndcg_sum / users).item()


class GraphedTrainStep:
    """One DIN training step (DIN.py:143-151: forward, BCE, backward,
    clip_grad_norm_, optimizer step) captured once into a HIP graph and
    replayed per batch.  Id form only: the embedding table stays resident on
    the device and each replay gathers its batch rows by index inside the
    graph, so a step costs one small index copy plus one graph launch.

    optimizer must be created with capturable=True (Adam/AdamW)."""

    def __init__(self, model, optimizer, criterion, table, hist_ids, target_ids, labels, batch_size, clip=1.0,
                 warmup=3):
        self.model, self.opt, self.crit = model, optimizer, criterion
        self.table, self.hist_all, self.tgt_all, self.lab_all = table, hist_ids, target_ids, labels
        self.B, self.clip = batch_size, clip
        dev = table.device
        self.idx = torch.zeros(batch_size, dtype=torch.long, device=dev)
        model.train()
        # warm-up and capture execute real steps: snapshot the model so that
        # they leave no trace (parameters, BN statistics, optimizer moments)
        snap = {k: v.detach().clone() for k, v in model.state_dict().items()}
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # warm-up on a side stream (allocator, lazy optimizer state)
            for _ in range(max(warmup, 1)):
                self._body()
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        self.opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(self.graph):
            self.loss = self._body()
        with torch.no_grad():
            for k, v in model.state_dict().items():
                v.copy_(snap[k])
            for st in self.opt.state.values():  # Adam(capturable): moments and step restart at 0
                for v in st.values():
                    if torch.is_tensor(v):
                        v.zero_()
            for p in model.parameters():
                if p.grad is not None:
                    p.grad.zero_()

    def _body(self):
        h = self.hist_all.index_select(0, self.idx)
        t = self.tgt_all.index_select(0, self.idx)
        y = self.lab_all.index_select(0, self.idx)
        loss = self.crit(self.model.forward_ids(self.table, t, h), y)
        loss.backward()
        nn.utils.clip_grad_norm_(self.model.parameters(), self.clip)
        self.opt.step()
        self.opt.zero_grad(set_to_none=False)
        return loss

    def step(self, batch_index: torch.Tensor):
        """Run one step on rows `batch_index` (device int64, length batch_size); returns the device loss."""
        self.idx.copy_(batch_index, non_blocking=True)
        self.graph.replay()
        return self.loss


class _HeadParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "bn0_w", "bn0_b", "fc1_w", "fc1_b", "bn1_w", "bn1_b", "fc2_w", "fc2_b", "bn2_w", "bn2_b", "fc3_w", "fc3_b",
        "bn0_rm", "bn0_rv", "bn1_rm", "bn1_rv", "bn2_rm", "bn2_rv", "bn0_nb", "bn1_nb", "bn2_nb",
        "g_bn0_w", "g_bn0_b", "g_fc1_w", "g_fc1_b", "g_bn1_w", "g_bn1_b", "g_fc2_w", "g_fc2_b", "g_bn2_w", "g_bn2_b",
        "g_fc3_w", "g_fc3_b")]


class FusedAdam(torch.optim.Optimizer):
    """The optimizer facade of a FusedTrainStep: torch.optim.Adam's
    hyper-parameters in one param group, so torch's LR schedulers
    (ReduceLROnPlateau, DIN.py:246,254) can read and set `lr`.  The update
    itself runs inside the fused step (nrk_clip_adam reads the rate from a
    device scalar the step refreshes whenever the group's lr changed), so a
    captured HIP graph follows the schedule without re-capture."""

    def __init__(self, params, lr, betas, eps, weight_decay):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    def step(self, closure=None):  # noqa: D401
        raise RuntimeError("FusedAdam is stepped by FusedTrainStep.step(); call that instead")


class FusedTrainStep:
    """One DIN training step (DIN.py:143-151) as ~25 launches in one HIP graph:
    gather + attention forward (libnrk), the whole train-mode MLP head forward
    and backward (nrk_din_head_train: 8 kernels instead of ~150 torch ops),
    attention backward (libnrk), and clip_grad_norm_ + Adam over ONE flat
    parameter buffer (nrk_clip_adam).  The model's parameters and gradients
    become views into flat buffers (state_dict keys and values unchanged).

    Same semantics as `train()` with torch.optim.Adam(lr, betas, eps,
    weight_decay) and clip_grad_norm_(clip): train-mode BatchNorm statistics,
    BCEWithLogits mean loss.  Dropout masks come from a counter-based hash of
    (seed, step, layer, row, col) instead of torch's Philox stream, so with
    dropout > 0 the masks differ from torch's (identical distribution)."""

    def __init__(self, model: "DIN", table, hist_ids, target_ids, labels, batch_size, lr=1.62e-3,
                 betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, clip=1.0, seed=1234, graph=True,
                 grad_hook=None, steps_per_graph=1):
        dev = table.device
        _lib.require_device(table, hist_ids, target_ids, labels, what="FusedTrainStep")
        self.model, self.table = model, table
        # the kernels read int32 ids and f32 labels: normalise whatever the caller passes
        # (torch's default int64 ids, (n, 1) or float64 labels)
        if hist_ids.dim() != 2:
            raise ValueError(f"FusedTrainStep: hist_ids must be (rows, L), got {tuple(hist_ids.shape)}")
        self.hist_all = hist_ids.to(torch.int32).contiguous()
        self.tgt_all = target_ids.reshape(-1).to(torch.int32).contiguous()
        self.lab_all = labels.reshape(-1).to(torch.float32).contiguous()
        if not (self.tgt_all.numel() == self.lab_all.numel() == self.hist_all.shape[0]):
            raise ValueError("FusedTrainStep: hist_ids, target_ids and labels must have one entry per row")
        self.B = int(batch_size)
        if self.B % 32:
            raise ValueError("FusedTrainStep: batch_size must be a multiple of 32")
        self.betas, self.eps, self.wd, self.clip, self.seed = betas, eps, weight_decay, clip, seed
        bns = (model.fc[0], model.fc[4], model.fc[8])
        mom = {bn.momentum for bn in bns}
        bn_eps = {bn.eps for bn in bns}
        if len(mom) != 1 or len(bn_eps) != 1 or None in mom or not all(bn.track_running_stats for bn in bns):
            raise ValueError("FusedTrainStep: the fused head needs one BatchNorm momentum (not None) and eps "
                             "shared by fc.0/fc.4/fc.8, with running statistics")
        self.bn_momentum, self.bn_eps = float(mom.pop()), float(bn_eps.pop())
        self.grad_hook = grad_hook  # e.g. data-parallel all_reduce of the flat gradient buffer
        attn0, attn2 = model.attn.attn[0], model.attn.attn[2]
        self.d = attn0.weight.shape[1] // 2
        self.A = attn0.weight.shape[0]
        self.F = model.fc[1].weight.shape[0]
        self.p_drop = float(model.fc[3].p)
        self.Dk = _kernel_dim(self.d)
        # flat parameter / gradient / moment buffers; parameters become views
        params = list(model.parameters())
        n = sum(p.numel() for p in params)
        self.P = torch.empty(n, dtype=torch.float32, device=dev)
        self.G = torch.zeros(n, dtype=torch.float32, device=dev)
        self.M = torch.zeros(n, dtype=torch.float32, device=dev)
        self.V = torch.zeros(n, dtype=torch.float32, device=dev)
        self.step_t = torch.zeros(1, dtype=torch.float32, device=dev)
        o = 0
        with torch.no_grad():
            for p in params:
                k = p.numel()
                self.P[o:o + k].copy_(p.reshape(-1))
                p.data = self.P[o:o + k].view_as(p)
                p.grad = self.G[o:o + k].view_as(p)
                o += k
        self.optimizer = FusedAdam(params, lr, betas, eps, weight_decay)
        self.lr_t = torch.full((1,), float(lr), dtype=torch.float32, device=dev)  # read by nrk_clip_adam
        self._lr_host = float(lr)
        fc = model.fc
        self.hp = _HeadParams(*[_lib.ptr(t) for t in (
            fc[0].weight, fc[0].bias, fc[1].weight, fc[1].bias, fc[4].weight, fc[4].bias, fc[5].weight, fc[5].bias,
            fc[8].weight, fc[8].bias, fc[9].weight, fc[9].bias,
            fc[0].running_mean, fc[0].running_var, fc[4].running_mean, fc[4].running_var, fc[8].running_mean,
            fc[8].running_var, fc[0].num_batches_tracked, fc[4].num_batches_tracked, fc[8].num_batches_tracked,
            fc[0].weight.grad, fc[0].bias.grad, fc[1].weight.grad, fc[1].bias.grad, fc[4].weight.grad,
            fc[4].bias.grad, fc[5].weight.grad, fc[5].bias.grad, fc[8].weight.grad, fc[8].bias.grad,
            fc[9].weight.grad, fc[9].bias.grad)])
        B, d, A, Dk = self.B, self.d, self.A, self.Dk
        L_ = _lib.load()
        # batch rows and losses of the K steps one graph replays (step(): K = 1 slot)
        self.K = max(1, int(steps_per_graph))
        self.idx_ring = torch.zeros((self.K, B), dtype=torch.long, device=dev)
        self.loss_ring = torch.zeros((self.K, 1), dtype=torch.float32, device=dev)
        self.idx, self.loss = self.idx_ring[0], self.loss_ring[0]
        self.pooled = torch.empty((B, Dk), dtype=torch.float32, device=dev)
        self.alpha = torch.empty((B, hist_ids.shape[1]), dtype=torch.float32, device=dev)
        self.logits = torch.empty(B, dtype=torch.float32, device=dev)
        self.dpooled = torch.empty((B, Dk), dtype=torch.float32, device=dev)
        self.dU = torch.empty((B, A), dtype=torch.float32, device=dev)
        self.dW1k = torch.empty((A, Dk), dtype=torch.float32, device=dev)
        sz = _lib.c_size(0)
        _lib.check(L_.nrk_din_head_workspace(B, d, self.F, sz), "din_head_workspace")
        self.ws_head = torch.empty(max(sz.value, 1), dtype=torch.uint8, device=dev)
        _lib.check(L_.nrk_din_attn_bwd_workspace(B, Dk, A, sz), "din_attn_bwd_workspace")
        self.ws_attn = torch.empty(max(sz.value, 1), dtype=torch.uint8, device=dev)
        _lib.check(L_.nrk_clip_adam_workspace(n, sz), "clip_adam_workspace")
        self.ws_opt = torch.zeros(max(sz.value, 1), dtype=torch.uint8, device=dev)  # holds a ticket: zeroed once
        self.n = n
        # fast path (bf16 table, emb_dim 64/128/256): one batch-assembly kernel
        # (rows -> ids, labels, f32 query, U = q W1q^T + b1, bf16 W1k) and an
        # attention backward that also forms dW1q / db1 and writes every
        # attention gradient in place: no torch ops left inside the step
        Lh = hist_ids.shape[1]
        max_l = 128  # d = 256, L > 64: the column-split backward in two half-samples per sample
        why = [w for w, bad in (("table is not bf16", table.dtype != torch.bfloat16),
                                (f"emb_dim {d} not in (64, 128, 256)", d not in (64, 128, 256)),
                                (f"history length {Lh} > {max_l}", Lh > max_l)) if bad]
        self.fast = not why
        # which path the step runs (the generic one has torch ops around the kernels)
        self.path = "fast" if self.fast else "generic: " + ", ".join(why)
        if not self.fast:
            warnings.warn(f"FusedTrainStep: {self.path} -> the generic step (torch GEMMs and gathers around the "
                          f"attention kernels), not the single-kernel-chain fast path", stacklevel=2)
        # fast path, d 64/128, L <= 64 (8-wave backward): the attention backward
        # forms dpooled from the head's state itself (nrk_din_attn_bwd_params_head;
        # one launch and the dpooled round trip fewer).  NRK_DIN_FUSE_DP=0: A/B hook.
        Lk = 32 if Lh <= 32 else 64
        self.fuse_dp = (self.fast and d in (64, 128) and Lh <= 64 and Lk * d >= 4096 and self.F == 32
                        and os.environ.get("NRK_DIN_FUSE_DP", "1") != "0")
        # fast path without a grad_hook: the gradient reduction also writes the
        # squared-norm partials clip_grad_norm_ reads (nrk_clip_adam_partials)
        self.norm_part = (torch.zeros(-(-n // 64), dtype=torch.float64, device=dev)
                          if self.fast and grad_hook is None else None)
        # gathers ahead (fast path): one nrk_din_batch launch assembles the rows of
        # all K steps of a graph (history ids, query rows, labels: nothing there
        # depends on the parameters); each step then only forms U and bf16 W1k
        # (nrk_din_batch_u).
        if self.fast:
            L = hist_ids.shape[1]
            self.hist_k = torch.empty((self.K, B, L), dtype=torch.int32, device=dev)
            self.q_k = torch.empty((self.K, B, d), dtype=torch.float32, device=dev)
            self.y_k = torch.empty((self.K, B), dtype=torch.float32, device=dev)
            self.hist_b, self.q_b, self.y_b = self.hist_k[0], self.q_k[0], self.y_k[0]
            self.U_b = torch.empty((B, A), dtype=torch.float32, device=dev)
            self.W1k_b = torch.empty((A, d), dtype=torch.bfloat16, device=dev)
        self.graph = self.graph_k = None
        if graph:
            snap = [t.detach().clone() for t in (self.P, self.M, self.V, self.step_t)]
            bufs = {k: v.detach().clone() for k, v in model.named_buffers()}
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                self._body()
            torch.cuda.current_stream(dev).wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self._body()
            if self.K > 1:  # K consecutive steps in one graph: one index copy and one launch per K steps
                self.graph_k = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph_k):
                    for k in range(self.K):
                        self._body(k, gather_n=self.K if k == 0 else 0)
            with torch.no_grad():  # capture ran real steps: restore the model and optimizer state
                for t, s in zip((self.P, self.M, self.V, self.step_t), snap):
                    t.copy_(s)
                for k, v in model.named_buffers():
                    v.copy_(bufs[k])

    def _body(self, k=0, gather_n=1):
        """Step k of a K-step sequence; gather_n > 0: first assemble the rows of
        steps k .. k + gather_n - 1 (fast path with gathers ahead)."""
        idx, loss = self.idx_ring[k], self.loss_ring[k]
        if self.fast:
            return self._body_fast(k, idx, loss, gather_n)
        L_ = _lib.load()
        m = self.model
        dev = self.table.device
        st = _lib.stream(dev)
        B, d, A, Dk = self.B, self.d, self.A, self.Dk
        hist = self.hist_all.index_select(0, idx)
        tgt = self.tgt_all.index_select(0, idx)
        y = self.lab_all.index_select(0, idx).reshape(-1)
        q = gather_rows(self.table, tgt)
        W1, b1 = m.attn.attn[0].weight, m.attn.attn[0].bias
        w2 = m.attn.attn[2].weight.reshape(-1)
        U = torch.addmm(b1, q, W1[:, :d].t())
        keys = _pad_last(self.table, Dk)
        dtype = _dtype_code(keys)
        W1k = _pad_last(W1[:, d:], Dk)
        W1k = W1k.contiguous() if dtype == _lib.NRK_DTYPE_F32 else W1k.to(torch.bfloat16)
        _lib.check(L_.nrk_din_attn_fwd(
            _lib.ptr(keys), _lib.ptr(hist), keys.shape[0], dtype, _lib.ptr(U), _lib.ptr(W1k), _lib.ptr(w2), 0.0, B,
            hist.shape[1], Dk, A, _lib.ptr(self.pooled), _lib.ptr(self.alpha), st), "din_attn_fwd")
        _lib.check(L_.nrk_din_head_train(
            _lib.ptr(q), _lib.ptr(self.pooled), Dk, _lib.ptr(y), B, d, self.F, self.bn_momentum, self.bn_eps, self.p_drop,
            self.seed,
            _lib.ptr(self.step_t), ctypes.byref(self.hp), _lib.ptr(self.logits), _lib.ptr(loss),
            _lib.ptr(self.dpooled), _lib.ptr(self.ws_head), self.ws_head.numel(), st), "din_head_train")
        gW2, gb2 = m.attn.attn[2].weight.grad, m.attn.attn[2].bias.grad
        _lib.check(L_.nrk_din_attn_bwd(
            _lib.ptr(keys), _lib.ptr(hist), keys.shape[0], dtype, _lib.ptr(U), _lib.ptr(W1k), _lib.ptr(w2), 0.0, B,
            hist.shape[1], Dk, A, _lib.ptr(self.dpooled), _lib.ptr(self.alpha), _lib.ptr(self.dU),
            _lib.ptr(self.dW1k), _lib.ptr(gW2), _lib.ptr(gb2), _lib.ptr(self.ws_attn), self.ws_attn.numel(), st),
            "din_attn_bwd")
        gW1, gb1 = W1.grad, b1.grad
        gW1[:, :d].copy_(self.dU.t() @ q)
        gW1[:, d:].copy_(self.dW1k[:, :d])
        torch.sum(self.dU, 0, out=gb1)
        if self.grad_hook is not None:
            self.grad_hook(self.G)
        _lib.check(L_.nrk_clip_adam(
            _lib.ptr(self.P), _lib.ptr(self.G), _lib.ptr(self.M), _lib.ptr(self.V), self.n, _lib.ptr(self.step_t),
            self._lr_host, _lib.ptr(self.lr_t), self.betas[0], self.betas[1], self.eps, self.wd, self.clip,
            _lib.ptr(self.ws_opt),
            self.ws_opt.numel(), st), "clip_adam")

    def _body_fast(self, k, idx, loss, gather_n):
        L_ = _lib.load()
        m = self.model
        st = _lib.stream(self.table.device)
        B, d, A = self.B, self.d, self.A
        L = self.hist_all.shape[1]
        N = self.table.shape[0]
        dt = _lib.NRK_DTYPE_BF16
        W1, b1 = m.attn.attn[0].weight, m.attn.attn[0].bias
        w2 = m.attn.attn[2].weight
        self.hist_b, self.q_b, self.y_b = self.hist_k[k], self.q_k[k], self.y_k[k]
        if gather_n > 0:
            _lib.check(L_.nrk_din_batch(
                _lib.ptr(self.idx_ring[k]), gather_n * B, _lib.ptr(self.hist_all), _lib.ptr(self.tgt_all),
                _lib.ptr(self.lab_all), self.hist_all.shape[0], L, _lib.ptr(self.table), N, dt, d, None, None, A,
                _lib.ptr(self.hist_b), _lib.ptr(self.q_b), _lib.ptr(self.y_b), None, None, st), "din_batch")
        _lib.check(L_.nrk_din_batch_u(_lib.ptr(self.q_b), B, d, _lib.ptr(W1), _lib.ptr(b1), A, _lib.ptr(self.U_b),
                                      _lib.ptr(self.W1k_b), st), "din_batch_u")
        t0 = KernelTimer.mark("fwd")
        _lib.check(L_.nrk_din_attn_fwd(
            _lib.ptr(self.table), _lib.ptr(self.hist_b), N, dt, _lib.ptr(self.U_b), _lib.ptr(self.W1k_b), _lib.ptr(w2),
            0.0, B, L, d, A, _lib.ptr(self.pooled), _lib.ptr(self.alpha), st), "din_attn_fwd")
        KernelTimer.push("fwd", t0)
        _lib.check(L_.nrk_din_head_train(
            _lib.ptr(self.q_b), _lib.ptr(self.pooled), d, _lib.ptr(self.y_b), B, d, self.F, self.bn_momentum,
            self.bn_eps, self.p_drop,
            self.seed, _lib.ptr(self.step_t), ctypes.byref(self.hp), _lib.ptr(self.logits), _lib.ptr(loss),
            None if self.fuse_dp else _lib.ptr(self.dpooled), _lib.ptr(self.ws_head), self.ws_head.numel(), st),
            "din_head_train")
        t0 = KernelTimer.mark("bwd")
        if self.fuse_dp:
            _lib.check(L_.nrk_din_attn_bwd_params_head(
                _lib.ptr(self.table), _lib.ptr(self.hist_b), N, dt, _lib.ptr(self.q_b), _lib.ptr(self.U_b),
                _lib.ptr(self.W1k_b), _lib.ptr(w2), B, L, d, A, _lib.ptr(self.pooled), _lib.ptr(self.alpha), self.F,
                ctypes.byref(self.hp), _lib.ptr(self.ws_head), self.ws_head.numel(), _lib.ptr(W1.grad),
                _lib.ptr(b1.grad), _lib.ptr(w2.grad), _lib.ptr(m.attn.attn[2].bias.grad), self.n,
                _lib.ptr(self.norm_part), _lib.ptr(self.ws_attn), self.ws_attn.numel(), st),
                "din_attn_bwd_params_head")
        else:
            _lib.check(L_.nrk_din_attn_bwd_params(
                _lib.ptr(self.table), _lib.ptr(self.hist_b), N, dt, _lib.ptr(self.q_b), _lib.ptr(self.U_b),
                _lib.ptr(self.W1k_b), _lib.ptr(w2), B, L, d, A, _lib.ptr(self.dpooled), _lib.ptr(self.alpha),
                _lib.ptr(self.pooled), _lib.ptr(W1.grad), _lib.ptr(b1.grad), _lib.ptr(w2.grad),
                _lib.ptr(m.attn.attn[2].bias.grad), None, self.n, _lib.ptr(self.norm_part), _lib.ptr(self.ws_attn),
                self.ws_attn.numel(), st), "din_attn_bwd_params")
        KernelTimer.push("bwd", t0)
        if self.grad_hook is not None:
            self.grad_hook(self.G)
        if self.norm_part is not None:
            _lib.check(L_.nrk_clip_adam_partials(
                _lib.ptr(self.P), _lib.ptr(self.G), _lib.ptr(self.M), _lib.ptr(self.V), self.n, _lib.ptr(self.step_t),
                self._lr_host, _lib.ptr(self.lr_t), self.betas[0], self.betas[1], self.eps, self.wd, self.clip,
                _lib.ptr(self.norm_part), self.norm_part.numel(), _lib.ptr(self.ws_opt), self.ws_opt.numel(), st),
                "clip_adam_partials")
            return
        _lib.check(L_.nrk_clip_adam(
            _lib.ptr(self.P), _lib.ptr(self.G), _lib.ptr(self.M), _lib.ptr(self.V), self.n, _lib.ptr(self.step_t),
            self._lr_host, _lib.ptr(self.lr_t), self.betas[0], self.betas[1], self.eps, self.wd, self.clip,
            _lib.ptr(self.ws_opt),
            self.ws_opt.numel(), st), "clip_adam")

    @property
    def lr(self) -> float:
        return float(self.optimizer.param_groups[0]["lr"])

    @lr.setter
    def lr(self, v: float):
        self.optimizer.param_groups[0]["lr"] = float(v)

    def _sync_lr(self):
        lr = self.lr
        if lr != self._lr_host:  # a scheduler changed the group's lr: refresh the device scalar
            self.lr_t.fill_(lr)
            self._lr_host = lr

    def step(self, batch_index: torch.Tensor):
        """One training step on rows `batch_index` (device int64, length B); returns the device loss."""
        self._sync_lr()
        self.idx.copy_(batch_index, non_blocking=True)
        if self.graph is not None:
            self.graph.replay()
        else:
            self._body()
        return self.loss

    def step_rows(self, batch_index: torch.Tensor):
        """One training step on ANY number of rows (> 1; the fused kernels need
        the fixed batch): fit()'s last partial batch, which the reference's
        DataLoader(shuffle=True) keeps (DIN.py:241).  Forward and backward run
        through the model's autograd path (the HIP attention kernels, a torch
        head), the gradients land in the step's flat buffer, then the same
        grad_hook and clip_grad_norm_ + Adam kernel as step() (shared moments,
        step count and lr).  Returns the device loss (1,).  With dropout > 0 the
        masks come from torch's generator, not the fused head's hash."""
        n = int(batch_index.numel())
        if n == self.B:
            return self.step(batch_index)
        self._sync_lr()
        m = self.model
        m.train()
        idx = batch_index.reshape(-1).to(torch.long)
        params = list(m.parameters())
        with torch.enable_grad():
            logits = m.forward_ids(self.table, self.tgt_all[idx], self.hist_all[idx])
            loss = nn.functional.binary_cross_entropy_with_logits(logits.reshape(-1), self.lab_all[idx])
            grads = torch.autograd.grad(loss, params)
        with torch.no_grad():
            for p, g in zip(params, grads):
                p.grad.copy_(g)
        if self.grad_hook is not None:
            self.grad_hook(self.G)
        L_ = _lib.load()
        _lib.check(L_.nrk_clip_adam(
            _lib.ptr(self.P), _lib.ptr(self.G), _lib.ptr(self.M), _lib.ptr(self.V), self.n, _lib.ptr(self.step_t),
            self._lr_host, _lib.ptr(self.lr_t), self.betas[0], self.betas[1], self.eps, self.wd, self.clip,
            _lib.ptr(self.ws_opt), self.ws_opt.numel(), _lib.stream(self.table.device)), "clip_adam")
        return loss.detach().reshape(1)

    def step_many(self, batch_indices: torch.Tensor):
        """K = steps_per_graph consecutive training steps, batch k on rows
        `batch_indices[k]` ((K, B) device int64), as ONE graph launch; returns
        the K device losses (K, 1).  Same result as K calls of step()."""
        if batch_indices.shape != (self.K, self.B):
            raise ValueError(f"step_many: expected batch indices of shape {(self.K, self.B)}, "
                             f"got {tuple(batch_indices.shape)}")
        self._sync_lr()
        self.idx_ring.copy_(batch_indices, non_blocking=True)
        if self.graph_k is not None:
            self.graph_k.replay()
        elif self.graph is not None and self.K == 1:
            self.graph.replay()
        else:
            for k in range(self.K):
                self._body(k, gather_n=self.K if k == 0 else 0)
        return self.loss_ring


def fit(model, table, hist_ids, target_ids, labels, eval_loader, epochs=10, batch_size=64, lr=1.62e-3,
        weight_decay=8.96e-5, clip=1.0, k=5, checkpoint=None, scheduler=None, seed=42, graph=True, log=None):
    """DIN.py:225-257 (main()) on the fused train step: per epoch, shuffle the
    rows (DataLoader(shuffle=True) -> torch.randperm from a generator seeded
    with `seed`), train on every full batch with the fused step and on the last
    partial batch of n % batch_size rows with FusedTrainStep.step_rows (as the
    reference's DataLoader keeps it), report the mean of the per-batch losses
    (DIN.py:153), evaluate
    (DIN.py:155-193), step the scheduler — by default
    ReduceLROnPlateau(mode='min', factor=0.5, patience=1) on the validation
    loss (DIN.py:246,254), any other LR scheduler with step() — and save the
    state_dict whenever NDCG@k beats the best so far (DIN.py:255-257).
    Returns one dict per epoch (train_loss, val_loss, ndcg, lr)."""
    dev = table.device
    trainer = FusedTrainStep(model, table, hist_ids, target_ids, labels, batch_size, lr=lr,
                             weight_decay=weight_decay, clip=clip, graph=graph)
    opt = trainer.optimizer
    plateau = scheduler is None
    sched = (torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.5, patience=1) if plateau
             else scheduler(opt))
    crit = nn.BCEWithLogitsLoss()
    gen = torch.Generator(device=dev).manual_seed(seed)
    n, B = trainer.hist_all.shape[0], trainer.B
    nb, tail = divmod(n, B)
    best, history = 0.0, []
    for epoch in range(epochs):
        lr_epoch = trainer.lr
        model.train()
        perm = torch.randperm(n, generator=gen, device=dev)
        total = torch.zeros((), dtype=torch.float64, device=dev)
        for b in range(nb):
            total += trainer.step(perm[b * B:(b + 1) * B])[0]
        if tail:
            total += trainer.step_rows(perm[nb * B:])[0]
        train_loss = (total / max(nb + (1 if tail else 0), 1)).item()
        val_loss, ndcg = evaluate(model, eval_loader, crit, dev, k)
        if plateau:
            sched.step(val_loss)
        else:
            opt._opt_called = True  # the fused step is the optimizer step (silences torch's order check)
            sched.step()
        history.append({"epoch": epoch + 1, "train_loss": train_loss, "val_loss": val_loss, "ndcg": ndcg,
                        "lr": lr_epoch})
        if log is not None:
            log(f"Epoch {epoch + 1}: Train {train_loss}, Validate {val_loss}, NDCG {ndcg}")
        if ndcg > best:
            best = ndcg
            if checkpoint is not None:
                torch.save({k_: v.detach().clone() for k_, v in model.state_dict().items()}, checkpoint)
    return history
