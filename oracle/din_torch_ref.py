"""oracle/din_torch_ref.py — TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline
leg and tests/; never the product).

The reference's DIN ranker as plain PyTorch-CPU fp32 (DIN.py:94-153), the
"PyTorch-CPU train step" BASELINE.md names as the configs[2] CPU baseline:

  TorchDIN.forward   DIN.py:103-111,130-133: the local activation unit over
                     [q repeated L times ; keys] (the reference's repeat + cat
                     form), ReLU, Linear(A, 1), softmax over all L slots,
                     weighted sum; then the BN/MLP head on [q ; pooled]
  train_step         DIN.py:143-151: BCEWithLogits (mean), backward,
                     clip_grad_norm_(1.0), Adam step

Same state_dict keys as the reference and as newsrecommend_amd.din.DIN, so
the golden fixtures made by the reference load directly
(tests/test_oracle_din.py pins it against them).
"""
from __future__ import annotations

import torch
import torch.nn as nn


class _Attn(nn.Module):
    def __init__(self, d, A):
        super().__init__()
        self.attn = nn.Sequential(nn.Linear(2 * d, A), nn.ReLU(), nn.Linear(A, 1))

    def forward(self, query, keys):
        b, L, d = keys.shape
        z = torch.cat([query.unsqueeze(1).expand(b, L, d), keys], dim=2).reshape(b * L, 2 * d)
        alpha = torch.softmax(self.attn(z).view(b, L), dim=1)
        return torch.bmm(alpha.unsqueeze(1), keys).squeeze(1)


class TorchDIN(nn.Module):
    def __init__(self, d, A, F, dropout):
        super().__init__()
        self.attn = _Attn(d, A)
        self.fc = nn.Sequential(
            nn.BatchNorm1d(2 * d), nn.Linear(2 * d, F), nn.ReLU(), nn.Dropout(dropout), nn.BatchNorm1d(F),
            nn.Linear(F, F // 2), nn.ReLU(), nn.Dropout(dropout), nn.BatchNorm1d(F // 2), nn.Linear(F // 2, 1))

    def forward(self, query, history):
        return self.fc(torch.cat([query, self.attn(query, history)], dim=1))


def train_step(model, opt, crit, query, history, label, clip=1.0):
    opt.zero_grad()
    loss = crit(model(query, history), label)
    loss.backward()
    nn.utils.clip_grad_norm_(model.parameters(), clip)
    opt.step()
    return loss
