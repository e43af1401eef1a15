"""Time pipeline.rerank at the configs[4] re-rank shape (4096 users x 201
candidates, d 256, L 50, A 128, F 32) over a 10M-row bf16 item table, without
the retrieval in front of it.  Prints ms per call (wall, synchronised).
usage: python tools/rerank_step.py [--users 4096] [--items 10000000] [--reps 10]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from newsrecommend_amd.data import zipf_ids
from newsrecommend_amd.din import DIN
from newsrecommend_amd.pipeline import rerank

ap = argparse.ArgumentParser()
ap.add_argument("--users", type=int, default=4096)
ap.add_argument("--items", type=int, default=10_000_000)
ap.add_argument("--cands", type=int, default=201)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
dev = torch.device("cuda", 0)
d, L = 256, 50
g = torch.Generator(device=dev).manual_seed(3)
table = (torch.randn((a.items, d), generator=g, device=dev) * 0.5).to(torch.bfloat16)
hist = zipf_ids(a.users * L, a.items, generator=g, device=dev).view(a.users, L).to(torch.int32)
lens = torch.randint(1, L + 1, (a.users,), generator=g, device=dev)
hist = torch.where(torch.arange(L, device=dev)[None] < lens[:, None], hist, torch.full_like(hist, -1))
cand = torch.randint(0, a.items, (a.users, a.cands), generator=g, device=dev, dtype=torch.int32)
torch.manual_seed(42)
model = DIN(d, 128, 32, 0.36).to(dev).eval()
out = rerank(model, table, hist, cand)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.reps):
    out = rerank(model, table, hist, cand)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / a.reps * 1e3
print(f"rerank {a.users} users x {a.cands} candidates: {ms:.3f} ms/call, "
      f"{a.users * a.cands / ms / 1e3:.1f} M samples/s, finite {bool(torch.isfinite(out).all())}", flush=True)
