"""Time the fused re-rank (nrk_din_rerank) without the retrieval in front of it.

  python tools/rerank_step.py [--users 4096] [--items 10000000] [--reps 10]
      configs[4]'s shape: 4096 users x 201 candidates, d 256, L 50, A 128, F 32,
      over a 10M-row bf16 item table (pipeline.rerank, rectangular lists)
  python tools/rerank_step.py --flow [--users 50000]
      the Retrieval.py flow's geometry: 364,047 items, 300 clusters of skewed
      sizes (mean ~1,210), every user scoring its whole cluster + the appended
      ground truth, L 64 (pipeline.rerank_ragged, shared lists projected once;
      --direct: a bf16 table through the row-staged nrk_din_rerank)
Prints ms per call (wall, synchronised) and the kernel's HIP-event time."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from newsrecommend_amd.data import zipf_ids
from newsrecommend_amd.din import DIN, KernelTimer
from newsrecommend_amd.pipeline import rerank, rerank_ragged

ap = argparse.ArgumentParser()
ap.add_argument("--users", type=int, default=None)
ap.add_argument("--items", type=int, default=None)
ap.add_argument("--cands", type=int, default=201)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--flow", action="store_true")
ap.add_argument("--direct", action="store_true", help="flow: the row-staged kernel (bf16 table, L <= 64)")
ap.add_argument("--A", type=int, default=128)
ap.add_argument("--F", type=int, default=32)
ap.add_argument("--f32", action="store_true", help="an fp32 item table (the projected path)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
d = 256
L = 64 if a.flow else 50
U = a.users or (50_000 if a.flow else 4096)
N = a.items or (364_047 if a.flow else 10_000_000)
g = torch.Generator(device=dev).manual_seed(3)
table = torch.randn((N, d), generator=g, device=dev) * 0.5
if not a.f32:
    table = table.to(torch.bfloat16)
hist = zipf_ids(U * L, N, generator=g, device=dev).view(U, L).to(torch.int32)
lens = torch.randint(1, L + 1, (U,), generator=g, device=dev)
hist = torch.where(torch.arange(L, device=dev)[None] < lens[:, None], hist, torch.full_like(hist, -1))
torch.manual_seed(42)
model = DIN(d, a.A, a.F, 0.36).to(dev).eval()

if a.flow:
    nl = 300
    w = torch.distributions.LogNormal(0.0, 1.0).sample((nl,)).to(dev)
    sizes = (w / w.sum() * N).long().clamp_min(1)
    sizes[-1] = N - sizes[:-1].sum()
    off = torch.zeros(nl + 1, dtype=torch.int64, device=dev)
    off[1:] = torch.cumsum(sizes, 0)
    rows = torch.randperm(N, device=dev).to(torch.int32)
    uc = torch.multinomial(sizes.double(), U, replacement=True, generator=g).sort().values  # users by cluster
    co, cl = off[uc], sizes[uc].to(torch.int32)
    extra = zipf_ids(U, N, generator=g, device=dev)
    width = cl.long() + 1
    oo = torch.cumsum(width, 0) - width
    n_out = int(width.sum())

    def call():
        return rerank_ragged(model, table, hist, rows, co, cl, extra, oo, n_out, direct=a.direct)
    samples = n_out
else:
    cand = torch.randint(0, N, (U, a.cands), generator=g, device=dev, dtype=torch.int32)

    def call():
        return rerank(model, table, hist, cand)
    samples = U * a.cands

out = call()
torch.cuda.synchronize()
t0 = time.perf_counter()
with KernelTimer() as kt:
    for _ in range(a.reps):
        out = call()
    torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / a.reps * 1e3
kms = kt.mean_ms("rerank")
pms = kt.mean_ms("rerank_project")
print(f"rerank {'flow' if a.flow else 'e2e'} {U} users, {samples} samples (A={a.A}, F={a.F}): {ms:.3f} ms/call wall, "
      f"{kms:.3f} ms kernel + {pms:.3f} ms projections (HIP events) = {samples / kms / 1e3:.1f} M samples/s, "
      f"{U / kms * 1e3:.0f} users/s, finite {bool(torch.isfinite(out).any())}", flush=True)
