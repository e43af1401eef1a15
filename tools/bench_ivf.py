"""IVF-Flat at the configs[3] shape on one GPU: build time (k-means on the
faiss subsample, assignment, list layout), per-stage search times, fallback
count and recall@k vs the exact flat search.
usage: python tools/bench_ivf.py [--nb 10000000 --d 128 --nlist 300 --nprobe 32 --nq 4096 --k 5]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from newsrecommend_amd import _lib, faiss as nf
from newsrecommend_amd.data import clustered_corpus

ap = argparse.ArgumentParser()
ap.add_argument("--nb", type=int, default=10_000_000)
ap.add_argument("--d", type=int, default=128)
ap.add_argument("--nlist", type=int, default=300)
ap.add_argument("--nprobe", type=int, default=32)
ap.add_argument("--nq", type=int, default=4096)
ap.add_argument("--k", type=int, default=5)
ap.add_argument("--niter", type=int, default=20)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--metric", default="l2")
ap.add_argument("vars", nargs="*")
a = ap.parse_args()
metric = nf.METRIC_L2 if a.metric == "l2" else nf.METRIC_INNER_PRODUCT
dev = torch.device("cuda", 0)
xb = clustered_corpus(a.nb, a.d, seed=1234, device=dev)
xq = clustered_corpus(a.nq, a.d, seed=4321, device=dev)
torch.cuda.synchronize()
t0 = time.perf_counter()
q = nf.IndexFlatL2(a.d)
ivf = nf.IndexIVFFlat(q, a.d, a.nlist, metric)
ivf.cp.niter = a.niter
ivf.train(xb)
torch.cuda.synchronize()
t1 = time.perf_counter()
ivf.add(xb)
torch.cuda.synchronize()
t2 = time.perf_counter()
sizes = torch.diff(ivf.list_off).cpu().numpy()
print(f"train {t1 - t0:.2f}s add {t2 - t1:.2f}s  list sizes min/mean/max {sizes.min()}/{sizes.mean():.0f}/{sizes.max()}",
      flush=True)
ivf.nprobe = a.nprobe
grid = [[(v.split("=")[0], x) for x in v.split("=")[1].split(",")] for v in a.vars] or [[("NONE", "0")]]
import itertools
for combo in itertools.product(*grid):
    for k_, v in combo:
        os.environ[k_] = v
    _, probe = q.search_device(xq, a.nprobe)
    D, I = ivf.search_device(xq, a.k, probe=probe)
    ev = [_lib.StageEvents() for _ in range(a.reps)]
    torch.cuda.synchronize()
    t = time.perf_counter()
    for e in ev:
        D, I = ivf.search_device(xq, a.k, stage_events=e, probe=probe)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / a.reps
    st = np.array([e.elapsed_ms() for e in ev]).mean(0)
    # full search incl. the coarse quantizer
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.reps):
        D, I = ivf.search_device(xq, a.k)
    torch.cuda.synchronize()
    full = (time.perf_counter() - t) / a.reps
    pr = probe.cpu().numpy()
    flops = 2.0 * a.d * float((sizes[pr]).sum())
    cnt_l = np.bincount(pr[pr >= 0].ravel(), minlength=a.nlist)
    # phase B rows per work item: waves x 32 x (2 query tiles per wave, 1 at d > 128)
    wq = 4 * 32 * (2 if a.d <= 128 else 1)
    padded = 2.0 * a.d * float((np.ceil(cnt_l / wq) * wq * sizes).sum())
    # MFMA work issued: waves skip query tiles past a list's last prober (32 rows
    # for the 32x32x16 collect, 16 for the 16x16x32 one)
    iss = {gq: 2.0 * a.d * float((np.ceil(cnt_l / gq) * gq * sizes).sum()) for gq in (16, 32)}
    print(f"{combo}: stages ms group {st[0]:.4f} screen {st[1]:.4f} merge {st[2]:.4f} fallback {st[3]:.4f}  "
          f"ivf wall {wall * 1e3:.3f} ms, full (with coarse) {full * 1e3:.3f} ms = {a.nq / full:,.0f} QPS; "
          f"screen {flops / st[1] / 1e9:.1f} TFLOP/s useful, {padded / st[1] / 1e9:.1f} incl. query-tile padding "
          f"(useful {flops / 1e12:.2f} TF, padded {padded / 1e12:.2f} TF; issued at 32 / 16-query tiles "
          f"{iss[32] / 1e12:.2f} / {iss[16] / 1e12:.2f} TF); fallback={int(ivf.last_fallback.item())}",
          flush=True)
flat = nf.IndexFlat(a.d, metric)
flat.add(xb)
_, If = flat.search_device(xq, a.k)
rec = np.mean([len(set(I[i].tolist()) & set(If[i].tolist())) / a.k for i in range(a.nq)])
print(f"recall@{a.k} vs exact flat = {rec:.4f}")
