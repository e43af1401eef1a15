"""Per-call latency of the reference's per-user loop (Retrieval.py:28-34:
centroid_index.search(profile, 1) for one profile at a time) through the
drop-in faiss module: numpy in, numpy out, 300 centroids x 256."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from newsrecommend_amd import faiss as nf

rng = np.random.default_rng(0)
cent = rng.standard_normal((300, 256)).astype(np.float32)
prof = rng.standard_normal((2000, 256)).astype(np.float32)
idx = nf.IndexFlatL2(256)
idx.add(cent)
for i in range(50):
    idx.search(prof[i:i + 1], 1)
torch.cuda.synchronize()
t = time.perf_counter()
for i in range(2000):
    _, I = idx.search(prof[i:i + 1], 1)
dt = (time.perf_counter() - t) / 2000
print(f"single-query search (300 x 256, k = 1): {dt * 1e6:.1f} us per call")
idx.search(prof, 1)  # grows the pinned staging once
t = time.perf_counter()
for _ in range(20):
    _, Ib = idx.search(prof, 1)
print(f"batched 2000 queries: {(time.perf_counter() - t) / 20 * 1e3:.3f} ms per call")
