"""Time the IVF coarse quantizer search (IndexFlatL2 over nlist centroids,
k = nprobe: the small exact path) in isolation, HIP events over R reps.
usage: python tools/quant_step.py [--nlist 300 --nq 4096 --d 128 --k 32 --reps 200]"""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from newsrecommend_amd import faiss as nf
from newsrecommend_amd.data import clustered_corpus

ap = argparse.ArgumentParser()
ap.add_argument("--nlist", type=int, default=300)
ap.add_argument("--nq", type=int, default=4096)
ap.add_argument("--d", type=int, default=128)
ap.add_argument("--k", type=int, default=32)
ap.add_argument("--reps", type=int, default=200)
a = ap.parse_args()
dev = torch.device("cuda", 0)
cent = clustered_corpus(a.nlist, a.d, seed=5, device=dev)
xq = clustered_corpus(a.nq, a.d, seed=4321, device=dev)
q = nf.IndexFlatL2(a.d, device=dev)
q.add(cent)
for _ in range(10):
    q.search_device(xq, a.k)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.reps):
    D, I = q.search_device(xq, a.k)
e1.record()
torch.cuda.synchronize()
print(f"quantizer search {a.nq} x {a.nlist} x {a.d}, k = {a.k}: {e0.elapsed_time(e1) / a.reps * 1e3:.1f} us per search")
