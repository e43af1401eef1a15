"""The 8-GPU shard geometries of bench.py's retrieval records, run on ONE GPU
(VERDICT r3 item 6b): each record's world-8 shard (rows [r n/8, (r+1) n/8) of
its corpus) searched by the world-8 global batch (8 x 4096 queries), as a rank
of the driver's 8-GPU run would.  Records per (record, rank) the queries the
certificate left uncertified (answered by the collect pass, in rounds of
16,384 slots) and those that reached the fp64 scans, plus the time of one
search.  Usage: python tools/shard_geometry.py [--ranks 0,7] [--out FILE]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from newsrecommend_amd import faiss as nf
from newsrecommend_amd.data import clustered_corpus

ap = argparse.ArgumentParser()
ap.add_argument("--ranks", default="0,7")
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--out", default=None)
a = ap.parse_args()
dev = torch.device("cuda", 0)
W = a.world
nq = 4096 * W
# (record, corpus rows, dim, metric, k): configs[1] flat IP, the IVF record's
# flat L2 leg, north_star's N1, configs[4]'s top-200 retrieval (queries: draws
# from the corpus mixture for all four; bench_e2e's are user profiles)
records = [("flat_ip_1m_128", 1_000_000, 128, nf.METRIC_INNER_PRODUCT, 5),
           ("flat_l2_10m_128", 10_000_000, 128, nf.METRIC_L2, 5),
           ("n1_ip_10m_256", 10_000_000, 256, nf.METRIC_INNER_PRODUCT, 5),
           ("e2e_ip_10m_256_k200", 10_000_000, 256, nf.METRIC_INNER_PRODUCT, 200)]
out = {"world": W, "queries": nq, "records": {}}
for name, n, d, metric, k in records:
    xb = clustered_corpus(n, d, seed=1234, device=dev)
    xq = clustered_corpus(nq, d, seed=4321, device=dev)
    for r in [int(x) for x in a.ranks.split(",")]:
        lo, hi = r * n // W, (r + 1) * n // W
        idx = nf.IndexFlat(d, metric, device=dev)
        idx.add(xb[lo:hi])
        idx.search_device(xq, k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        idx.search_device(xq, k)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        rec = {"shard_rows": hi - lo, "uncertified": int(idx.last_fallback.item()),
               "fp64_scanned": int(idx.last_exact_scan.item()), "ms_per_search": ms}
        out["records"][f"{name}/rank{r}"] = rec
        print(name, r, rec, flush=True)
        del idx
        torch.cuda.empty_cache()
    del xb, xq
    torch.cuda.empty_cache()
print(json.dumps(out), flush=True)
if a.out:
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
