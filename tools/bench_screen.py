"""Time the k-NN stages for env-selected kernel variants, interleaved in one
process (MI355X: cross-process variance is larger than most deltas).
usage: python tools/bench_screen.py VAR=val1,val2 [VAR2=...] [--nb N --nq Q --k K --d D --metric ip]"""
import argparse, itertools, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from newsrecommend_amd import _lib, faiss as nf
from newsrecommend_amd.data import clustered_corpus

ap = argparse.ArgumentParser()
ap.add_argument("vars", nargs="*")
ap.add_argument("--nb", type=int, default=1_000_000)
ap.add_argument("--nq", type=int, default=4096)
ap.add_argument("--d", type=int, default=128)
ap.add_argument("--k", type=int, default=5)
ap.add_argument("--metric", default="ip")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--queries", choices=["corpus", "profiles"], default="corpus",
                help="profiles: bench.py e2e's user profiles (mean of 1..50 Zipf-drawn corpus rows)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
xb = clustered_corpus(a.nb, a.d, seed=1234, device=dev)
if a.queries == "corpus":
    xq = clustered_corpus(a.nq, a.d, seed=4321, device=dev)
else:  # as bench.py bench_e2e
    from newsrecommend_amd.data import zipf_ids
    g = torch.Generator(device=dev).manual_seed(11)
    L = 50
    hist = zipf_ids(a.nq * L, a.nb, generator=g, device=dev).view(a.nq, L).long()
    lens = torch.randint(1, L + 1, (a.nq,), generator=g, device=dev)
    valid = (torch.arange(L, device=dev)[None] < lens[:, None]).unsqueeze(-1)
    xq = (xb.to(torch.bfloat16)[hist].float() * valid).sum(1) / valid.sum(1)
idx = nf.IndexFlat(a.d, 0 if a.metric == "ip" else 1, device=dev)
idx.add(xb)
grid = [[(v.split("=")[0], x) for x in v.split("=")[1].split(",")] for v in a.vars] or [[("NONE", "0")]]
combos = list(itertools.product(*grid))
ref = None
res = {c: [] for c in combos}
fbs = {c: 0 for c in combos}
for r in range(a.rounds):
    for c in combos:
        for k, v in c:
            os.environ[k] = v
        ev = [_lib.StageEvents() for _ in range(a.reps)]
        D, I = idx.search_device(xq, a.k)  # warm
        for e in ev:
            D, I = idx.search_device(xq, a.k, stage_events=e)
        st = np.array([e.elapsed_ms() for e in ev]).mean(0)
        res[c].append(st)
        if ref is None:
            ref = I.clone()
        ok = "" if ref is None else ("ok" if torch.equal(I, ref) else "DIFF")
        fb = int(idx.last_fallback.item())
        fbs[c] = max(fbs[c], fb)
        print(f"round {r} {c}: stages ms {np.round(st, 4).tolist()} fallback={fb} {ok}", flush=True)
for c in combos:
    m = np.median(np.array(res[c]), 0)
    flops = 2.0 * a.nq * a.nb * a.d
    print(f"{c}: screen {m[1]:.4f} ms = {flops / m[1] / 1e9:.1f} TFLOP/s; merge {m[2]:.4f}; total {m.sum():.4f}; "
          f"stages {np.round(m, 4).tolist()}; fallback {fbs[c]}; id checksum {int(ref.sum())}")
