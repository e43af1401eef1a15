"""Time the DIN attention kernels for env-selected variants, interleaved in one process.
usage: python tools/bench_din.py VAR=a,b ... [--B 4096 --L 50 --d 128 --A 128 --items 2000000]"""
import argparse, itertools, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from newsrecommend_amd.din import AttentionLayer, KernelTimer
from newsrecommend_amd.data import synthetic_click_rows

ap = argparse.ArgumentParser()
ap.add_argument("vars", nargs="*")
ap.add_argument("--B", type=int, default=4096)
ap.add_argument("--L", type=int, default=50)
ap.add_argument("--d", type=int, default=128)
ap.add_argument("--A", type=int, default=128)
ap.add_argument("--items", type=int, default=2_000_000)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
table = (torch.randn((a.items, a.d), generator=g, device=dev) * 0.5).to(torch.bfloat16)
hist, tgt, lab = synthetic_click_rows(a.B, a.items, a.L, seed=7, device=dev)
torch.manual_seed(0)
layer = AttentionLayer(a.d, a.A).to(dev)
q = table[tgt.long()].float()
grid = [[(v.split("=")[0], x) for x in v.split("=")[1].split(",")] for v in a.vars] or [[("NONE", "0")]]
combos = list(itertools.product(*grid))
res = {c: [] for c in combos}
ref = None
for r in range(a.rounds):
    for c in combos:
        for k, v in c:
            os.environ[k] = v
        with KernelTimer() as kt:
            for _ in range(a.reps):
                out = layer.forward_ids(q, table, hist)
                out.backward(torch.ones_like(out))
        torch.cuda.synchronize()
        f, b = kt.mean_ms("fwd", skip=1), kt.mean_ms("bwd", skip=1)
        if ref is None:
            ref = out.detach().clone()
        err = (out.detach() - ref).abs().max().item()
        res[c].append((f, b))
        print(f"round {r} {c}: fwd {f:.4f} ms bwd {b:.4f} ms  max|out-ref| {err:.2e}", flush=True)
fb = a.L * a.d * 2 + 4 * a.L + 4 * a.A + 4 * a.d + 4 * a.L
for c in combos:
    f, b = np.median(np.array(res[c]), 0)
    print(f"{c}: fwd {f:.4f} ms = {a.B * fb / f / 1e6:.0f} GB/s ; bwd {b:.4f} ms = {a.B * (fb + 4 * a.A) / b / 1e6:.0f} GB/s")
