"""Replay the configs[2] fused DIN train step (B = 4096 by default) for kernel
traces and wall time: python tools/din_step.py [--B 4096 --steps 50 --drop 0.36]
Under `rocprofv3 --kernel-trace`, tools/step_breakdown.py TRACE clip_adam
prints one step's kernels."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from newsrecommend_amd.data import synthetic_click_rows
from newsrecommend_amd.din import DIN, FusedTrainStep

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=4096)
ap.add_argument("--steps", type=int, default=50)
ap.add_argument("--drop", type=float, default=0.36)
ap.add_argument("--items", type=int, default=2_000_000)
ap.add_argument("--rows", type=int, default=1_000_000)
ap.add_argument("--k", type=int, default=1, help="steps per graph launch (FusedTrainStep.step_many)")
ap.add_argument("--d", type=int, default=128, help="emb_dim (256: the reference's corpus width)")
ap.add_argument("--L", type=int, default=50, help="history length")
a = ap.parse_args()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
table = (torch.randn((a.items, a.d), generator=g, device=dev) * 0.5).to(torch.bfloat16)
hist, tgt, lab = synthetic_click_rows(a.rows, a.items, a.L, seed=7, device=dev)
torch.manual_seed(42)
model = DIN(a.d, 128, 32, a.drop).to(dev)
tr = FusedTrainStep(model, table, hist, tgt, lab, a.B, lr=1.62e-3, weight_decay=8.96e-5, clip=1.0, steps_per_graph=a.k)
perm = torch.randperm(a.rows, device=dev)
nb = a.rows // a.B
for s in range(5):
    tr.step(perm[(s % nb) * a.B:(s % nb + 1) * a.B])
torch.cuda.synchronize()
t0 = time.perf_counter()
for s in range(0, a.steps, a.k):
    b = s % (nb - nb % a.k)
    loss = (tr.step(perm[b * a.B:(b + 1) * a.B]) if a.k == 1 else
            tr.step_many(perm[b * a.B:(b + a.k) * a.B].view(a.k, a.B))[-1])
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / a.steps
print(f"d={a.d} L={a.L} B={a.B} ({tr.path}): {dt * 1e6:.1f} us/step = {a.B / dt / 1e6:.2f} M samples/s, loss {loss.item():.4f}", flush=True)
