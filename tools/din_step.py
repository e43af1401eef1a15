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
ap.add_argument("--ktime", action="store_true",
                help="per-workgroup phase times of the head-fused backward and (NRK_DIN_FWD_PAIR=0, set here) "
                     "of the wave-per-sample forward")
ap.add_argument("--hktime", action="store_true",
                help="per-block phase stamps of the fast head's kernels (nrk_debug_head_ktimes)")
a = ap.parse_args()
if a.hktime:
    os.environ["NRK_KTIME"] = "1"
if a.ktime:
    os.environ["NRK_KTIME"] = "1"
    os.environ.setdefault("NRK_DIN_FWD_PAIR", "0")
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
table = (torch.randn((a.items, 128), generator=g, device=dev) * 0.5).to(torch.bfloat16)
hist, tgt, lab = synthetic_click_rows(a.rows, a.items, 50, seed=7, device=dev)
torch.manual_seed(42)
model = DIN(128, 128, 32, a.drop).to(dev)
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
print(f"B={a.B}: {dt * 1e6:.1f} us/step = {a.B / dt / 1e6:.2f} M samples/s, loss {loss.item():.4f}", flush=True)
if a.ktime:
    import ctypes
    import numpy as np
    from newsrecommend_amd import _lib
    nwg = 256
    buf = np.zeros(4096 * 8 * 9 + 1024 * 8, dtype=np.uint64)
    _lib.check(_lib.load().nrk_debug_ktimes(buf.ctypes.data, buf.size), "debug_ktimes")
    t = buf[:nwg * 8].reshape(nwg, 8).astype(np.int64)
    t0 = t[:, 0].min()
    us = (t - t0) / 100.0  # 100 MHz ticks -> us
    names = ["entry", "ids", "first", "loop", "flush", "exit"]
    for i, n in enumerate(names):
        c = us[:, i]
        print(f"  {n:6s} min {c.min():7.2f} med {np.median(c):7.2f} max {c.max():7.2f} us", flush=True)
    d = us[:, 3] - us[:, 2]
    print(f"  loop span per WG: min {d.min():.2f} med {np.median(d):.2f} max {d.max():.2f} us", flush=True)
    if os.environ.get("NRK_DEEP8_PIPE") == "1":
        k2 = buf[4096 * 8:4096 * 8 + nwg * 64].reshape(nwg, 8, 8).astype(np.float64)
        nit = k2[:, :, 5].max()
        for j, n in enumerate(["wait+barrier", "issue", "stage A", "stage B", "stage C"]):
            c = k2[:, :, j] / np.maximum(k2[:, :, 5], 1)  # cycles per iteration
            print(f"  {n:13s} cycles/iter: wave0 med {np.median(c[:, 0]):7.0f}  all-waves med {np.median(c):7.0f} "
                  f"max {c.max():7.0f}", flush=True)
        print(f"  iterations per WG {nit:.0f}", flush=True)
    f = buf[4096 * 8 * 9:].reshape(1024, 8).astype(np.int64)
    f = f[:min(512, (a.B + 3) // 4)]  # the d = 128 forward's grid
    fu = (f - f[:, 0].min()) / 100.0
    for j, n in enumerate(["fwd entry", "s0 landed", "s0 done", "s1 landed", "s1 done", "s2 landed", "s2 done"]):
        c = fu[:, j]
        if (f[:, j] > 0).all():
            print(f"  {n:10s} min {c.min():7.2f} med {np.median(c):7.2f} max {c.max():7.2f} us", flush=True)
if a.hktime:
    import numpy as np
    from newsrecommend_amd import _lib
    buf = np.zeros(8 * 128 * 8, dtype=np.uint64)
    _lib.check(_lib.load().nrk_debug_head_ktimes(buf.ctypes.data, buf.size), "debug_head_ktimes")
    t = buf.reshape(8, 128, 8).astype(np.int64)
    names = ["stats0", "fwd1", "fwd2", "fwd3", "bwd2", "bwd1", "reduce"]
    base = t[0, :, 0][t[0, :, 0] > 0].min()
    for k, n in enumerate(names):
        blk = t[k][t[k, :, 0] > 0]
        if len(blk) == 0:
            continue
        us = (blk - base) / 100.0
        cols = []
        for i in range(8):
            ok = blk[:, i] > 0  # blocks that stamp slot i (hf_reduce: the G blocks only past s0)
            if ok.any():
                v = us[ok, i]
                cols.append(f"s{i}: med {np.median(v):7.2f} [{v.min():7.2f}, {v.max():7.2f}]")
        print(f"  {n:7s} " + "  ".join(cols), flush=True)
