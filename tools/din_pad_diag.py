"""Diagnose the fused train step's W1 gradient against the fp64 oracle on
padded histories (tests/test_din_bf16_oracle.py's c3-shape check, one step):
error split into W1's query / key halves, per padding pattern."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from newsrecommend_amd.data import synthetic_click_rows
from newsrecommend_amd.din import DIN, FusedTrainStep
from oracle import din_oracle as o


def bf(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(torch.bfloat16).float().numpy()


def run(d, L, B, A, F, pad):
    dev = torch.device("cuda")
    N = 6000
    g = torch.Generator(device=dev).manual_seed(21)
    table = (torch.randn((N, d), generator=g, device=dev) * 0.5).to(torch.bfloat16)
    hist, tgt, lab = synthetic_click_rows(max(4 * B, 2048), N, L, seed=9, device=dev)
    if "none" in pad:
        hist[0::7] = -1
    if "one" in pad:
        hist[1::7, 1:] = -1
    torch.manual_seed(3)
    model = DIN(d, A, F, 0.0).to(dev)
    fused = FusedTrainStep(model, table, hist, tgt, lab, B, lr=1.62e-3, weight_decay=8.96e-5, clip=1.0, graph=False)
    T = table.float().cpu().numpy().astype(np.float64)
    H, Tg, Y = hist.cpu().numpy(), tgt.cpu().numpy(), lab.cpu().numpy().reshape(-1, 1).astype(np.float64)
    p = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in model.state_dict().items() if "num_batches" not in k}
    p["attn.attn.0.weight"][:, d:] = bf(p["attn.attn.0.weight"][:, d:].astype(np.float32))
    rows = np.arange(B)
    fused.step(torch.from_numpy(rows).to(dev))
    q = T[Tg[rows]]
    keys = np.where(H[rows][..., None] >= 0, T[np.maximum(H[rows], 0)], 0.0)
    lo, pooled, _, cache = o.din_forward(p, q, keys, train=True)
    gr = o.din_backward(p, cache, lo, Y[rows])
    g_cl, nrm = o.clip_grad_norm(gr, 1.0)
    ref = g_cl["attn.attn.0.weight"]
    got = model.attn.attn[0].weight.grad.detach().cpu().numpy().astype(np.float64)
    e = np.abs(got - ref)
    print(f"d={d} L={L} pad={pad}: norm {nrm:.4g}, max|g| {np.abs(ref).max():.4g}, err q-half {e[:, :d].max():.3g}, "
          f"k-half {e[:, d:].max():.3g}, rel {e.max() / np.abs(ref).max():.3g}; argmax {np.unravel_index(e.argmax(), e.shape)}")
    for n in ("attn.attn.0.bias", "attn.attn.2.weight", "fc.1.weight"):
        r = g_cl[n].reshape(-1)
        gg = dict(model.named_parameters())[n].grad.detach().cpu().numpy().reshape(-1).astype(np.float64)
        print(f"   {n}: rel {np.abs(gg - r).max() / np.abs(r).max():.3g}")


for pad in ("", "none", "one", "none+one"):
    run(128, 50, 512, 128, 32, pad)
run(256, 100, 256, 128, 32, "none+one")
