"""Time the corpus producer (nrk_embed via ArticleEmbeddingModel.embed) on
synthetic features: python tools/embed_step.py [--n 10000000] [--reps 5]
Prints ms per pass, rows/s, fp32-equivalent TF/s and the bf16 MFMA rate."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from newsrecommend_amd.embedding import ArticleEmbeddingModel

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda", 0)
torch.manual_seed(5)
m = ArticleEmbeddingModel().to(dev).eval()
x = torch.randn((a.n, 253), device=dev)
y = m.embed(x)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.reps):
    y = m.embed(x)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / a.reps
f32 = 2.0 * (253 * 512 + 512 * 256) * a.n / dt / 1e12
bf = 6 * 2.0 * (256 * 512 + 512 * 256) * a.n / dt / 1e12
with torch.no_grad():
    ref = m(x[:2048])
print(f"embed n={a.n}: {dt * 1e3:.3f} ms/pass = {a.n / dt / 1e6:.1f} M rows/s, {f32:.1f} fp32-equiv TF/s "
      f"({f32 / 157.3:.3f} of the fp32 MFMA peak), {bf:.0f} bf16 MFMA TF/s ({bf / 2500:.3f}); "
      f"max |y - module forward| {float((y[:2048] - ref).abs().max()):.3g}", flush=True)
