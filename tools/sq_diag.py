"""Break down the numpy single-query search latency (host staging, library call, copy-back, stream sync)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from newsrecommend_amd import faiss as nf
rng = np.random.default_rng(0)
cent = rng.standard_normal((300, 256)).astype(np.float32)
prof = rng.standard_normal((2000, 256)).astype(np.float32)
idx = nf.IndexFlatL2(256); idx.add(cent)
for i in range(50): idx.search(prof[i:i+1], 1)
torch.cuda.synchronize()
hb = idx._host_buffers(1, 1)
st = torch.cuda.current_stream()
T = {"stage": 0., "launch": 0., "copyback": 0., "sync": 0.}
for i in range(500):
    t0 = time.perf_counter()
    hb["hq"][:1].numpy()[...] = prof[i:i+1]
    hb["dq"][:1].copy_(hb["hq"][:1], non_blocking=True)
    t1 = time.perf_counter()
    idx._launch(hb["dq"][:1], 1, 1, hb["dD"][:1].view(1, 1), hb["dI"][:1].view(1, 1), None)
    t2 = time.perf_counter()
    hb["hD"][:1].copy_(hb["dD"][:1], non_blocking=True); hb["hI"][:1].copy_(hb["dI"][:1], non_blocking=True)
    t3 = time.perf_counter()
    st.synchronize()
    t4 = time.perf_counter()
    T["stage"] += t1 - t0; T["launch"] += t2 - t1; T["copyback"] += t3 - t2; T["sync"] += t4 - t3
print({k: round(v / 500 * 1e6, 1) for k, v in T.items()}, "us per call")
