"""Time the DIN step's small fp32 GEMM shapes under a few formulations."""
import torch, time
dev = torch.device("cuda")
B, d, A = 4096, 128, 128
q = torch.randn(B, d, device=dev); W = torch.randn(A, 2 * d, device=dev); b = torch.randn(A, device=dev)
dU = torch.randn(B, A, device=dev)
Wq = W[:, :d]
Wqc = Wq.contiguous()
Wqt = Wq.t().contiguous()
variants = {
    "addmm(b,q,Wq.t()) strided": lambda: torch.addmm(b, q, Wq.t()),
    "addmm(b,q,Wqc.t())": lambda: torch.addmm(b, q, Wqc.t()),
    "addmm(b,q,Wqt)": lambda: torch.addmm(b, q, Wqt),
    "mm(q,Wqt)+b": lambda: torch.mm(q, Wqt) + b,
    "linear(q,Wqc,b)": lambda: torch.nn.functional.linear(q, Wqc, b),
    "bf16 addmm": lambda: torch.addmm(b.bfloat16(), q.bfloat16(), Wqt.bfloat16()),
    "dU.t()@q": lambda: dU.t() @ q,
    "mm(dU.t().contiguous(), q)": lambda: torch.mm(dU.t().contiguous(), q),
    "(q.t()@dU).t()": lambda: (q.t() @ dU).t(),
    "splitK16 bmm+sum": lambda: torch.bmm(dU.view(16, B // 16, A).transpose(1, 2), q.view(16, B // 16, d)).sum(0),
    "splitK32 bmm+sum": lambda: torch.bmm(dU.view(32, B // 32, A).transpose(1, 2), q.view(32, B // 32, d)).sum(0),
    "splitK64 bmm+sum": lambda: torch.bmm(dU.view(64, B // 64, A).transpose(1, 2), q.view(64, B // 64, d)).sum(0),
}
for name, f in variants.items():
    for _ in range(5): f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20): f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10): g.replay()
    torch.cuda.synchronize()
    print(f"{name:32s} {(time.perf_counter() - t) / 200 * 1e6:8.1f} us")
