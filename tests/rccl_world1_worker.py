"""Worker for tests/test_dist_gpu.py::test_rccl_branch_world1: a world-1
`nccl` (RCCL) process group on cuda:0 plus a gloo group over the same rank, so
the `== "nccl"` branches of newsrecommend_amd.dist run on DEVICE buffers
(all_gather_into_tensor, all_to_all_single with split sizes, all_reduce) and
are compared bit for bit with the gloo branches (host copies).  Also captures
the data-parallel gradient all_reduce inside FusedTrainStep's HIP graph (the
form an N-GPU DIN run uses) and checks it against the un-hooked step.

    MASTER_ADDR=127.0.0.1 MASTER_PORT=P RANK=0 WORLD_SIZE=1 \
        python tests/rccl_world1_worker.py <out.json>
"""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out = sys.argv[1]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    gloo = dist.new_group(backend="gloo")
    from newsrecommend_amd import faiss as nf
    from newsrecommend_amd.dist import all_gather_results, all_reduce_mean_, scatter_results

    res = {"backend": dist.get_backend(), "gloo_backend": dist.get_backend(gloo)}
    g = torch.Generator(device=dev).manual_seed(1)
    nq, k = 333, 10
    S = torch.randn((nq, k), generator=g, device=dev, dtype=torch.float64).sort(1, descending=True).values
    I = torch.randint(0, 1 << 40, (nq, k), generator=g, device=dev)
    Sa, Ia = all_gather_results(S, I)
    Sb, Ib = all_gather_results(S, I, gloo)
    res["all_gather_device"] = Sa.is_cuda and Ia.is_cuda
    res["all_gather_equal"] = bool(torch.equal(Sa, Sb) and torch.equal(Ia, Ib) and torch.equal(Sa[0], S)
                                   and torch.equal(Ia[0], I))
    Sa, Ia = scatter_results(S, I)
    Sb, Ib = scatter_results(S, I, gloo)
    res["scatter_equal"] = bool(torch.equal(Sa, Sb) and torch.equal(Ia, Ib) and torch.equal(Sa[0], S))
    # merge after the RCCL gather == the input lists (one shard)
    Dm, Im, Sm = nf.topk_merge(*all_gather_results(S, I), k, nf.METRIC_INNER_PRODUCT)
    res["merge_equal"] = bool(torch.equal(Im, I) and torch.equal(Sm, S))
    t = torch.randn(100_003, generator=g, device=dev)
    a, b = t.clone(), t.clone()
    all_reduce_mean_(a)
    all_reduce_mean_(b, gloo)
    res["all_reduce_equal"] = bool(torch.equal(a, b) and torch.equal(a, t))

    # DIN data-parallel hook inside the captured step graph (RCCL all_reduce
    # captured into a HIP graph) == the same steps without the hook
    from newsrecommend_amd.data import synthetic_click_rows
    from newsrecommend_amd.din import DIN, FusedTrainStep

    table = (torch.randn((4000, 64), generator=g, device=dev) * 0.5).to(torch.bfloat16)
    hist, tgt, lab = synthetic_click_rows(2048, 4000, 20, seed=5, device=dev)
    torch.manual_seed(0)
    ma = DIN(64, 64, 32, 0.0).to(dev)
    mb = DIN(64, 64, 32, 0.0).to(dev)
    mb.load_state_dict(ma.state_dict())
    ta = FusedTrainStep(ma, table, hist, tgt, lab, 256, lr=1e-3, graph=True, grad_hook=lambda G: all_reduce_mean_(G),
                        steps_per_graph=2)
    tb = FusedTrainStep(mb, table, hist, tgt, lab, 256, lr=1e-3, graph=True, steps_per_graph=2)
    idx = torch.arange(1024, device=dev).view(2, 2, 256)
    for r in range(2):
        ta.step_many(idx[r])
        tb.step_many(idx[r])
    torch.cuda.synchronize()
    res["dp_graph_equal"] = bool(torch.equal(ta.P, tb.P) and torch.equal(ta.M, tb.M) and torch.equal(ta.V, tb.V))
    res["dp_graph_loss_equal"] = bool(torch.equal(ta.loss_ring, tb.loss_ring))
    torch.cuda.synchronize()
    with open(out, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
