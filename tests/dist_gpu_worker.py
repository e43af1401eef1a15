"""Worker for tests/test_dist_gpu.py: one rank of a world-2 gloo group, both
ranks on cuda:0 (the GPU box has one card).  Runs the PRODUCT's sharding code
(newsrecommend_amd.dist: ShardedIndexFlat / ShardedIndexIVFFlat add_full +
search_device, all_gather_results, nrk_topk_merge) and the data-parallel
FusedTrainStep gradient hook, and writes what it saw to <out>/rank<r>.json.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port P tests/dist_gpu_worker.py <out_dir>
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _mixture(nb, nq, d, seed, centers=40):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((centers, d)).astype(np.float32)
    xb = (c[rng.integers(0, centers, nb)] + 0.35 * rng.standard_normal((nb, d))).astype(np.float32)
    xq = (c[rng.integers(0, centers, nq)] + 0.35 * rng.standard_normal((nq, d))).astype(np.float32)
    return xq, xb


def main():
    out_dir = sys.argv[1]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from newsrecommend_amd import faiss as nf
    from newsrecommend_amd.dist import ShardedIndexFlat, ShardedIndexIVFFlat, all_reduce_mean_

    res = {"rank": rank, "world": world}
    # ---- flat: sharded == one index over the whole corpus (ties across shards included)
    xq, xb = _mixture(50_001, 300, 64, seed=5)
    xb[40_000] = xb[7]  # duplicate in the other shard: the lower global id must win
    xq[0] = xb[7]
    q = torch.from_numpy(xq).to(dev)
    for metric in (nf.METRIC_INNER_PRODUCT, nf.METRIC_L2):
        sh = ShardedIndexFlat(64, metric, device=dev)
        sh.add_full(torch.from_numpy(xb).to(dev))
        D, I = sh.search_device(q, 10)
        one = nf.IndexFlat(64, metric, device=dev)
        one.add(xb)
        D1, I1 = one.search_device(q, 10)
        res[f"flat{metric}_I_equal"] = bool(torch.equal(I, I1))
        res[f"flat{metric}_D_equal"] = bool(torch.equal(D, D1))
        res[f"flat{metric}_local_rows"] = sh.local.ntotal
        # the all_to_all form (configs[4]'s user-sharded re-rank): this rank's query slice only
        from newsrecommend_amd.dist import shard_range

        Do, Io = sh.search_device_own(q, 10)
        qlo, qhi = shard_range(q.shape[0], rank, world)
        res[f"flat{metric}_own_equal"] = bool(torch.equal(Io, I1[qlo:qhi]) and torch.equal(Do, D1[qlo:qhi]))
    # ---- IVF: replicated deterministic k-means, row-split lists == single IVF
    xq, xb = _mixture(60_000, 257, 32, seed=6)
    sh = ShardedIndexIVFFlat(32, 24, nf.METRIC_L2, device=dev)
    sh.local.cp.niter = 4
    sh.train(xb)
    sh.add_full(torch.from_numpy(xb).to(dev))
    sh.nprobe = 5
    D, I = sh.search_device(torch.from_numpy(xq).to(dev), 7)
    one = nf.IndexIVFFlat(nf.IndexFlatL2(32, device=dev), 32, 24, nf.METRIC_L2, device=dev)
    one.cp.niter = 4
    one.train(xb)
    one.add(xb)
    one.nprobe = 5
    D1, I1 = one.search_device(torch.from_numpy(xq).to(dev), 7)
    res["ivf_centroids_equal"] = bool(torch.equal(sh.quantizer._xb[:24], one.quantizer._xb[:24]))
    res["ivf_I_equal"] = bool(torch.equal(I, I1))
    res["ivf_D_equal"] = bool(torch.equal(D, D1))
    # ---- DIN data parallel: the hooked gradient is the rank mean, replicas stay identical
    from newsrecommend_amd.data import synthetic_click_rows
    from newsrecommend_amd.din import DIN, FusedTrainStep

    g = torch.Generator(device=dev).manual_seed(3)
    table = (torch.randn((4000, 64), generator=g, device=dev) * 0.5).to(torch.bfloat16)
    hist, tgt, lab = synthetic_click_rows(2048, 4000, 20, seed=5, device=dev)
    B = 256
    torch.manual_seed(0)  # identical initial replicas
    m_dp = DIN(64, 64, 32, 0.0).to(dev)
    m_solo = DIN(64, 64, 32, 0.0).to(dev)
    m_solo.load_state_dict(m_dp.state_dict())
    seen = {}

    def dp_hook(G):
        all_reduce_mean_(G)
        seen["dp"] = G.clone()

    def solo_hook(G):
        seen["solo"] = G.clone()

    dp = FusedTrainStep(m_dp, table, hist, tgt, lab, B, lr=1e-3, graph=False, grad_hook=dp_hook)
    solo = FusedTrainStep(m_solo, table, hist, tgt, lab, B, lr=1e-3, graph=False, grad_hook=solo_hook)
    err_mean, err_param = 0.0, 0.0
    for s in range(3):
        idx = torch.arange((2 * s + rank) * B, (2 * s + rank + 1) * B, device=dev)  # each rank its own rows
        dp.step(idx)
        solo.step(idx)
        solo.P.copy_(dp.P)  # keep the solo replica on the dp trajectory: one step's gradient each time
        solo.M.copy_(dp.M)
        solo.V.copy_(dp.V)
        for (_, a), (_, b) in zip(m_dp.named_buffers(), m_solo.named_buffers()):
            b.copy_(a)
        grads = [torch.empty_like(seen["solo"]).cpu() for _ in range(world)]
        dist.all_gather(grads, seen["solo"].cpu())
        mean = torch.stack(grads).mean(0).to(dev)
        err_mean = max(err_mean, (seen["dp"] - mean).abs().max().item() / max(mean.abs().max().item(), 1e-30))
        params = [torch.empty_like(dp.P).cpu() for _ in range(world)]
        dist.all_gather(params, dp.P.cpu())
        err_param = max(err_param, (params[0] - params[-1]).abs().max().item())
    res["dp_grad_rel_err"] = err_mean
    res["dp_replica_param_diff"] = err_param
    torch.cuda.synchronize()
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
