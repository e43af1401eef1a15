"""CPU, world_size 2 over gloo: the shard exchange of newsrecommend_amd.dist
(pack -> one all_gather -> unpack) feeding the merge gives exactly the
single-index result.  The per-shard search here is the oracle (no GPU in this
container); on the GPU box test_knn_gpu covers the device merge kernel."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from newsrecommend_amd.dist import all_gather_results, shard_range
        from oracle import knn_oracle as ko

        rng = np.random.default_rng(3)
        xb = rng.standard_normal((2501, 20)).astype(np.float32)
        xb[2400] = xb[11]  # cross-shard duplicate: tie must resolve to the lower global id
        xq = rng.standard_normal((33, 20)).astype(np.float32)
        xq[0] = xb[11]
        k = 6
        for metric in (ko.METRIC_IP, ko.METRIC_L2):
            lo, hi = shard_range(xb.shape[0], rank, world)
            _, I, S = ko.exact_search(xq, xb[lo:hi], k, metric, id_offset=lo)
            S_all, I_all = all_gather_results(torch.from_numpy(S), torch.from_numpy(I))
            _, Im, Sm = ko.merge(S_all.numpy(), I_all.numpy(), k, metric)
            _, Ig, Sg = ko.exact_search(xq, xb, k, metric)
            ok = np.array_equal(Im, Ig) and np.array_equal(Sm, Sg)
            np.save(os.path.join(out_dir, f"ok_{metric}_{rank}.npy"), np.array([ok, Im[0, 1] == 2400]))
    finally:
        dist.destroy_process_group()


def test_two_rank_exchange_and_merge(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for metric in (0, 1):
        for r in range(world):
            ok, tie = np.load(tmp_path / f"ok_{metric}_{r}.npy")
            assert ok and tie


def _ivf_worker(rank, world, port, out_dir):
    """Sharded IVF (configs[3] layout): replicated centroids, each rank's rows
    of every list, one exchange, merge == single-index IVF search."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from newsrecommend_amd.dist import all_gather_results, shard_range
        from oracle import ivf_oracle as io
        from oracle import knn_oracle as ko

        rng = np.random.default_rng(5)
        xb = rng.standard_normal((3001, 16)).astype(np.float32)
        xq = rng.standard_normal((20, 16)).astype(np.float32)
        cent, _ = io.kmeans(xb, 12, niter=3)  # identical on every rank (deterministic)
        assign, _ = io.assign_nearest(xb, cent)
        k, nprobe = 5, 3
        lo, hi = shard_range(xb.shape[0], rank, world)
        oks = []
        for metric in (ko.METRIC_IP, ko.METRIC_L2):
            _, I, S, _ = io.ivf_search(xq, xb[lo:hi], cent, assign[lo:hi], nprobe, k, metric)
            I = np.where(I >= 0, I + lo, -1)
            S_all, I_all = all_gather_results(torch.from_numpy(S), torch.from_numpy(I))
            _, Im, Sm = ko.merge(S_all.numpy(), I_all.numpy(), k, metric)
            _, Ig, Sg, _ = io.ivf_search(xq, xb, cent, assign, nprobe, k, metric)
            oks.append(np.array_equal(Im, Ig) and np.array_equal(Sm, Sg))
        np.save(os.path.join(out_dir, f"ivf_ok_{rank}.npy"), np.array(oks))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharded_ivf(tmp_path):
    world = 2
    mp.spawn(_ivf_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert np.load(tmp_path / f"ivf_ok_{r}.npy").all()


def _scatter_worker(rank, world, port, out_dir):
    """The all_to_all exchange of the user-sharded e2e (ShardedIndexFlat.
    search_device_own): rank r receives every shard's lists for its own query
    slice only, and their merge equals the single-index result of that slice."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from newsrecommend_amd.dist import scatter_results, shard_range
        from oracle import knn_oracle as ko

        rng = np.random.default_rng(9)
        xb = rng.standard_normal((1999, 24)).astype(np.float32)
        xq = rng.standard_normal((37, 24)).astype(np.float32)  # odd: unequal query slices
        xb[1500] = xb[4]
        xq[0] = xb[4]  # a cross-shard tie in each query slice
        xq[20] = xb[4]
        k = 7
        oks = []
        for metric in (ko.METRIC_IP, ko.METRIC_L2):
            lo, hi = shard_range(xb.shape[0], rank, world)
            _, I, S = ko.exact_search(xq, xb[lo:hi], k, metric, id_offset=lo)
            S_own, I_own = scatter_results(torch.from_numpy(S), torch.from_numpy(I))
            qlo, qhi = shard_range(xq.shape[0], rank, world)
            assert S_own.shape == (world, qhi - qlo, k)
            _, Im, Sm = ko.merge(S_own.numpy(), I_own.numpy(), k, metric)
            _, Ig, Sg = ko.exact_search(xq[qlo:qhi], xb, k, metric)
            oks.append(np.array_equal(Im, Ig) and np.array_equal(Sm, Sg))
        np.save(os.path.join(out_dir, f"scatter_ok_{rank}.npy"), np.array(oks))
    finally:
        dist.destroy_process_group()


def test_two_rank_scatter_exchange(tmp_path):
    world = 2
    mp.spawn(_scatter_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert np.load(tmp_path / f"scatter_ok_{r}.npy").all()
