#!/usr/bin/env python3
"""bench.py — the driver's benchmark contract for the NewsRecommend hot path.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Headline (BASELINE.json `metric`, configs[1]): exact flat retrieval, 1M x 128
items, batches of nq = 4096 queries per GPU, k = 5, inner product.  One STEP =
one search of one batch (inputs resident in HBM).  At N > 1 the corpus is
row-sharded over the ranks (north_star: per-shard exact top-k lists merged
after ONE RCCL all_gather, newsrecommend_amd.dist) and the global batch is
N x 4096 queries, every rank searching all of them against its shard: the
per-GPU work is that of one GPU at N = 1 (weak scaling).  value = queries
answered / max-over-ranks wall time of the K timed steps.

Secondary record `ivf` (configs[3] shape): IVF-Flat nlist=300, nprobe=32 over
10M x 128 items (L2), rows split over the ranks, exact top-k per rank merged
after one all_gather; recall@5 against the exact flat search; N x 4096
queries per step.  `n1_retrieval_10m_256_k5` (north_star's target): flat IP
k = 5 over 10M x 256, corpus sharded the same way, N x 4096 queries.

Secondary record `e2e` (configs[4] shape): flat top-200 over 10M x 256 items
(corpus sharded) for N x 4096 users -> ground truth appended -> DIN re-rank of
this rank's 4096 users (users sharded) -> NDCG@5; value = users/s end to end.

Secondary record `din` (configs[2]): DIN training, bf16 table of 2M items,
5M synthetic click rows, L = 50, d = 128, A = 128, F = 32; one step = fwd +
bwd + clip + Adam on a batch of --din-batch rows; data-parallel replicas with
a gradient all_reduce at N > 1.

Rank 0 prints ONE JSON line.  `roofline` is the screening kernel (MFMA-bound)
timed live with HIP events on its launch stream; `cpu_baseline` times the
oracle's restatement of faiss-cpu's flat search on this host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
BF16_DENSE_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16 MFMA
HBM_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# Rehearsal of the N > 1 code paths on a one-GPU box (never the measured
# configuration): NRK_BENCH_BACKEND=gloo with NRK_BENCH_ONE_DEVICE=1 runs every
# rank on cuda:0 and carries the collectives over gloo host copies.
BACKEND = os.environ.get("NRK_BENCH_BACKEND", "nccl")


def setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if os.environ.get("NRK_BENCH_ONE_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if BACKEND == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(BACKEND)
    return rank, world, torch.device("cuda", local)


def barrier(world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x: float, world: int, dev) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev if BACKEND == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_cores() -> int:
    n = os.environ.get("OMP_NUM_THREADS")
    return int(n) if n else len(os.sched_getaffinity(0))


# ------------------------------------------------------------ retrieval --
def bench_flat(args, rank, world, dev):
    from newsrecommend_amd import _lib
    from newsrecommend_amd.data import clustered_corpus
    from newsrecommend_amd.dist import ShardedIndexFlat

    metric = 0 if args.metric == "ip" else 1
    xb = clustered_corpus(args.nb, args.d, seed=1234, device=dev)
    nq = args.nq * world  # global batch: args.nq queries per GPU
    xq = clustered_corpus(nq, args.d, seed=4321, device=dev)
    index = ShardedIndexFlat(args.d, metric, device=dev)
    index.add_full(xb)
    keep_full = rank == 0
    xb_host = xb.cpu().numpy() if keep_full else None
    del xb
    torch.cuda.empty_cache()
    nb_local = index.local.ntotal

    for _ in range(args.warmup):
        D, I = index.search_device(xq, args.k)
    barrier(world)
    evs = [_lib.StageEvents() for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s in range(args.steps):
        D, I = index.search_device(xq, args.k) if world > 1 else index.local.search_device(
            xq, args.k, stage_events=evs[s])[:2]
        if world > 1:  # stage timing of the local search only
            pass
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    qps = nq * args.steps / el

    # per-stage device times (rank-local), averaged over the timed steps
    if world > 1:  # one extra instrumented local search per step-count for the stage split
        for s in range(args.steps):
            index.local.search_device(xq, args.k, exact_scores=True, id_offset=index.offset, stage_events=evs[s])
        torch.cuda.synchronize()
    st = np.array([e.elapsed_ms() for e in evs])
    stage_ms = st.mean(0)
    screen_ms = float(stage_ms[1])
    flops = 2.0 * nq * nb_local * args.d
    achieved = flops / (screen_ms * 1e-3) / 1e12
    fallback = index.local.fallback_counts.tolist()

    out = {
        "value": qps, "unit": "queries/s", "ms_per_step": el / args.steps * 1e3,
        "stages_ms": {"query_prepare+tau_prepass": float(stage_ms[0]), "screen": screen_ms,
                      "merge_rescore": float(stage_ms[2]), "exact_fallback": float(stage_ms[3])},
        "fallback_queries": fallback[0], "exact_scan_queries": fallback[1],
        "roofline": {"bound": "mfma", "kernel": _screen_kernel_name(nq, nb_local, args.d, args.k, metric),
                     "achieved": achieved, "peak": BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / BF16_DENSE_TFLOPS,
                     "traffic": _pmc_traffic(f"nb={args.nb},d={args.d},nq={args.nq},k={args.k},metric={args.metric},"
                                             f"gpus={world}"),
                     "algorithmic": f"2*nq*nb_local*d = {flops:.4g} flop per launch"},
    }
    if rank == 0:
        out["recall_at_5"], out["exact_match"] = _recall(args, xq, xb_host, D, I, metric)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = _cpu_flat(args, xq, xb_host, metric)
    return out


def _recall(args, xq, xb_host, D, I, metric):
    from oracle import knn_oracle as ko

    sample = np.arange(0, xq.shape[0], max(1, xq.shape[0] // 64))
    q = xq.cpu().numpy()[sample]
    _, Io, _ = ko.exact_search(q, xb_host, args.k, metric)
    Ig = I.cpu().numpy()[sample]
    rec = float(np.mean([len(set(a[:5]) & set(b[:5])) / min(5, args.k) for a, b in zip(Ig, Io)]))
    return rec, bool(np.array_equal(Ig, Io))


def _timed_sample(fn, n_total, n0, budget_s, align=64):
    """Run fn(n) on a first sample of n0 units, then scale n so the second run
    takes about budget_s; returns (n, seconds) of the second run."""
    t = time.perf_counter()
    fn(n0)
    dt = max(time.perf_counter() - t, 1e-3)
    n = int(min(n_total, max(n0, n0 * budget_s / dt)))
    n = max(n0, (n // align) * align)
    t = time.perf_counter()
    fn(n)
    return n, time.perf_counter() - t


def _cpu_flat(args, xq, xb_host, metric, nb=None, d=None, k=None):
    """faiss-cpu IndexFlat's blocked-sgemm search restated on all host cores
    (oracle/cpu_baselines.flat_search, torch CPU kernels), on a bounded query
    sample against the FULL corpus."""
    from oracle import cpu_baselines as cb

    cores = cpu_cores()
    torch.set_num_threads(cores)
    q = xq.cpu()
    xb = torch.from_numpy(xb_host)
    norms = (xb * xb).sum(1) if metric == 1 else None
    k = args.k if k is None else k
    n, dt = _timed_sample(lambda n: cb.flat_search(q[:n], xb, k, metric, xb_norms=norms), q.shape[0], 64,
                          args.cpu_seconds)
    return {"value": n / dt, "unit": "queries/s", "cores": cores, "kind": "port",
            "sample": f"{n} of the {q.shape[0]} queries x full {xb.shape[0]}x{xb.shape[1]} corpus, k={k}, "
                      f"oracle.cpu_baselines.flat_search (faiss exhaustive_*_blas restated: torch-CPU fp32 sgemm "
                      f"blocks + running top-k, {cores} threads), {dt:.1f} s"}


def _screen_kernel_name(nq, nb, d, k, metric):
    """The flat main-pass kernel libnrk runs for this search, as the library
    itself plans it (nrk_knn_flat_main_pass)."""
    import ctypes

    from newsrecommend_amd import _lib

    buf = ctypes.create_string_buffer(256)
    _lib.check(_lib.load().nrk_knn_flat_main_pass(nq, nb, d, k, metric, buf, 256), "knn_flat_main_pass")
    return buf.value.decode()


def _pmc_traffic(key):
    """HBM bytes per launch of the record's dominant kernel from a committed
    rocprofv3 --pmc summary for this exact workload (profiles/pmc_screen.json,
    FETCH_SIZE x2 + WRITE_SIZE from separate passes), else null."""
    p = os.path.join(ROOT, "profiles", "pmc_screen.json")
    try:
        return json.load(open(p)).get(key, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


# ------------------------------------------------------------------ IVF --
def bench_ivf(args, rank, world, dev):
    """configs[3]: IVF-Flat nlist=300, nprobe=32 over 10M x 128 (squared L2),
    the corpus rows split over the ranks (every list partially on every rank),
    per-rank exact top-k merged after one all_gather.  One step = one search
    of a 4096-query batch INCLUDING the coarse quantizer."""
    from newsrecommend_amd import _lib, faiss as nf
    from newsrecommend_amd.data import clustered_corpus
    from newsrecommend_amd.dist import ShardedIndexIVFFlat

    d, k, nlist, nprobe = args.d, args.k, args.ivf_nlist, args.ivf_nprobe
    nq = args.nq * world  # global batch: args.nq queries per GPU (weak scaling)
    xb = clustered_corpus(args.ivf_nb, d, seed=1234, device=dev)
    xq = clustered_corpus(nq, d, seed=4321, device=dev)
    barrier(world)
    t0 = time.perf_counter()
    index = ShardedIndexIVFFlat(d, nlist, nf.METRIC_L2, device=dev)
    index.local.cp.niter = args.ivf_niter
    index.train(xb)
    index.add_full(xb)
    index.nprobe = nprobe
    barrier(world)
    build_s = max_over_ranks(time.perf_counter() - t0, world, dev)
    for _ in range(args.warmup):
        D, I = index.search_device(xq, k)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        D, I = index.search_device(xq, k)
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    qps = nq * args.steps / el
    index.local.check_guards()  # the last search's index guards (include/nrk.h nrk_ivf_search_status)
    # rank-local stage split (instrumented, outside the timed region)
    _, probe = index.quantizer.search_device(xq, nprobe)
    evs = [_lib.StageEvents() for _ in range(max(3, min(args.steps, 10)))]
    for e in evs:
        index.local.search_device(xq, k, probe=probe, stage_events=e)
    torch.cuda.synchronize()
    st = np.array([e.elapsed_ms() for e in evs]).mean(0)
    sizes = torch.diff(index.local.list_off).cpu().numpy()
    pr = probe.cpu().numpy()
    flops = 2.0 * d * float(sizes[pr[pr >= 0]].sum())
    achieved = flops / (st[1] * 1e-3) / 1e12
    out = {
        "metric": "IVF-Flat retrieval QPS", "value": qps, "unit": "queries/s", "ms_per_step": el / args.steps * 1e3,
        "config": {"workload": f"configs[3]: IVF-Flat nlist={nlist} nprobe={nprobe}, {args.ivf_nb}x{d}, "
                               f"batch={nq}, k={k}, L2", "parallelism": f"list-shard{world} + RCCL all_gather merge"
                   if world > 1 else "single GPU", "kmeans_niter": args.ivf_niter},
        "build_s": build_s,
        "stages_ms": {"prepare+phaseA+grouping": float(st[0]), "collect_screen": float(st[1]),
                      "exact_rescore": float(st[2]), "fallback": float(st[3])},
        "fallback_queries": int(index.local.last_fallback.item()),
        "exact_scan_queries": int(index.local.last_exact_scan.item()),
        "roofline": {"bound": "mfma", "kernel": "screen16_collect_kernel<128, 2, 4, 64, true, 3> (IVF collect, bf16 v_mfma_f32_16x16x32)",
                     "achieved": achieved, "peak": BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / BF16_DENSE_TFLOPS,
                     "traffic": _pmc_traffic(f"ivf:nb={args.ivf_nb},d={d},nq={nq},k={k},nlist={nlist},"
                                             f"nprobe={nprobe},gpus={world}"),
                     "algorithmic": f"2*d*sum(probed local list sizes) = {flops:.4g} flop per launch"},
    }
    # recall@5 against the exact flat search over the whole corpus (our flat
    # path is bit-exact vs the oracle, tests/test_knn_gpu.py)
    if rank == 0:
        flat = nf.IndexFlat(d, nf.METRIC_L2, device=dev)
        flat.add(xb)
        _, If = flat.search_device(xq, k)
        Ig, Ie = I.cpu().numpy(), If.cpu().numpy()
        out["recall_at_5"] = float(np.mean([len(set(a[:5]) & set(b[:5])) / min(5, k) for a, b in zip(Ig, Ie)]))
        if not args.no_flat_l2:
            out["flat_l2_10m"] = _flat_l2_leg(args, flat, xq, k)
        del flat
        if world == 1:
            out["oracle_match"] = _ivf_oracle_check(index, xb, xq, I, k, nprobe)
            if not args.no_cpu_baseline:
                out["cpu_baseline"] = _cpu_ivf(args, index, xb, xq, k, nprobe)
    return out


def _flat_l2_leg(args, flat, xq, k):
    """IndexFlatL2 over the same 10M x 128 corpus (exact flat L2, single GPU):
    QPS, stage split and the number of queries the L2 certificate could not
    cover (they take the fp64 fallback scan)."""
    from newsrecommend_amd import _lib

    for _ in range(2):
        flat.search_device(xq, k)
    torch.cuda.synchronize()
    steps = max(3, min(args.steps, 10))
    evs = [_lib.StageEvents() for _ in range(steps)]
    t0 = time.perf_counter()
    for e in evs:
        flat.search_device(xq, k, stage_events=e)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st = np.array([e.elapsed_ms() for e in evs]).mean(0)
    return {"metric": "IndexFlatL2 QPS", "value": xq.shape[0] * steps / el, "unit": "queries/s",
            "ms_per_step": el / steps * 1e3, "config": f"flat L2 {flat.ntotal}x{flat.d}, batch={xq.shape[0]}, k={k}",
            "stages_ms": {"query_prepare+tau_prepass": float(st[0]), "screen": float(st[1]),
                          "merge_rescore": float(st[2]), "exact_fallback": float(st[3])},
            "fallback_queries": int(flat.last_fallback.item()),
            "exact_scan_queries": int(flat.last_exact_scan.item())}


def _ivf_oracle_check(index, xb, xq, I, k, nprobe):
    """A few queries against oracle/ivf_oracle.py on the full corpus."""
    from oracle import ivf_oracle as io

    sample = np.arange(0, xq.shape[0], xq.shape[0] // 4)
    cent = index.quantizer._xb[: index.local.nlist].cpu().numpy()
    assign = index.local._assign.cpu().numpy()
    _, Io, _, _ = io.ivf_search(xq[sample].cpu().numpy(), xb.cpu().numpy(), cent, assign, nprobe, k, 1)
    return bool(np.array_equal(I[sample].cpu().numpy(), Io))


def _cpu_ivf(args, index, xb, xq, k, nprobe):
    """faiss-cpu IndexIVFFlat.search restated on all host cores
    (oracle/cpu_baselines.ivf_search: coarse sgemm top-nprobe, then each
    probed list scanned in place from a list-major copy, batched per list),
    on a bounded query sample."""
    from oracle import cpu_baselines as cb

    cores = cpu_cores()
    torch.set_num_threads(cores)
    lists = cb.IvfLists(xb.cpu().numpy(), index.local._assign.cpu().numpy(),
                        index.quantizer._xb[: index.local.nlist].cpu().numpy())
    q = xq.cpu()
    n, dt = _timed_sample(lambda n: cb.ivf_search(q[:n], lists, nprobe, k, 1), q.shape[0], 64, args.cpu_seconds)
    return {"value": n / dt, "unit": "queries/s", "cores": cores, "kind": "port",
            "sample": f"{n} of the {q.shape[0]} queries (nprobe={nprobe}) over the {xb.shape[0]}x{xb.shape[1]} IVF "
                      f"index, oracle.cpu_baselines.ivf_search (faiss IndexIVFFlat restated: in-place list scans, "
                      f"torch-CPU sgemm per list, {cores} threads), {dt:.1f} s"}


# -------------------------------------------------- N1 (north_star) --
def bench_n1(args, rank, world, dev, index, xb):
    """north_star's target workload: exact flat IP retrieval, k = 5, over the
    10M x 256 corpus (configs[4]'s corpus, sharded over the ranks), 4096-query
    batches from the same mixture.  One step = one batch.  Recall@5 and exact
    match on a query sample vs the oracle; cpu_baseline = the faiss-cpu
    IndexFlatIP port on all host cores over a bounded query sample."""
    from newsrecommend_amd import _lib
    from newsrecommend_amd.data import clustered_corpus

    n, d, k = xb.shape[0], xb.shape[1], 5
    nq = args.nq * world  # global batch: args.nq queries per GPU (weak scaling)
    xq = clustered_corpus(nq, d, seed=4321, device=dev)
    for _ in range(args.warmup):
        index.search_device(xq, k)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        D, I = index.search_device(xq, k)
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    evs = [_lib.StageEvents() for _ in range(min(args.steps, 10))]
    for e in evs:
        index.local.search_device(xq, k, id_offset=index.offset, stage_events=e)
    torch.cuda.synchronize()
    st = np.array([e.elapsed_ms() for e in evs]).mean(0)
    flops = 2.0 * nq * index.local.ntotal * d
    achieved = flops / (st[1] * 1e-3) / 1e12
    out = {
        "metric": "retrieval QPS @ recall@5 (north_star target: 10M x 256, k = 5)", "value": nq * args.steps / el,
        "unit": "queries/s", "ms_per_step": el / args.steps * 1e3,
        "config": {"workload": f"north_star: flat IP {n}x{d}, batch={nq}, k={k}",
                   "parallelism": f"corpus-shard{world} + all_gather merge" if world > 1 else "single GPU"},
        "stages_ms": {"query_prepare+tau_prepass": float(st[0]), "screen": float(st[1]),
                      "merge_rescore": float(st[2]), "exact_fallback": float(st[3])},
        "fallback_queries": int(index.local.last_fallback.item()),
        "exact_scan_queries": int(index.local.last_exact_scan.item()),
        "roofline": {"bound": "mfma", "kernel": _screen_kernel_name(nq, index.local.ntotal, d, k, 0),
                     "achieved": achieved, "peak": BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / BF16_DENSE_TFLOPS,
                     "traffic": _pmc_traffic(f"n1:nb={n},d={d},nq={nq},k={k},metric=ip,gpus={world}"),
                     "algorithmic": f"2*nq*nb_local*d = {flops:.4g} flop per launch"},
    }
    if rank == 0:
        from oracle import knn_oracle as ko

        xb_host = xb.cpu().numpy()
        sample = np.arange(0, nq, nq // 16)
        _, Io, _ = ko.exact_search(xq[sample].cpu().numpy(), xb_host, k, 0)
        Ig = I[sample].cpu().numpy()
        out["recall_at_5"] = float(np.mean([len(set(a) & set(b)) / k for a, b in zip(Ig, Io)]))
        out["exact_match_sample"] = bool(np.array_equal(Ig, Io))
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = _cpu_flat(args, xq, xb_host, 0, k=k)
        del xb_host
    return out


# ------------------------------------------------------------------ E2E --
def bench_e2e(args, rank, world, dev):
    """configs[4]: flat top-200 retrieval over 10M x 256 items (corpus rows
    sharded, exact per-shard lists merged after one all_gather) for a batch of
    user profiles, ground truth appended when missing (finialize_retrieval.py),
    then DIN re-rank of the 201 candidates of this rank's share of the users
    (users sharded: replicas) and NDCG@5.  One step = one batch of
    --e2e-users users end to end."""
    from newsrecommend_amd.data import clustered_corpus, zipf_ids
    from newsrecommend_amd.din import DIN
    from newsrecommend_amd.dist import ShardedIndexFlat, shard_range
    from newsrecommend_amd.pipeline import ndcg_at_k, rerank

    n, d, L, kr = args.e2e_nb, 256, 50, args.e2e_k
    U = args.e2e_users * world  # global batch of users: e2e_users per GPU (weak scaling)
    xb = clustered_corpus(n, d, seed=1234, device=dev)
    index = ShardedIndexFlat(d, 0, device=dev)
    index.add_full(xb)
    table = xb  # the DIN item table: the same fp32 embeddings (embedding_generate.py:119-122), on every rank
    n1 = bench_n1(args, rank, world, dev, index, xb) if not args.no_n1 else None
    del xb
    torch.cuda.empty_cache()
    g = torch.Generator(device=dev).manual_seed(11)
    hist = zipf_ids(U * L, n, generator=g, device=dev).view(U, L).to(torch.int32)
    lens = torch.randint(1, L + 1, (U,), generator=g, device=dev)
    hist = torch.where(torch.arange(L, device=dev)[None] < lens[:, None], hist, torch.full_like(hist, -1))
    valid = (hist >= 0).unsqueeze(-1)
    profiles = (table[hist.clamp_min(0).long()].float() * valid).sum(1) / valid.sum(1)
    gt = zipf_ids(U, n, generator=g, device=dev).to(torch.int32)
    torch.manual_seed(42)
    model = DIN(d, 128, 32, 0.36).to(dev).eval()
    ulo, uhi = shard_range(U, rank, world)

    def step():
        _, I = index.search_device_own(profiles, kr)  # this rank's users' candidates (one all_to_all)
        cand = I.to(torch.int32)
        g_ = gt[ulo:uhi]
        hit = (cand == g_[:, None]).any(1)
        cand = torch.cat([cand, torch.where(hit, torch.full_like(g_, -1), g_)[:, None]], 1)
        logits = rerank(model, table, hist[ulo:uhi], cand)
        labels = (cand == g_[:, None]) & (cand >= 0)
        return cand, logits, ndcg_at_k(logits, labels, 5)

    for _ in range(args.warmup):
        step()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        cand, logits, nd = step()
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    # stage split (rank-local, outside the timed region)
    from newsrecommend_amd.din import KernelTimer

    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(3):
        index.search_device_own(profiles, kr)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    with KernelTimer() as kt:
        for _ in range(3):
            rerank(model, table, hist[ulo:uhi], cand)
        torch.cuda.synchronize()
    t3 = time.perf_counter()
    rr = _rerank_roofline(kt.mean_ms("rerank"), kt.mean_ms("rerank_project"), hist[ulo:uhi], d, 128, 32, L,
                          f"rerank:e2e,users={uhi - ulo},C={kr + 1},d={d},gpus={world}", table.element_size(),
                          n_samples=float(cand.shape[0] * cand.shape[1]), proj_rows=cand.numel())
    # the dominant kernel (the top-200 screen, ~95 % of the step): the local search's
    # stages with HIP events on the library's launch stream
    from newsrecommend_amd import _lib

    evs = [_lib.StageEvents() for _ in range(3)]
    for e in evs:
        index.local.search_device(profiles, kr, exact_scores=True, id_offset=index.offset, stage_events=e)
    torch.cuda.synchronize()
    st = np.array([e.elapsed_ms() for e in evs]).mean(0)
    nb_local = index.local.ntotal
    flops = 2.0 * U * nb_local * d
    achieved = flops / (st[1] * 1e-3) / 1e12
    out = {
        "metric": "end-to-end users/s (retrieve top-200 + DIN re-rank + NDCG@5)", "value": U * args.steps / el,
        "unit": "users/s", "ms_per_step": el / args.steps * 1e3,
        "config": {"workload": f"configs[4]: {n}x{d} flat IP top-{kr} -> DIN re-rank (d={d}, A=128, F=32, L={L}), "
                               f"{U} users per step",
                   "parallelism": (f"corpus-shard{world} retrieval, RCCL all_to_all of each user slice's lists, "
                                   f"user-shard{world} re-rank") if world > 1 else "single GPU"},
        "stages_ms": {"retrieve": (t2 - t1) / 3 * 1e3, "rerank": (t3 - t2) / 3 * 1e3},
        "retrieve_stages_ms": {"query_prepare+tau_prepass": float(st[0]), "screen": float(st[1]),
                               "merge_rescore": float(st[2]), "exact_fallback": float(st[3])},
        "roofline": {"bound": "mfma", "kernel": _screen_kernel_name(U, nb_local, d, kr, 0),
                     "achieved": achieved, "peak": BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / BF16_DENSE_TFLOPS,
                     "traffic": _pmc_traffic(f"e2e:nb={n},d={d},nq={U},k={kr},metric=ip,gpus={world}"),
                     "algorithmic": f"2*users*nb_local*d = {flops:.4g} flop per launch (the top-{kr} screen, "
                                    f"{st[1]:.3f} ms HIP events)"},
        "rerank_samples_per_step": int((uhi - ulo) * (kr + 1)),
        "rerank_kernel_ms": kt.mean_ms("rerank"), "rerank_project_ms": kt.mean_ms("rerank_project"),
        "rerank_path": __import__("newsrecommend_amd.pipeline", fromlist=["rerank"]).rerank.path,
        "rerank_roofline": rr["hbm"], "rerank_valu": rr["valu"], "rerank_project_roofline": rr["proj"],
        "table_dtype": str(table.dtype).replace("torch.", ""),
        "ndcg_at_5_mean_rank0": float(nd.mean().item()),
        "fallback_queries": int(index.local.last_fallback.item()),
        "exact_scan_queries": int(index.local.last_exact_scan.item()),
    }
    if n1 is not None:
        out["n1_retrieval_10m_256_k5"] = n1
    if rank == 0:
        # re-rank parity on a few users: the reference's per-user forward
        # (DIN.py:168-173: model(cand, his.expand(C, -1, -1))) on the same rows
        errs = []
        with torch.no_grad():
            for u in range(0, uhi - ulo, max(1, (uhi - ulo) // 4)):
                c = cand[u][cand[u] >= 0].long()
                h = hist[ulo + u]
                keys = torch.where(h[None, :, None] >= 0, table[h.clamp_min(0).long()][None].float(), 0.0)
                ref = model(table[c].float(), keys.expand(len(c), -1, -1)).view(-1)
                errs.append(float((logits[u][cand[u] >= 0] - ref).abs().max()))
        out["rerank_vs_per_user_forward_max_abs"] = max(errs)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = _cpu_e2e(args, profiles, table, hist, gt, model, kr)
    del index, table
    torch.cuda.empty_cache()
    return out


def _cpu_torch_din(model, d, A, F):
    """oracle/din_torch_ref.TorchDIN (the reference's module restated in torch)
    holding `model`'s weights, eval mode, on the CPU."""
    from oracle.din_torch_ref import TorchDIN

    m = TorchDIN(d, A, F, 0.0).eval()
    m.load_state_dict({k: v.detach().float().cpu() for k, v in model.state_dict().items()})
    return m


def _cpu_rerank_user(m, xb, h, cand, chunk=1024):
    """DIN.py:166-173 for one user on the CPU: model(cand_emb, his.expand(C, -1, -1)),
    zero rows for padded history slots, candidates in chunks."""
    keys = torch.where(h[:, None] >= 0, xb[h.clamp_min(0)], 0.0)
    out = []
    for c0 in range(0, cand.shape[0], chunk):
        c = cand[c0:c0 + chunk]
        out.append(m(xb[c], keys[None].expand(c.shape[0], -1, -1)).view(-1))
    return torch.cat(out)


def _cpu_e2e(args, profiles, table, hist, gt, model, kr):
    """configs[4] end to end on the host cores over a bounded user sample:
    faiss-cpu's flat IP top-200 (oracle/cpu_baselines.flat_search) over the FULL
    corpus, the ground truth appended when missing, the reference's per-user
    DIN forward (TorchDIN) over the 200-201 candidates and NDCG@5."""
    from oracle import cpu_baselines as cb

    cores = cpu_cores()
    torch.set_num_threads(cores)
    xb = table.float().cpu()
    q, h, g = profiles.float().cpu(), hist.long().cpu(), gt.long().cpu()
    m = _cpu_torch_din(model, xb.shape[1], 128, 32)

    def run(n):
        _, I = cb.flat_search(q[:n], xb, kr, 0)
        with torch.no_grad():
            for u in range(n):
                c = I[u]
                if not bool((c == g[u]).any()):
                    c = torch.cat([c, g[u:u + 1]])
                lg = _cpu_rerank_user(m, xb, h[u], c)
                top = torch.topk(lg, 5).indices
                hit = (c[top] == g[u]).double()
                float((hit / torch.log2(torch.arange(2, 7, dtype=torch.float64))).sum())

    n, dt = _timed_sample(run, q.shape[0], 16, args.cpu_seconds, align=16)
    return {"value": n / dt, "unit": "users/s", "cores": cores, "kind": "port",
            "sample": f"{n} of the {q.shape[0]} users: flat IP top-{kr} over the full {xb.shape[0]}x{xb.shape[1]} "
                      f"corpus (oracle.cpu_baselines.flat_search), GT appended, the reference's per-user DIN "
                      f"forward (oracle.din_torch_ref, PyTorch-CPU fp32) and NDCG@5, {cores} threads, {dt:.1f} s"}


def _rerank_roofline(ms, ms_proj, hist, d, A, F, L, key, es, n_samples, proj_rows):
    """Rooflines of the re-rank (nrk_din_rerank_project(_hist) +
    nrk_din_rerank_projected), ALGORITHMIC bytes:
      main kernel: per scored candidate its projection [U' | Q1] (4 (A + F) B),
        id and logit (8 B); per user its L ids and the projections of its nv
        valid history rows;
      projections: per projected candidate row its table row (es * d B), id
        and projection out; per history slot its id and projection out, plus
        the nv valid rows;
    VALU work of the main kernel = 2 lane-ops (add, |.|-fma) per (candidate,
    scored row, attention unit), scored rows = nv + 1 padding row when nv < L,
    against the 78.6 T lane-op/s of the fp32 vector peak (157.3 TFLOP/s
    counting an fma as 2).  es: table element size (4: the reference's f32)."""
    nv = (hist >= 0).sum(1).double()
    nr = nv + (nv < L).double()
    U = hist.shape[0]
    ops = n_samples * float(nr.mean()) * A * 2
    pw = 4 * (A + F)
    byt = n_samples * (pw + 8) + float((4 * L + pw * nv).sum())
    byt_p = proj_rows * (es * d + 4 + pw) + U * L * (4 + pw) + float(nv.sum()) * es * d
    kern = f"din_rerank_lane_kernel<{A}, {F}> (projected)" if F <= 64 else f"din_rerank_kernel<.., {A}, {F}, PROJ> (projected)"
    sec = ms * 1e-3
    gbs = byt / sec / 1e9
    gbs_p = byt_p / (ms_proj * 1e-3) / 1e9 if ms_proj > 0 else 0.0
    return {"hbm": {"bound": "hbm", "binding": "valu (the scoring; see valu)", "kernel": kern, "achieved": gbs,
                    "peak": HBM_GBS, "unit": "GB/s", "frac": gbs / HBM_GBS, "traffic": _pmc_traffic(key),
                    "algorithmic": f"{byt:.4g} B per launch ({pw + 8} B per candidate + the users' ids and history "
                                   f"projections), {ms:.3f} ms (HIP events, the main kernel alone)"},
            "valu": {"achieved": ops / sec / 1e12, "peak": 78.6, "unit": "T lane-ops/s",
                     "frac": ops / sec / 1e12 / 78.6,
                     "algorithmic": f"{ops:.4g} lane-ops (2 per candidate x scored row x unit)"},
            "proj": {"bound": "hbm", "kernel": f"din_rerank_project_kernel<{d}, {es == 4}> (candidates + history)",
                     "achieved": gbs_p, "peak": HBM_GBS, "unit": "GB/s", "frac": gbs_p / HBM_GBS,
                     "algorithmic": f"{byt_p:.4g} B ({proj_rows} candidate rows + {U * L} history slots: "
                                    f"{es * d} B row in, {pw} B out), {ms_proj:.3f} ms (HIP events)"}}


def bench_retrieval_flow(args, rank, world, dev):
    """Retrieval.py:1-36 -> finialize_retrieval.py -> DIN.py:155-193 at the
    reference's own sizes: 364,047 x 256 article embeddings (synthetic mixture),
    faiss Clustering(256, 300) with niter 80 and an IndexHNSWFlat(256, 32)
    assignment index, index.search(xb, 1) -> cluster lists, 50,000 user
    profiles -> nearest centroid (one IndexFlatL2 search) -> the WHOLE cluster
    as candidates (ground truth appended when missing) -> DIN(256, 128, 32)
    re-rank with max_history 64 -> per-user BCE + NDCG@5.  Users are split
    over the ranks (replicas).  value = users/s of the candidate + re-rank +
    NDCG stage (the reference's evaluate() loop); build_s = k-means + assignment."""
    from newsrecommend_amd import faiss as nf
    from newsrecommend_amd.data import clustered_corpus, zipf_ids
    from newsrecommend_amd.din import DIN
    from newsrecommend_amd.dist import shard_range
    from newsrecommend_amd.pipeline import rerank_clusters

    n, d, nlist, L = 364_047, 256, 300, 64
    U = args.flow_users
    xb = clustered_corpus(n, d, seed=1234, device=dev)
    table = xb  # the reference's fp32 article embeddings (embedding_generate.py:119-122)
    barrier(world)
    t0 = time.perf_counter()
    clustering = nf.Clustering(d, nlist)
    clustering.niter = 80
    index = nf.IndexHNSWFlat(d, 32, device=dev)
    clustering.train(xb, index)
    centroids = clustering.centroids.reshape(nlist, d)
    _, assign = index.search_device(xb, 1)  # Retrieval.py:21
    assign = assign[:, 0]
    cluster_rows = torch.sort(assign, stable=True).indices.to(torch.int32)  # corpus row order inside a cluster
    cluster_off = torch.zeros(nlist + 1, dtype=torch.int64, device=dev)
    cluster_off[1:] = torch.cumsum(torch.bincount(assign, minlength=nlist), 0)
    centroid_index = nf.IndexFlatL2(d, device=dev)
    centroid_index.add(centroids)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    g = torch.Generator(device=dev).manual_seed(21)
    hist = zipf_ids(U * L, n, generator=g, device=dev).view(U, L)
    lens = torch.randint(1, L + 1, (U,), generator=g, device=dev)
    hist = torch.where(torch.arange(L, device=dev)[None] < lens[:, None], hist, torch.full_like(hist, -1))
    valid = (hist >= 0).unsqueeze(-1)
    profiles = (xb[hist.clamp_min(0).long()] * valid).sum(1) / valid.sum(1)  # mean of the clicked embeddings
    last = zipf_ids(U, n, generator=g, device=dev)
    lo, hi = shard_range(U, rank, world)
    torch.manual_seed(42)
    model = DIN(d, 128, 32, 0.36).to(dev).eval()

    def stage():
        _, I = centroid_index.search_device(profiles[lo:hi], 1)  # Retrieval.py:28-34 as one search
        return rerank_clusters(model, table, hist[lo:hi], I[:, 0], cluster_off, cluster_rows, last[lo:hi], k=5,
                               batch_samples=1 << 21, append_missing=True)

    res = stage()  # warm-up
    barrier(world)
    t0 = time.perf_counter()
    res = stage()
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    from newsrecommend_amd.din import KernelTimer

    with KernelTimer() as kt:  # the re-rank kernels, outside the timed region
        stage()
        torch.cuda.synchronize()
    sizes = torch.diff(cluster_off)
    _, Iu = centroid_index.search_device(profiles[lo:hi], 1)
    cand_per_user = sizes[Iu[:, 0]].double()
    out = {"metric": "Retrieval.py -> evaluate() users/s (whole-cluster candidates)", "value": U / el,
           "unit": "users/s", "ms": el * 1e3, "build_s": build_s,
           "config": f"{n}x{d} corpus, Clustering(k={nlist}, niter=80) + IndexHNSWFlat(M=32) assignment, {U} users, "
                     f"whole nearest cluster + GT appended, DIN(256, 128, 32), L={L}, {table.dtype} table",
           "cluster_size_min_mean_max": [int(sizes.min()), float(sizes.double().mean()), int(sizes.max())],
           "candidates_per_user_mean": float(cand_per_user.mean()),
           "rerank_samples_per_s": float(cand_per_user.sum()) * world / el,
           "rerank_kernel_ms": kt.mean_ms("rerank"), "rerank_project_ms": kt.mean_ms("rerank_project"),
           "table_dtype": str(table.dtype).replace("torch.", ""),
           **{k_: v_ for k_, v_ in zip(("rerank_roofline", "rerank_valu", "rerank_project_roofline"), _rerank_roofline(
               kt.mean_ms("rerank"), kt.mean_ms("rerank_project"), hist[lo:hi], d, 128, 32, L,
               f"rerank:flow,users={hi - lo},gpus={world}", table.element_size(),
               n_samples=float(cand_per_user.sum()) + (hi - lo), proj_rows=int(xb.shape[0]) + (hi - lo)).values())},
           "rerank_path": __import__("newsrecommend_amd.pipeline", fromlist=["rerank"]).rerank.path,
           "ndcg_at_5_mean_rank0": float(res["ndcg"].mean()), "loss_mean_rank0": float(res["loss"].mean())}
    out["roofline"] = dict(out["rerank_roofline"])  # the dominant kernel (the re-rank, ~99 % of the stage)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = _cpu_flow(args, xb, centroids, cluster_off, cluster_rows, profiles, hist, last, model)
    del xb, table, index, centroid_index
    torch.cuda.empty_cache()
    return out


def _cpu_flow(args, xb, centroids, cluster_off, cluster_rows, profiles, hist, last, model):
    """The Retrieval.py -> evaluate() stage on the host cores over a bounded user
    sample: nearest centroid (flat L2), the whole cluster as candidates with the
    ground truth appended when missing, the reference's per-user DIN forward
    (TorchDIN, chunks of 1024 candidates), per-user BCE and NDCG@5."""
    from oracle import cpu_baselines as cb

    cores = cpu_cores()
    torch.set_num_threads(cores)
    x, cen = xb.float().cpu(), centroids.float().cpu()
    off, rows = cluster_off.cpu(), cluster_rows.long().cpu()
    q, h, g = profiles.float().cpu(), hist.long().cpu(), last.long().cpu()
    m = _cpu_torch_din(model, x.shape[1], 128, 32)

    def run(n):
        _, I = cb.flat_search(q[:n], cen, 1, 1)
        with torch.no_grad():
            for u in range(n):
                cl = int(I[u, 0])
                c = rows[int(off[cl]):int(off[cl + 1])]
                lab = (c == g[u]).float()
                if not bool(lab.any()):
                    c = torch.cat([c, g[u:u + 1]])
                    lab = torch.cat([lab, torch.ones(1)])
                lg = _cpu_rerank_user(m, x, h[u], c)
                float(torch.nn.functional.binary_cross_entropy_with_logits(lg, lab))
                top = torch.topk(lg, min(5, lg.shape[0])).indices
                float((lab[top].double() / torch.log2(torch.arange(2, 2 + top.shape[0], dtype=torch.float64))).sum())

    n, dt = _timed_sample(run, q.shape[0], 4, args.cpu_seconds, align=4)
    return {"value": n / dt, "unit": "users/s", "cores": cores, "kind": "port",
            "sample": f"{n} of the {q.shape[0]} users: nearest of {cen.shape[0]} centroids, the whole cluster "
                      f"(+ GT) through the reference's per-user DIN forward (oracle.din_torch_ref, PyTorch-CPU "
                      f"fp32, 1024-candidate chunks), BCE and NDCG@5, {cores} threads, {dt:.1f} s"}


# ------------------------------------------------------------- embedding --
FP32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense fp32 MFMA (no TF32 on gfx950)


def bench_embed(args, rank, world, dev):
    """The corpus producer (embedding_generate.py:109-131):
    ArticleEmbeddingModel in eval mode over N x 253 article features ->
    N x 256 embeddings (fp32, as the reference), inputs resident in HBM.
    Sizes: the reference's 364,047 articles and configs[4]'s 10M corpus, each
    shard of N / world rows on its rank (replicas: no collective).  One
    nrk_embed launch per pass (embed_mlp_kernel: both layers, h on chip).
    Roofline: 2 (253 * 512 + 512 * 256) fp32 flop per row against the fp32
    MFMA peak (the products are fp32-exact), and the bf16 MFMA work the kernel
    issues for them, 6 x 2 (256 * 512 + 512 * 256) flop per row (three-plane
    split, six products), against the dense bf16 peak."""
    from newsrecommend_amd.embedding import ArticleEmbeddingModel

    torch.manual_seed(5)
    model = ArticleEmbeddingModel().to(dev).eval()
    with torch.no_grad():  # non-trivial BN statistics (folded into fc.4 by embed())
        bn = model.fc[3]
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 1.5)
    flop_row = 2.0 * (253 * 512 + 512 * 256)
    mfma_row = 6 * 2.0 * (256 * 512 + 512 * 256)
    out = {"metric": "article embeddings/s (corpus producer, fp32)", "unit": "rows/s",
           "kernel": "embed_mlp_kernel (nrk_embed)",
           "roofline_note": f"fp32 MFMA peak {FP32_MFMA_TFLOPS} TF; {flop_row:.0f} fp32 flop per row; "
                            f"{mfma_row:.0f} bf16 MFMA flop per row issued (6 products of 3-plane splits) vs "
                            f"{BF16_DENSE_TFLOPS} TF"}
    for name, n_total in (("reference_364047", 364_047), ("corpus_10m", args.e2e_nb)):
        n = -(-n_total // world)
        g = torch.Generator(device=dev).manual_seed(9 + rank)
        x = torch.randn((n, 253), generator=g, device=dev)
        for _ in range(2):
            model.embed(x)
        barrier(world)
        reps = 5 if n < 1_000_000 else 3
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()  # nrk_embed launches on torch's current stream
        for _ in range(reps):
            y = model.embed(x)
        e1.record()
        barrier(world)
        el = max_over_ranks(time.perf_counter() - t0, world, dev) / reps
        ev_ms = e0.elapsed_time(e1) / reps
        rec = {"value": n * world / el, "ms_per_pass": el * 1e3, "rows_per_gpu": n,
               "achieved_tflops": flop_row * n / el / 1e12,
               "frac_fp32_mfma": flop_row * n / el / 1e12 / FP32_MFMA_TFLOPS,
               "bf16_mfma_tflops": mfma_row * n / el / 1e12,
               "frac_bf16_mfma": mfma_row * n / el / 1e12 / BF16_DENSE_TFLOPS, "kernel_ms_hip_events": ev_ms}
        if rank == 0 and name == "reference_364047":
            # parity on a row sample: the reference's eval forward (fc as nn.Sequential, BN unfolded), fp32
            with torch.no_grad():
                ref = model(x[:4096])
            rec["max_abs_vs_module_forward"] = float((y[:4096] - ref).abs().max())
        out[name] = rec
        del x, y
        torch.cuda.empty_cache()
    out["value"] = out["corpus_10m"]["value"]
    c10 = out["corpus_10m"]
    tf_bf16 = mfma_row * c10["rows_per_gpu"] / (c10["kernel_ms_hip_events"] * 1e-3) / 1e12
    tf_f32 = flop_row * c10["rows_per_gpu"] / (c10["kernel_ms_hip_events"] * 1e-3) / 1e12
    out["roofline"] = {"bound": "mfma", "kernel": "embed_mlp_kernel (nrk_embed), 10M rows",
                       "achieved": tf_bf16, "peak": BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
                       "frac": tf_bf16 / BF16_DENSE_TFLOPS, "traffic": None,
                       "fp32_equivalent": {"achieved": tf_f32, "peak": FP32_MFMA_TFLOPS,
                                           "frac": tf_f32 / FP32_MFMA_TFLOPS},
                       "algorithmic": f"{mfma_row:.0f} bf16 MFMA flop per row issued (fp32-exact products as six "
                                      f"3-plane bf16 products; {flop_row:.0f} fp32 flop per row) x "
                                      f"{c10['rows_per_gpu']} rows, {c10['kernel_ms_hip_events']:.3f} ms (HIP events)"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cores = cpu_cores()
        torch.set_num_threads(cores)
        mc = ArticleEmbeddingModel().eval()
        mc.load_state_dict({k: v.cpu() for k, v in model.state_dict().items()})
        xc = torch.randn((65536, 253))

        def run(n):
            with torch.no_grad():
                for lo in range(0, n, 8192):
                    mc(xc[lo % 65536:lo % 65536 + 8192])

        n, dt = _timed_sample(run, 10**8, 8192, args.cpu_seconds / 2, align=8192)
        out["cpu_baseline"] = {"value": n / dt, "unit": "rows/s", "cores": cores, "kind": "port",
                               "sample": f"{n} rows in batches of 8192 through the reference's eval-mode module "
                                         f"(PyTorch-CPU fp32, {cores} threads; the reference itself runs batch-1 "
                                         f"forwards, embedding_generate.py:118-121), {dt:.1f} s"}
    return out


# ------------------------------------------------------------------ DIN --
DIN_STEPS_PER_GRAPH = 8  # fused steps per HIP-graph launch (one index copy + one launch per 8 steps)


def bench_din(args, rank, world, dev):
    from newsrecommend_amd.data import synthetic_click_rows
    from newsrecommend_amd.din import DIN, KernelTimer

    torch.manual_seed(42)
    n_items, L, d, A, F = args.din_items, 50, 128, 128, 32
    g = torch.Generator(device=dev).manual_seed(1)
    table = (torch.randn((n_items, d), generator=g, device=dev) * 0.5).to(torch.bfloat16)
    rows = args.din_rows
    hist, tgt, lab = synthetic_click_rows(rows, n_items, L, seed=7 + rank, device=dev)
    model = DIN(d, A, F, 0.36).to(dev)
    crit = torch.nn.BCEWithLogitsLoss()
    B = args.din_batch
    perm = torch.randperm(rows, device=dev)
    nbatch = rows // B
    fused = not args.din_eager
    # the data-parallel step is graphed too when the gradient all_reduce is RCCL
    # (captured inside the graph: tests/rccl_world1_worker.py); gloo
    # rehearsals carry host copies, which a graph cannot capture
    graphed = fused and (world == 1 or BACKEND == "nccl")
    opt = torch.optim.Adam(model.parameters(), lr=1.62e-3, weight_decay=8.96e-5)
    if fused:
        from newsrecommend_amd.din import FusedTrainStep

        from newsrecommend_amd.dist import all_reduce_mean_

        def allreduce(G):  # RCCL on the flat gradient buffer (gloo: a host copy)
            all_reduce_mean_(G)

        trainer = FusedTrainStep(model, table, hist, tgt, lab, B, lr=1.62e-3, weight_decay=8.96e-5, clip=1.0,
                                 graph=graphed, grad_hook=allreduce if world > 1 else None,
                                 steps_per_graph=DIN_STEPS_PER_GRAPH if graphed else 1)

    def run(s0, n):
        """steps s0 .. s0 + n - 1: K-step graph launches where K consecutive batches are contiguous in perm"""
        s, loss = s0, None
        while s < s0 + n:
            K = trainer.K if fused else 1
            if K > 1 and s + K <= s0 + n and s % nbatch + K <= nbatch:
                b = s % nbatch
                loss = trainer.step_many(perm[b * B:(b + K) * B].view(K, B))[-1]
                s += K
            else:
                loss = step(s)
                s += 1
        return loss

    def step(s):
        idx = perm[(s % nbatch) * B:(s % nbatch + 1) * B]
        if fused:
            return trainer.step(idx)
        logits = model.forward_ids(table, tgt[idx], hist[idx])
        loss = crit(logits, lab[idx])
        opt.zero_grad(set_to_none=True)
        loss.backward()
        if world > 1:
            from newsrecommend_amd.dist import all_reduce_mean_

            flat = all_reduce_mean_(torch.cat([p.grad.reshape(-1) for p in model.parameters()]))
            o = 0
            for p in model.parameters():
                n = p.numel()
                p.grad.copy_(flat[o:o + n].view_as(p))
                o += n
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        return loss

    # a training epoch is thousands of steps: time at least 20 K-step graph
    # launches (160 steps, ~30 ms) so the fixed launch/sync cost of a 20-step
    # window does not masquerade as per-step time; warmup rounded to K so the
    # timed steps are whole K-step launches
    K = trainer.K if fused else 1
    n_steps = max(args.steps, 20 * K)
    n_warm = -(-max(args.warmup, 1) // K) * K
    model.train()
    run(0, n_warm)
    barrier(world)
    t0 = time.perf_counter()
    loss = run(n_warm, n_steps)
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    # attention kernel times: a few extra steps of the same path, outside the
    # graph, with HIP events on the launch stream around the two attention calls
    with KernelTimer() as kt:
        for s in range(4):
            if fused:
                trainer.idx.copy_(perm[s * B:(s + 1) * B])
                trainer._body()
            else:
                lg = model.forward_ids(table, tgt[perm[:B]], hist[perm[:B]])
                crit(lg, lab[perm[:B]]).backward()
        torch.cuda.synchronize()
    sps = B * n_steps * world / el
    fwd_ms, bwd_ms = kt.mean_ms("fwd", skip=1), kt.mean_ms("bwd", skip=1)
    # algorithmic bytes per sample: history ids + bf16 key rows, the U row and
    # outputs (fwd: pooled, alpha); bwd adds dpooled, alpha, q and the dU row
    fwd_bytes = B * (4 * L + L * d * 2 + 4 * A + 4 * d + 4 * L)
    bwd_bytes = B * (4 * L + L * d * 2 + 4 * A + 4 * d + 4 * L + 4 * d + 2 * 4 * A)
    STEP_BYTES = L * d * 2 + d * 2 + 4 * (L + 1) + 4
    step_gbs = STEP_BYTES * B * n_steps / el / 1e9  # per GPU
    fwd_gbs = fwd_bytes / (fwd_ms * 1e-3) / 1e9
    bwd_gbs = bwd_bytes / (bwd_ms * 1e-3) / 1e9
    din_key = f"B={B},L={L},d={d},A={A},gpus={world}"  # profiles/pmc_screen.json (tools/din_pmc.sh)
    out = {
        "metric": "DIN train samples/s", "value": sps, "unit": "samples/s", "ms_per_step": el / n_steps * 1e3,
        "steps": n_steps, "warmup": n_warm,
        "config": {"workload": "configs[2]: DIN train bf16, 5M synthetic click rows, seq_len=50, emb_dim=128",
                   "rows": rows, "items": n_items, "batch": B, "attn_units": A, "fc_units": F,
                   "parallelism": f"dp{world}",
                   "step": ((f"fused head/optimizer kernels, one hip graph per {DIN_STEPS_PER_GRAPH} steps"
                             + (" (RCCL grad all_reduce captured in the graph)" if world > 1 else "")) if graphed else
                            "fused head/optimizer kernels + gloo grad all_reduce") if fused else "eager torch"},
        "final_loss": float(loss.reshape(-1)[0].item()),
        "kernels_ms": {"attn_fwd": fwd_ms, "attn_bwd (8-wave + reduce)" if fused else "attn_bwd+reduce": bwd_ms},
        "roofline_step": {"bound": "hbm", "achieved": step_gbs, "peak": HBM_GBS, "unit": "GB/s",
                          "frac": step_gbs / HBM_GBS,
                          "traffic": _pmc_traffic(f"din_step:{din_key}") if fused and graphed else None,
                          "algorithmic": f"{STEP_BYTES} B/sample (SURVEY.md 8d: L*d*2 + d*2 + 4*(L+1) + 4) x "
                                         f"samples/s over the whole step"},
        "roofline_fwd": {"bound": "hbm", "achieved": fwd_gbs, "peak": HBM_GBS, "unit": "GB/s",
                         "frac": fwd_gbs / HBM_GBS, "traffic": _pmc_traffic(f"din_fwd:{din_key}") if fused else None,
                         "algorithmic": f"{fwd_bytes // B} B/sample x {B} samples"},
        "roofline_bwd": {"bound": "hbm", "achieved": bwd_gbs, "peak": HBM_GBS, "unit": "GB/s",
                         "frac": bwd_gbs / HBM_GBS, "traffic": _pmc_traffic(f"din_bwd:{din_key}") if fused else None,
                         "algorithmic": f"{bwd_bytes // B} B/sample x {B} samples"},
    }
    # the dominant launch of the step: the attention backward (8-wave kernel + slab reduction)
    out["roofline"] = dict(out["roofline_bwd"], kernel=("din_bwd_deep8g_kernel<128, 64> + din_bwd_reduce_params_kernel"
                                                        if fused else "attention backward + reduction"))
    if fused and world == 1 and args.din_sweep:
        out["batch_sweep"] = {str(bs): _din_rate(table, hist, tgt, lab, d, A, F, bs, dev) for bs in (16384, 65536)}
    if fused and world == 1 and args.din_d256:
        out["d256"] = _din_d256(args, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = _cpu_din(args, n_items, L, d, A, F)
    return out


def _din_d256(args, dev):
    """The reference's own training shape (DIN.py:16 EMBED_DIM = 256 from the
    corpus of embedding_generate.py:14; main(): A 128, F 32, max_history 64,
    DIN.py:233-237) on the fused step: its batch 64 (DIN.py:236) and the
    bench's 4096, bf16 table of --din-items rows, synthetic click rows."""
    from newsrecommend_amd.data import synthetic_click_rows

    d, L, A, F = 256, 64, 128, 32
    g = torch.Generator(device=dev).manual_seed(2)
    table = (torch.randn((args.din_items, d), generator=g, device=dev) * 0.5).to(torch.bfloat16)
    hist, tgt, lab = synthetic_click_rows(1_000_000, args.din_items, L, seed=8, device=dev)
    out = {"config": f"d={d}, A={A}, F={F}, L={L}, dropout 0.36, bf16 table {args.din_items}x{d}"}
    for B in (64, 4096):
        path = []
        rate = _din_rate(table, hist, tgt, lab, d, A, F, B, dev, steps=200 if B == 64 else 40, path=path)
        out[f"B={B}"] = {"samples_per_s": rate, "us_per_step": B / rate * 1e6, "path": path[0]}
    # max_history 128, the top of the reference's Optuna range (DIN.py:207): two
    # half-samples per sample in the column-split backward
    hist, tgt, lab = synthetic_click_rows(1_000_000, args.din_items, 128, seed=8, device=dev)
    path = []
    rate = _din_rate(table, hist, tgt, lab, d, A, F, 4096, dev, steps=40, path=path)
    out["L=128,B=4096"] = {"samples_per_s": rate, "us_per_step": 4096 / rate * 1e6, "path": path[0]}
    del table, hist, tgt, lab
    torch.cuda.empty_cache()
    return out


def _din_rate(table, hist, tgt, lab, d, A, F, B, dev, steps=10, path=None):
    """samples/s of the graphed fused train step at batch B (fresh model)."""
    from newsrecommend_amd.din import DIN, FusedTrainStep

    torch.manual_seed(43)
    m = DIN(d, A, F, 0.36).to(dev)
    tr = FusedTrainStep(m, table, hist, tgt, lab, B, lr=1.62e-3, weight_decay=8.96e-5, clip=1.0)
    if path is not None:
        path.append(tr.path)
    perm = torch.randperm(hist.shape[0], device=dev)
    nb = hist.shape[0] // B
    for s in range(3):
        tr.step(perm[(s % nb) * B:(s % nb + 1) * B])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        tr.step(perm[(s % nb) * B:(s % nb + 1) * B])
    torch.cuda.synchronize()
    return B * steps / (time.perf_counter() - t0)


def _cpu_din(args, n_items, L, d, A, F, B=4096):
    """The reference's PyTorch-CPU fp32 train step (oracle/din_torch_ref,
    pinned to DIN.py's own train() by tests/test_oracle_din.py) on all host
    cores, batch B, including the history gather from a host table
    (TrainDataset.__getitem__, DIN.py:81-92), on a bounded number of steps."""
    from oracle.din_torch_ref import TorchDIN, train_step

    cores = cpu_cores()
    torch.set_num_threads(cores)
    g = torch.Generator().manual_seed(0)
    n_tab = min(n_items, 200_000)
    table = torch.randn((n_tab, d), generator=g) * 0.5
    torch.manual_seed(42)
    m = TorchDIN(d, A, F, 0.36).train()
    opt = torch.optim.Adam(m.parameters(), lr=1.62e-3, weight_decay=8.96e-5)
    crit = torch.nn.BCEWithLogitsLoss()

    def steps(n):
        for _ in range(n):
            ln = torch.randint(1, L + 1, (B, 1), generator=g)
            ids = torch.randint(0, n_tab, (B, L), generator=g)
            keys = table[ids] * (torch.arange(L)[None, :] < ln).unsqueeze(-1)
            q = table[torch.randint(0, n_tab, (B,), generator=g)]
            y = (torch.rand((B, 1), generator=g) < 0.5).float()
            train_step(m, opt, crit, q, keys, y)

    n, dt = _timed_sample(steps, 10**9, 2, args.cpu_seconds / 2, align=1)
    return {"value": n * B / dt, "unit": "samples/s", "cores": cores, "kind": "port",
            "sample": f"{n} train steps x {B} rows (L={L}, d={d}, A={A}, F={F}), oracle.din_torch_ref "
                      f"(the reference's DIN train step in PyTorch-CPU fp32, {cores} threads, gather included), "
                      f"{dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["flat", "din", "ivf", "e2e", "flow", "embed", "all"], default="all")
    ap.add_argument("--nb", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--nq", type=int, default=4096)
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--metric", choices=["ip", "l2"], default="ip")
    ap.add_argument("--ivf-nb", type=int, default=10_000_000)
    ap.add_argument("--ivf-nlist", type=int, default=300)
    ap.add_argument("--ivf-nprobe", type=int, default=32)
    ap.add_argument("--ivf-niter", type=int, default=20)
    ap.add_argument("--e2e-nb", type=int, default=10_000_000)
    ap.add_argument("--e2e-users", type=int, default=4096)
    ap.add_argument("--e2e-k", type=int, default=200)
    ap.add_argument("--flow-users", type=int, default=50_000, help="users of the Retrieval.py -> evaluate() record")
    ap.add_argument("--din-rows", type=int, default=5_000_000)
    ap.add_argument("--din-items", type=int, default=2_000_000)
    ap.add_argument("--din-batch", type=int, default=4096)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--din-eager", action="store_true", help="no HIP-graph capture of the DIN train step")
    ap.add_argument("--din-sweep", type=int, default=1, help="also report the fused step at B=16384, 65536")
    ap.add_argument("--din-d256", type=int, default=1, help="also report the fused step at d=256, L=64 (B=64, 4096)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-n1", action="store_true", help="skip the north_star 10M x 256 k=5 retrieval record")
    ap.add_argument("--no-flat-l2", action="store_true", help="skip the IndexFlatL2 10M x 128 record")
    ap.add_argument("--record-timeout", type=float, default=900.0, help="seconds per record process")
    ap.add_argument("--no-isolate", action="store_true",
                    help="run every record in this process (default: one child process per record)")
    ap.add_argument("--record", default=None, help=argparse.SUPPRESS)  # internal: the child's record
    ap.add_argument("--record-out", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.record:
        return child_main(args)
    if not args.no_isolate:
        return isolated_main(args)

    rank, world, dev = setup(args)
    rec = {"metric": METRIC, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
           "data": "synthetic"}
    if args.workload in ("flat", "all"):
        r = bench_flat(args, rank, world, dev)
        rec.update({k: r[k] for k in ("value", "unit", "ms_per_step")})
        rec["config"] = {"workload": f"configs[1]: flat kNN {args.nb}x{args.d}, batch={args.nq} queries per GPU, "
                                     f"k={args.k}, {args.metric.upper()}", "nb": args.nb, "d": args.d, "nq": args.nq,
                         "global_batch": args.nq * world, "k": args.k,
                         "metric": args.metric, "screen": "bf16 MFMA, fp32 accumulate", "rescore": "f64 exact",
                         "parallelism": f"corpus-shard{world} + RCCL all_gather merge" if world > 1 else "single GPU"}
        for k in ("roofline", "stages_ms", "fallback_queries", "recall_at_5", "exact_match", "cpu_baseline"):
            if k in r:
                rec[k] = r[k]
    if args.workload in ("ivf", "all"):
        r = bench_ivf(args, rank, world, dev)
        if args.workload == "ivf":
            rec.update({"metric": r["metric"], "value": r["value"], "unit": r["unit"], "ms_per_step": r["ms_per_step"],
                        "config": r["config"], "roofline": r["roofline"]})
            if "cpu_baseline" in r:
                rec["cpu_baseline"] = r["cpu_baseline"]
        rec["ivf"] = r
        torch.cuda.empty_cache()
    if args.workload in ("e2e", "flow", "all"):
        r = bench_retrieval_flow(args, rank, world, dev)
        if args.workload == "flow":
            rec.update({"metric": r["metric"], "value": r["value"], "unit": r["unit"], "ms_per_step": r["ms"]})
        rec["retrieval_py_flow"] = r
        torch.cuda.empty_cache()
    if args.workload in ("e2e", "all"):
        r = bench_e2e(args, rank, world, dev)
        if args.workload == "e2e":
            rec.update({"metric": r["metric"], "value": r["value"], "unit": r["unit"], "ms_per_step": r["ms_per_step"],
                        "config": r["config"]})
        rec["e2e"] = r
    if args.workload in ("embed", "all"):
        r = bench_embed(args, rank, world, dev)
        if args.workload == "embed":
            rec.update({"metric": r["metric"], "value": r["value"], "unit": r["unit"],
                        "ms_per_step": r["corpus_10m"]["ms_per_pass"]})
        rec["embed"] = r
        torch.cuda.empty_cache()
    if args.workload in ("din", "all"):
        r = bench_din(args, rank, world, dev)
        if args.workload == "din":
            rec.update({"metric": r["metric"], "value": r["value"], "unit": r["unit"], "ms_per_step": r["ms_per_step"],
                        "config": r["config"], "scaling": "weak", "roofline": r["roofline"]})
            if "cpu_baseline" in r:
                rec["cpu_baseline"] = r["cpu_baseline"]
        rec["din"] = r
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


# ------------------------------------------------------------- isolation --
# Each record runs in its own child process (the same script with --record),
# so a fault in one record's kernels (round 5: an illegal address inside the
# IVF searches took the whole line down) costs that record only: the parent
# merges what every child wrote and marks a failed record {"error": ...}.  The
# parent never touches the GPU (no HIP runtime state to fork from); at N > 1
# its ranks keep in step over a gloo group and each record's children form
# their own group (RCCL) on a port of their own.
RECORDS = ("flat", "ivf", "flow", "e2e", "embed", "din")


def _records_for(workload):
    return {"all": RECORDS, "e2e": ("flow", "e2e")}.get(workload, (workload,))


def run_record(name, args, rank, world, dev):
    if name == "flat":
        return bench_flat(args, rank, world, dev)
    return {"ivf": bench_ivf, "flow": bench_retrieval_flow, "e2e": bench_e2e, "embed": bench_embed,
            "din": bench_din}[name](args, rank, world, dev)


def child_main(args):
    rank, world, dev = setup(args)
    out = run_record(args.record, args, rank, world, dev)
    if rank == 0:
        with open(args.record_out, "w") as f:
            json.dump(out, f)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def isolated_main(args):
    import subprocess
    import tempfile

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        dist.init_process_group("gloo")
    base_port = int(os.environ.get("MASTER_PORT", "29500"))
    rec = {"metric": METRIC, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
           "data": "synthetic"}
    results = {}
    tmpdir = tempfile.mkdtemp(prefix="nrk_bench_")
    for i, name in enumerate(_records_for(args.workload)):
        if world > 1:
            dist.barrier()
        out = os.path.join(tmpdir, f"{name}.json")
        cmd = [sys.executable, "-u", os.path.abspath(__file__), *sys.argv[1:], "--record", name, "--record-out", out]
        env = dict(os.environ)
        if world > 1:  # the children's own rendezvous (rank 0's child serves the store)
            env["MASTER_PORT"] = str(base_port + 17 + i)
            env["TORCHELASTIC_USE_AGENT_STORE"] = "False"
        t0 = time.perf_counter()
        try:
            r = subprocess.run(cmd, env=env, timeout=args.record_timeout)
            rc = r.returncode
        except subprocess.TimeoutExpired:
            rc = "timeout"
        log(f"bench: record {name} rc={rc} ({time.perf_counter() - t0:.1f} s)")
        if rank == 0:
            try:
                with open(out) as f:
                    results[name] = json.load(f)
            except (OSError, ValueError):
                results[name] = {"error": f"record process exited with {rc} and wrote no result "
                                          f"(its stderr is above in the log)"}
    if rank == 0:
        r = results.get("flat")
        if r is not None and "error" not in r:
            rec.update({k: r[k] for k in ("value", "unit", "ms_per_step")})
            rec["config"] = {"workload": f"configs[1]: flat kNN {args.nb}x{args.d}, batch={args.nq} queries per GPU, "
                                         f"k={args.k}, {args.metric.upper()}", "nb": args.nb, "d": args.d,
                             "nq": args.nq, "global_batch": args.nq * world, "k": args.k, "metric": args.metric,
                             "screen": "bf16 MFMA, fp32 accumulate", "rescore": "f64 exact",
                             "parallelism": f"corpus-shard{world} + RCCL all_gather merge" if world > 1 else
                             "single GPU"}
            for k in ("roofline", "stages_ms", "fallback_queries", "recall_at_5", "exact_match", "cpu_baseline"):
                if k in r:
                    rec[k] = r[k]
        elif r is not None:
            rec["flat"] = r
        for name in ("ivf", "flow", "e2e", "embed", "din"):
            if name not in results:
                continue
            r = results[name]
            rec["retrieval_py_flow" if name == "flow" else name] = r
            if args.workload == name and "error" not in r:  # a single secondary record is the line's metric
                ms = r["corpus_10m"]["ms_per_pass"] if name == "embed" else r.get("ms_per_step", r.get("ms"))
                rec.update({"metric": r["metric"], "value": r["value"], "unit": r["unit"], "ms_per_step": ms})
                for k in ("config", "roofline", "cpu_baseline"):
                    if k in r:
                        rec[k] = r[k]
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
