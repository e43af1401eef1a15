"""faiss-compatible flat indexes on MI355X (drop-in for the subset of the faiss
Python API the reference's retrieval path uses).

Reference call sites (Retrieval.py):
  :12-18 clustering = faiss.Clustering(256, 300); .niter; .train(x, IndexHNSWFlat(256, 32))
  :21-23 _, assign = index.search(xb, 1); cluster_to_articles (IndexIVFFlat.list_ids)
  :25  centroid_index = faiss.IndexFlatL2(embeddings_size)
  :26  centroid_index.add(centroids)
  :31-32 _, I = centroid_index.search(profile, 1)
  :19  faiss.vector_float_to_array(clustering.centroids)
and the generalisations in BASELINE.json (IndexFlatIP, nq = 4096 batches).

Semantics (restated in oracle/knn_exact.c): exact search; IP = largest inner
product first, L2 = smallest SQUARED distance first; ties -> lower id; ids are
insertion order; k > ntotal pads I with -1 and D with -/+FLT_MAX.  Inputs are
converted like faiss's wrapper does (C-contiguous float32, shape (n, d));
numpy in -> numpy out.  Torch CUDA tensors are accepted too and stay on the
device (no host round trip).

Storage per index (HBM): xb f32 [N][d] for the exact rescoring, a bf16
[N][dp] screening copy, and per-row {||x||^2, bf16 residual norm}.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

METRIC_INNER_PRODUCT = _lib.NRK_METRIC_INNER_PRODUCT
METRIC_L2 = _lib.NRK_METRIC_L2


def vector_float_to_array(v) -> np.ndarray:
    """faiss.vector_float_to_array (Retrieval.py:19): a float32 numpy copy."""
    if isinstance(v, torch.Tensor):
        return v.detach().float().cpu().numpy().reshape(-1).copy()
    return np.asarray(v, dtype=np.float32).reshape(-1).copy()


def _default_device():
    if not torch.cuda.is_available():
        raise _lib.NrkError("newsrecommend_amd.faiss needs a GPU (HIP path, no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


class _FallbackCounters:
    """Diagnostics of the last search (include/nrk.h n_fallback), device views."""

    @property
    def last_fallback(self):
        """int32[1]: queries the main path did not answer (flat: not covered by
        the certificate, answered by the collect pass; IVF: collect overflow)."""
        return None if self.fallback_counts is None else self.fallback_counts[0:1]

    @property
    def last_exact_scan(self):
        """int32[1]: of those, queries answered by the fp64 corpus scan."""
        return None if self.fallback_counts is None else self.fallback_counts[1:2]


class IndexFlat(_FallbackCounters):
    """Exhaustive index (faiss.IndexFlat).  `metric` as faiss.MetricType."""

    def __init__(self, d: int, metric: int = METRIC_L2, device=None):
        if metric not in (METRIC_INNER_PRODUCT, METRIC_L2):
            raise ValueError(f"unsupported metric {metric}")
        self.d = int(d)
        self.metric_type = int(metric)
        self.is_trained = True
        self.device = torch.device(device) if device is not None else _default_device()
        self.dp = _lib.load().nrk_padded_dim(self.d)
        self._ws = None
        # device int32[2] (include/nrk.h n_fallback): [0] queries the certificate
        # did not cover, [1] of those, answered by the fp64 scan
        self.fallback_counts = None
        self.reset()

    # -------------------------------------------------------------- storage
    @property
    def ntotal(self) -> int:
        return int(self._n)

    def reset(self):
        self._n = 0
        self._cap = 0
        self._xb = torch.empty((0, self.d), dtype=torch.float32, device=self.device)
        self._xbh = torch.empty((0, self.dp), dtype=torch.int16, device=self.device)
        self._meta = torch.empty((0, 2), dtype=torch.float32, device=self.device)
        self._stats = torch.zeros(4, dtype=torch.float32, device=self.device)

    def _grow(self, need: int):
        if need <= self._cap:
            return
        cap = max(need, int(self._cap * 1.5) + 1024)
        for name, width, dt in (("_xb", self.d, torch.float32), ("_xbh", self.dp, torch.int16),
                                ("_meta", 2, torch.float32)):
            old = getattr(self, name)
            new = torch.empty((cap, width), dtype=dt, device=self.device)
            if self._n:
                new[: self._n].copy_(old[: self._n])
            setattr(self, name, new)
        self._cap = cap

    def _as_input(self, x):
        if isinstance(x, torch.Tensor):
            t = x.detach()
            if t.dim() != 2 or t.shape[1] != self.d:
                raise AssertionError(f"expected (n, {self.d}) input, got {tuple(t.shape)}")
            return t.to(device=self.device, dtype=torch.float32).contiguous(), False
        a = np.ascontiguousarray(x, dtype=np.float32)
        if a.ndim != 2 or a.shape[1] != self.d:
            raise AssertionError(f"expected (n, {self.d}) input, got {a.shape}")
        return torch.from_numpy(a).to(self.device, non_blocking=False), True

    def _as_query(self, xq) -> torch.Tensor:
        """Device-path query check: a GPU tensor on this index's device, (nq, d),
        converted to contiguous float32 (bf16/f16/f64 or strided views are
        converted, a host tensor or a wrong shape raises)."""
        if not isinstance(xq, torch.Tensor):
            raise TypeError("search_device takes a torch tensor on the GPU (use search() for numpy input)")
        _lib.require_device(xq, what="search_device")
        if xq.device != self.device:
            raise _lib.NrkError(f"search_device: queries on {xq.device}, index on {self.device}")
        if xq.dim() != 2 or xq.shape[1] != self.d:
            raise AssertionError(f"expected (n, {self.d}) queries, got {tuple(xq.shape)}")
        return xq.detach().to(torch.float32).contiguous()

    def add(self, x):
        """Append vectors (ids continue from ntotal), faiss Index.add."""
        xt, _ = self._as_input(x)
        n = xt.shape[0]
        if n == 0:
            return
        self._grow(self._n + n)
        lo, hi = self._n, self._n + n
        with torch.cuda.device(self.device):
            self._xb[lo:hi].copy_(xt)
            _lib.check(_lib.load().nrk_flat_prepare(
                _lib.ptr(self._xb[lo:hi]), n, self.d, _lib.ptr(self._xbh[lo:hi]), _lib.ptr(self._meta[lo:hi]),
                _lib.ptr(self._stats), _lib.stream(self.device)), "flat_prepare")
        self._n = hi

    def reconstruct(self, i: int) -> np.ndarray:
        return self._xb[int(i)].cpu().numpy().copy()

    # --------------------------------------------------------------- search
    def _workspace(self, nbytes: int):
        # zero-filled on growth: no slot of a fresh workspace holds garbage, even
        # one a kernel reads before writing (the search re-initialises what it uses)
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = torch.zeros(max(nbytes, 1), dtype=torch.uint8, device=self.device)
        return self._ws

    def _launch(self, xq: torch.Tensor, nq: int, k: int, D, I, S, id_offset: int = 0, stage_events=None):
        """nrk_knn_flat over device buffers (xq (nq, d) f32, D / I / S (nq, k)) on the device's stream."""
        L = _lib.load()
        if self.fallback_counts is None:
            self.fallback_counts = torch.zeros(2, dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            sz = _lib.c_size(0)
            _lib.check(L.nrk_knn_flat_workspace(nq, self._n, self.d, k, sz), "knn_flat_workspace")
            ws = self._workspace(sz.value)
            n = self._n
            _lib.check(L.nrk_knn_flat(
                _lib.ptr(xq), nq, _lib.ptr(self._xb[:n]) if n else None, _lib.ptr(self._xbh[:n]) if n else None,
                _lib.ptr(self._meta[:n]) if n else None, _lib.ptr(self._stats), n, self.d, k, self.metric_type,
                _lib.ptr(D), _lib.ptr(I), _lib.ptr(S), int(id_offset), _lib.ptr(self.fallback_counts), _lib.ptr(ws),
                ws.numel(), stage_events.ev if stage_events is not None else None, _lib.stream(self.device)),
                "knn_flat")

    def search_device(self, xq: torch.Tensor, k: int, exact_scores: bool = False, id_offset: int = 0,
                      stage_events=None):
        """Device-in, device-out search: returns (D f32, I int64[, S f64]) on the GPU."""
        k = int(k)
        if k <= 0:
            raise ValueError("k must be positive")
        xq = self._as_query(xq)
        nq = xq.shape[0]
        D = torch.empty((nq, k), dtype=torch.float32, device=self.device)
        I = torch.empty((nq, k), dtype=torch.int64, device=self.device)
        S = torch.empty((nq, k), dtype=torch.float64, device=self.device) if exact_scores else None
        self._launch(xq, nq, k, D, I, S, id_offset, stage_events)
        return (D, I, S) if exact_scores else (D, I)

    def _host_buffers(self, nq: int, k: int):
        """Persistent staging for numpy searches: pinned host query / result
        buffers and their device twins, grown to the largest call."""
        hb = getattr(self, "_hb", None)
        if hb is None or hb["nq"] < nq or hb["nqk"] < nq * k:
            cq = max(nq, hb["nq"] if hb else 0)
            ck = max(nq * k, hb["nqk"] if hb else 0)
            dev = self.device
            hb = {"nq": cq, "nqk": ck,
                  "hq": torch.empty((cq, self.d), dtype=torch.float32).pin_memory(),
                  "hD": torch.empty(ck, dtype=torch.float32).pin_memory(),
                  "hI": torch.empty(ck, dtype=torch.int64).pin_memory(),
                  "dq": torch.empty((cq, self.d), dtype=torch.float32, device=dev),
                  "dD": torch.empty(ck, dtype=torch.float32, device=dev),
                  "dI": torch.empty(ck, dtype=torch.int64, device=dev)}
            self._hb = hb
        return hb

    def search(self, x, k):
        """faiss Index.search(x, k) -> (D, I).  numpy in, numpy out: the queries
        go through a pinned staging buffer (one async copy each way, one stream
        sync), so the reference's one-profile-at-a-time loop (Retrieval.py:28-34)
        pays a few tens of microseconds per call, not a synchronous copy each way."""
        if isinstance(x, torch.Tensor):
            xt, _ = self._as_input(x)
            return self.search_device(xt, k)
        k = int(k)
        if k <= 0:
            raise ValueError("k must be positive")
        a = np.ascontiguousarray(x, dtype=np.float32)
        if a.ndim != 2 or a.shape[1] != self.d:
            raise AssertionError(f"expected (n, {self.d}) input, got {a.shape}")
        nq = a.shape[0]
        if nq == 0:
            return np.empty((0, k), np.float32), np.empty((0, k), np.int64)
        hb = self._host_buffers(nq, k)
        hb["hq"][:nq].numpy()[...] = a
        with torch.cuda.device(self.device):
            st = torch.cuda.current_stream(self.device)
            dq = hb["dq"][:nq]
            dq.copy_(hb["hq"][:nq], non_blocking=True)
            D, I = hb["dD"][:nq * k].view(nq, k), hb["dI"][:nq * k].view(nq, k)
            self._launch(dq, nq, k, D, I, None)
            hb["hD"][:nq * k].copy_(hb["dD"][:nq * k], non_blocking=True)
            hb["hI"][:nq * k].copy_(hb["dI"][:nq * k], non_blocking=True)
            st.synchronize()
        return hb["hD"][:nq * k].numpy().reshape(nq, k).copy(), hb["hI"][:nq * k].numpy().reshape(nq, k).copy()


class IndexFlatIP(IndexFlat):
    def __init__(self, d: int, device=None):
        super().__init__(d, METRIC_INNER_PRODUCT, device)


class IndexFlatL2(IndexFlat):
    def __init__(self, d: int, device=None):
        super().__init__(d, METRIC_L2, device)


class IndexHNSWFlat(IndexFlat):
    """faiss.IndexHNSWFlat(d, M) (Retrieval.py:16), the assignment index of the
    reference's k-means and of `index.search(xb, 1)` (Retrieval.py:21).

    faiss's HNSW is an approximate graph walk over the centroids; on the GPU a
    brute-force pass over a few hundred centroids is cheaper than a graph walk,
    so this index answers EXACTLY (recall 1.0, a superset of HNSW's quality;
    DESIGN.md).  `M` and `hnsw.efSearch` are accepted and recorded only."""

    class _Params:
        def __init__(self, M):
            self.M = M
            self.efSearch = 16
            self.efConstruction = 40

    def __init__(self, d: int, M: int = 32, metric: int = METRIC_L2, device=None):
        super().__init__(d, metric, device)
        self.hnsw = self._Params(int(M))


# ------------------------------------------------------------- k-means --
class Clustering:
    """faiss.Clustering(d, k) (Retrieval.py:12-18): `.niter`, `.verbose`,
    `.seed`, `.max_points_per_centroid`, `.spherical`, `.train(x, index)`,
    `.centroids`, `.obj`.

    Algorithm (faiss's, with the deterministic choices restated in
    oracle/ivf_oracle.py): subsample to k * max_points_per_centroid rows,
    init from random distinct rows, then `niter` x {assign with `index`
    (reset + add(centroids) + search(x, 1), as faiss does), centroid = mean of
    members (nrk_group_by_list + nrk_kmeans_update: fp64 sums in id order),
    split empty clusters}.  All arithmetic on the GPU; only the split step
    reads the k cluster sizes back."""

    def __init__(self, d: int, k: int, device=None):
        self.d = int(d)
        self.k = int(k)
        self.niter = 25
        self.nredo = 1
        self.verbose = False
        self.spherical = False
        self.seed = 1234
        self.max_points_per_centroid = 256
        self.min_points_per_centroid = 39
        self.device = torch.device(device) if device is not None else None
        self.centroids = torch.empty(0, dtype=torch.float32)
        self.obj: list[float] = []
        self.iteration_stats: list[dict] = []

    def _subsample(self, x: torch.Tensor) -> torch.Tensor:
        n = x.shape[0]
        cap = self.k * self.max_points_per_centroid
        if n > cap:
            perm = np.sort(np.random.default_rng(self.seed).permutation(n)[:cap])
            return x[torch.from_numpy(perm).to(x.device)].contiguous()
        return x

    def _split(self, cent: torch.Tensor, counts: np.ndarray, n: int) -> int:
        """faiss split_clusters: refill empty clusters from a size-weighted
        random cluster with a +-1/1024 symmetric perturbation."""
        if (counts > 0).all():
            return 0
        c = cent.cpu().numpy()
        k, d = c.shape
        rng = np.random.default_rng(1234)
        hassign = counts.astype(np.float64).copy()
        up, dn = np.float32(1 + 1.0 / 1024), np.float32(1 - 1.0 / 1024)
        even = (np.arange(d) % 2) == 0
        nsplit = 0
        for ci in range(k):
            if hassign[ci] != 0:
                continue
            cj = 0
            while True:
                if rng.random() < (hassign[cj] - 1.0) / float(n - k):
                    break
                cj = (cj + 1) % k
            c[ci] = c[cj]
            c[ci] = np.where(even, c[ci] * up, c[ci] * dn)
            c[cj] = np.where(even, c[cj] * dn, c[cj] * up)
            hassign[ci] = np.floor(hassign[cj] / 2)
            hassign[cj] -= hassign[ci]
            nsplit += 1
        cent.copy_(torch.from_numpy(c))
        return nsplit

    def train(self, x, index=None):
        L = _lib.load()
        if index is None:
            index = IndexFlatL2(self.d, device=self.device)
        dev = index.device
        xt = x.detach().to(dev, torch.float32).contiguous() if isinstance(x, torch.Tensor) else \
            torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(dev)
        if xt.dim() != 2 or xt.shape[1] != self.d:
            raise AssertionError(f"expected (n, {self.d}) training data")
        n0 = xt.shape[0]
        if n0 < self.k:
            raise RuntimeError(f"Number of training points ({n0}) should be at least as large as number of "
                               f"clusters ({self.k})")
        xs = self._subsample(xt)
        n = xs.shape[0]
        init = np.random.default_rng(self.seed + 1).permutation(n)[: self.k]
        cent = xs[torch.from_numpy(init).to(dev)].contiguous()
        list_off = torch.empty(self.k + 1, dtype=torch.int64, device=dev)
        pos2id = torch.empty(n, dtype=torch.int64, device=dev)
        pos2list = torch.empty(n, dtype=torch.int32, device=dev)
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
        sz = _lib.c_size(0)
        _lib.check(L.nrk_group_by_list_workspace(n, self.k, sz), "group_by_list_workspace")
        ws = torch.empty(max(sz.value, 1), dtype=torch.uint8, device=dev)
        self.obj = []
        self.iteration_stats = []
        with torch.cuda.device(dev):
            for it in range(self.niter):
                index.reset()
                index.add(cent)
                _, I, S = index.search_device(xs, 1, exact_scores=True)
                labels = I[:, 0].contiguous()
                obj = float(S[:, 0].sum().item())
                _lib.check(L.nrk_group_by_list(_lib.ptr(labels), n, self.k, _lib.ptr(list_off), _lib.ptr(pos2id),
                                               _lib.ptr(pos2list), _lib.ptr(bad), _lib.ptr(ws), ws.numel(),
                                               _lib.stream(dev)), "group_by_list")
                _lib.check(L.nrk_kmeans_update(_lib.ptr(xs), self.d, _lib.ptr(list_off), _lib.ptr(pos2id), self.k,
                                               _lib.ptr(cent), _lib.stream(dev)), "kmeans_update")
                counts = torch.diff(list_off).cpu().numpy()
                nsplit = self._split(cent, counts, n)
                if self.spherical:
                    cent.div_(cent.double().norm(dim=1, keepdim=True).clamp_min(1e-20).float())
                self.obj.append(obj)
                self.iteration_stats.append({"obj": obj, "nsplit": nsplit})
                if self.verbose:
                    print(f"  Iteration {it} objective={obj:g} nsplit={nsplit}")
        index.reset()
        index.add(cent)
        self.centroids = cent
        return self


def kmeans_assign(index: "IndexFlat", x: torch.Tensor):
    """labels of x under `index` (nearest centroid), device in/out."""
    _, I = index.search_device(x, 1)
    return I[:, 0].contiguous()


# --------------------------------------------------------------- IVF --
class IndexIVFFlat(_FallbackCounters):
    """faiss.IndexIVFFlat(quantizer, d, nlist, metric) (BASELINE configs[3]).

    train(x): faiss Clustering(d, nlist) with the quantizer as the assignment
    index (the quantizer ends up holding the centroids).  add(x): ids continue
    from ntotal; rows are assigned by the quantizer and the inverted lists
    (ids ascending inside a list) are rebuilt on the device.  search(x, k):
    the quantizer's top-`nprobe` lists, then nrk_ivf_search: the exact top-k
    among the probed lists' items (D/I as IndexFlat).  HBM per row: f32 row
    (exact rescoring) + bf16 list-major screening row + norms + 12 B of list
    bookkeeping."""

    def __init__(self, quantizer: IndexFlat, d: int, nlist: int, metric: int = METRIC_L2, device=None):
        if metric not in (METRIC_INNER_PRODUCT, METRIC_L2):
            raise ValueError(f"unsupported metric {metric}")
        self.quantizer = quantizer
        self.d = int(d)
        self.nlist = int(nlist)
        self.metric_type = int(metric)
        self.nprobe = 1
        # faiss's IndexIVF constructor: cp.niter = 10 (Level1Quantizer) and
        # spherical k-means for inner-product indexes
        self.cp = Clustering(d, nlist)
        self.cp.niter = 10
        self.cp.spherical = self.metric_type == METRIC_INNER_PRODUCT
        self.device = quantizer.device if device is None else torch.device(device)
        self.is_trained = quantizer.ntotal == self.nlist
        self.flat = IndexFlat(d, metric, device=self.device)  # id-order rows, bf16 copy, norms, stats
        self._assign = torch.empty(0, dtype=torch.int64, device=self.device)
        self._ws = None
        self.fallback_counts = None
        self.guard_word = None  # device int32[1]: the last search's guard word (check_guards)
        self._lists_valid = True
        self._n_lists = 0
        self.list_off = torch.zeros(self.nlist + 1, dtype=torch.int64, device=self.device)
        self.pos2id = torch.empty(0, dtype=torch.int64, device=self.device)
        self.pos2list = torch.empty(0, dtype=torch.int32, device=self.device)
        self.xbh_ivf = torch.empty((0, self.flat.dp), dtype=torch.int16, device=self.device)
        self.meta_ivf = torch.empty((0, 2), dtype=torch.float32, device=self.device)
        self.max_list = 0

    @property
    def ntotal(self) -> int:
        return self.flat.ntotal

    def train(self, x):
        if self.quantizer.ntotal == self.nlist and self.is_trained:
            return
        self.cp.train(x, self.quantizer)
        self.is_trained = True

    def _rebuild_lists(self):
        L = _lib.load()
        n = self.ntotal
        dev = self.device
        with torch.cuda.device(dev):
            self.pos2id = torch.empty(n, dtype=torch.int64, device=dev)
            self.pos2list = torch.empty(n, dtype=torch.int32, device=dev)
            bad = torch.zeros(1, dtype=torch.int32, device=dev)
            sz = _lib.c_size(0)
            _lib.check(L.nrk_group_by_list_workspace(n, self.nlist, sz), "group_by_list_workspace")
            ws = torch.empty(max(sz.value, 1), dtype=torch.uint8, device=dev)
            _lib.check(L.nrk_group_by_list(_lib.ptr(self._assign), n, self.nlist, _lib.ptr(self.list_off),
                                           _lib.ptr(self.pos2id), _lib.ptr(self.pos2list), _lib.ptr(bad),
                                           _lib.ptr(ws), ws.numel(), _lib.stream(dev)), "group_by_list")
            self.xbh_ivf = torch.empty((n, self.flat.dp), dtype=torch.int16, device=dev)
            self.meta_ivf = torch.empty((n, 2), dtype=torch.float32, device=dev)
            _lib.check(L.nrk_ivf_pack(_lib.ptr(self.pos2id), n, self.d, _lib.ptr(self.flat._xbh[:n]),
                                      _lib.ptr(self.flat._meta[:n]), _lib.ptr(self.xbh_ivf), _lib.ptr(self.meta_ivf),
                                      _lib.stream(dev)), "ivf_pack")
            if int(bad.item()):
                raise _lib.NrkError("IndexIVFFlat.add: assignment outside [0, nlist)")
            sizes = torch.diff(self.list_off)
            self.max_list = int(sizes.max().item()) if n else 0

    def add(self, x):
        if not self.is_trained:
            raise RuntimeError("IndexIVFFlat: train() before add()")
        xt, _ = self.flat._as_input(x)
        if xt.shape[0] == 0:
            return
        labels = kmeans_assign(self.quantizer, xt)
        self.flat.add(xt)
        self._assign = torch.cat([self._assign, labels])
        self._rebuild_lists()

    def reset(self):
        self.flat.reset()
        self._assign = torch.empty(0, dtype=torch.int64, device=self.device)
        self.list_off.zero_()
        self.max_list = 0

    def get_list_size(self, l: int) -> int:
        return int((self.list_off[l + 1] - self.list_off[l]).item())

    def list_ids(self, l: int) -> np.ndarray:
        """ids of inverted list l, ascending (cluster_to_articles, Retrieval.py:22-23)."""
        lo, hi = int(self.list_off[l].item()), int(self.list_off[l + 1].item())
        return self.pos2id[lo:hi].cpu().numpy()

    def _workspace(self, nbytes: int):
        # zero-filled on growth: no slot of a fresh workspace holds garbage, even
        # one a kernel reads before writing (the search re-initialises what it uses)
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = torch.zeros(max(nbytes, 1), dtype=torch.uint8, device=self.device)
        return self._ws

    def search_device(self, xq: torch.Tensor, k: int, exact_scores: bool = False, id_offset: int = 0,
                      stage_events=None, probe: torch.Tensor | None = None, check: bool = False):
        """Device-in, device-out IVF search -> (D, I[, S]).  check=True syncs and
        raises if the search's index guards tripped (check_guards)."""
        k = int(k)
        if k <= 0:
            raise ValueError("k must be positive")
        L = _lib.load()
        xq = self.flat._as_query(xq)
        nq = xq.shape[0]
        nprobe = max(1, min(int(self.nprobe), self.nlist))
        dev = self.device
        if probe is None:
            _, probe = self.quantizer.search_device(xq, nprobe)
        else:
            _lib.require_device(probe, what="IndexIVFFlat.search_device")
            if probe.shape != (nq, nprobe):
                raise AssertionError(f"probe must be ({nq}, {nprobe}), got {tuple(probe.shape)}")
            probe = probe.to(device=dev, dtype=torch.int64)
            if int(probe.max().item()) >= self.nlist:
                raise ValueError("probe holds a list number >= nlist")
        probe = probe.contiguous()
        D = torch.empty((nq, k), dtype=torch.float32, device=dev)
        I = torch.empty((nq, k), dtype=torch.int64, device=dev)
        S = torch.empty((nq, k), dtype=torch.float64, device=dev) if exact_scores else None
        if self.fallback_counts is None:
            self.fallback_counts = torch.zeros(2, dtype=torch.int32, device=dev)
        if self.guard_word is None:
            self.guard_word = torch.zeros(1, dtype=torch.int32, device=dev)
        n = self.ntotal
        f = self.flat
        with torch.cuda.device(dev):
            sz = _lib.c_size(0)
            _lib.check(L.nrk_ivf_search_workspace(nq, nprobe, self.nlist, self.max_list, self.d, k, sz),
                       "ivf_search_workspace")
            ws = self._workspace(sz.value)
            _lib.check(L.nrk_ivf_search(
                _lib.ptr(xq), nq, _lib.ptr(probe), nprobe, _lib.ptr(f._xb[:n]) if n else None,
                _lib.ptr(self.xbh_ivf) if n else None, _lib.ptr(self.meta_ivf) if n else None, _lib.ptr(f._stats),
                _lib.ptr(self.list_off), _lib.ptr(self.pos2id) if n else None,
                _lib.ptr(self.pos2list) if n else None, self.nlist, n, self.max_list, self.d, k, self.metric_type,
                _lib.ptr(D), _lib.ptr(I), _lib.ptr(S), int(id_offset), _lib.ptr(self.fallback_counts), _lib.ptr(ws),
                ws.numel(), stage_events.ev if stage_events is not None else None, _lib.stream(dev)), "ivf_search")
            # the search's guard word -> self.guard_word (device, no sync; include/nrk.h)
            _lib.check(L.nrk_ivf_search_status(_lib.ptr(ws), ws.numel(), _lib.ptr(self.guard_word),
                                               _lib.stream(dev)), "ivf_search_status")
        if check:
            self.check_guards()
        return (D, I, S) if exact_scores else (D, I)

    def check_guards(self):
        """Raise NrkError if the last search's guard word is nonzero: an index
        it read back from its own workspace was out of range (the access was
        skipped, the result is not valid).  Synchronises with the device."""
        g = int(self.guard_word.item())
        if g:
            names = [n for b, n in ((1, "seed position"), (2, "candidate position"), (4, "collect query row"),
                                    (8, "candidate count"), (16, "fallback query"), (32, "probed list"),
                                    (64, "gathered pair"), (128, "collected position")) if g & b]
            raise _lib.NrkError(f"ivf_search: index guard tripped (0x{g:x}: {', '.join(names)})")

    def search(self, x, k):
        xt, was_numpy = self.flat._as_input(x)
        D, I = self.search_device(xt, k)
        if was_numpy:  # the copy to the host syncs anyway: check the index guards with it
            D, I = D.cpu().numpy(), I.cpu().numpy()
            self.check_guards()
        return D, I


def knn_exact(xq: torch.Tensor, xb: torch.Tensor, k: int, metric: int = METRIC_L2, id_offset: int = 0):
    """Exact fp64 brute force on the GPU (no screening) -> (D, I, S)."""
    dev = _lib.require_device(xq, xb, what="knn_exact")
    xq = xq.float().contiguous()
    xb = xb.float().contiguous()
    nq, d = xq.shape
    D = torch.empty((nq, k), dtype=torch.float32, device=dev)
    I = torch.empty((nq, k), dtype=torch.int64, device=dev)
    S = torch.empty((nq, k), dtype=torch.float64, device=dev)
    with torch.cuda.device(dev):
        _lib.check(_lib.load().nrk_knn_exact(_lib.ptr(xq), nq, _lib.ptr(xb), xb.shape[0], d, k, metric, _lib.ptr(D),
                                             _lib.ptr(I), _lib.ptr(S), id_offset, _lib.stream(dev)), "knn_exact")
    return D, I, S


def topk_merge(S_parts: torch.Tensor, I_parts: torch.Tensor, k: int, metric: int):
    """Merge [nparts][nq][k] exact-score lists -> (D, I, S) (multi-GPU shard merge)."""
    dev = _lib.require_device(S_parts, I_parts, what="topk_merge")
    nparts, nq, kk = S_parts.shape
    if kk != k:
        raise ValueError("k mismatch")
    D = torch.empty((nq, k), dtype=torch.float32, device=dev)
    I = torch.empty((nq, k), dtype=torch.int64, device=dev)
    S = torch.empty((nq, k), dtype=torch.float64, device=dev)
    with torch.cuda.device(dev):
        _lib.check(_lib.load().nrk_topk_merge(_lib.ptr(S_parts.contiguous()), _lib.ptr(I_parts.contiguous()), nparts,
                                              nq, k, metric, _lib.ptr(D), _lib.ptr(I), _lib.ptr(S),
                                              _lib.stream(dev)), "topk_merge")
    return D, I, S
