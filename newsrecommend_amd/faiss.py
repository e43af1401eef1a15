"""faiss-compatible flat indexes on MI355X (drop-in for the subset of the faiss
Python API the reference's retrieval path uses).

Reference call sites (Retrieval.py):
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


class IndexFlat:
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
        self.last_fallback = None  # device int32[1]: queries that needed the exact scan
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
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)
        return self._ws

    def search_device(self, xq: torch.Tensor, k: int, exact_scores: bool = False, id_offset: int = 0,
                      stage_events=None):
        """Device-in, device-out search: returns (D f32, I int64[, S f64]) on the GPU."""
        k = int(k)
        if k <= 0:
            raise ValueError("k must be positive")
        nq = xq.shape[0]
        L = _lib.load()
        D = torch.empty((nq, k), dtype=torch.float32, device=self.device)
        I = torch.empty((nq, k), dtype=torch.int64, device=self.device)
        S = torch.empty((nq, k), dtype=torch.float64, device=self.device) if exact_scores else None
        if self.last_fallback is None:
            self.last_fallback = torch.zeros(1, dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            sz = _lib.c_size(0)
            _lib.check(L.nrk_knn_flat_workspace(nq, self._n, self.d, k, sz), "knn_flat_workspace")
            ws = self._workspace(sz.value)
            n = self._n
            _lib.check(L.nrk_knn_flat(
                _lib.ptr(xq), nq, _lib.ptr(self._xb[:n]) if n else None, _lib.ptr(self._xbh[:n]) if n else None,
                _lib.ptr(self._meta[:n]) if n else None, _lib.ptr(self._stats), n, self.d, k, self.metric_type,
                _lib.ptr(D), _lib.ptr(I), _lib.ptr(S), int(id_offset), _lib.ptr(self.last_fallback), _lib.ptr(ws),
                ws.numel(), stage_events.ev if stage_events is not None else None, _lib.stream(self.device)),
                "knn_flat")
        return (D, I, S) if exact_scores else (D, I)

    def search(self, x, k):
        """faiss Index.search(x, k) -> (D, I)."""
        xt, was_numpy = self._as_input(x)
        D, I = self.search_device(xt, k)
        if was_numpy:
            return D.cpu().numpy(), I.cpu().numpy()
        return D, I


class IndexFlatIP(IndexFlat):
    def __init__(self, d: int, device=None):
        super().__init__(d, METRIC_INNER_PRODUCT, device)


class IndexFlatL2(IndexFlat):
    def __init__(self, d: int, device=None):
        super().__init__(d, METRIC_L2, device)


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
