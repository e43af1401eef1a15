"""oracle/knn_oracle.py — TEST INFRASTRUCTURE ONLY (checker / CPU baseline,
never the product).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module.

Three CPU restatements of the faiss flat-search contract (Retrieval.py:21,
25-32; semantics in knn_exact.c's header — faiss itself is unavailable
offline, so this part of the oracle is "parity unpinned"):

  exact_search  ctypes -> liboracle_knn.so: fp64 sequential-d scores, ties to
                the lower id.  THE oracle: the GPU path must equal it bit for
                bit (indices and the fp32-rounded scores).
  numpy_search  an independent numpy float64 restatement (BLAS order), used
                only to cross-check exact_search.
  faiss_port    faiss-cpu's own algorithm for nq >= 20 (faiss
                exhaustive_*_blas: fp32 sgemm over 4096-query x 1024-row
                blocks, ||x||^2 + ||y||^2 - 2<x,y> for L2, per-query heap
                top-k) — timed as the CPU baseline (kind "port").
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle_knn.so")
METRIC_IP, METRIC_L2 = 0, 1
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["gcc", "-O2", "-fopenmp", "-shared", "-fPIC", "-std=c11",
                            os.path.join(HERE, "knn_exact.c"), "-o", LIB, "-lm"], check=True)
        lib = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        lib.oracle_knn_exact.argtypes = [P, ctypes.c_int64, P, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         P, P, P, ctypes.c_int64]
        lib.oracle_knn_exact.restype = ctypes.c_int
        lib.oracle_topk_merge.argtypes = [P, P, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int, P, P, P]
        lib.oracle_topk_merge.restype = ctypes.c_int
        _lib = lib
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def exact_search(xq, xb, k, metric, id_offset=0):
    """-> D (nq, k) f32, I (nq, k) int64, S (nq, k) f64."""
    xq = np.ascontiguousarray(xq, np.float32)
    xb = np.ascontiguousarray(xb, np.float32)
    nq, d = xq.shape
    D = np.empty((nq, k), np.float32)
    I = np.empty((nq, k), np.int64)
    S = np.empty((nq, k), np.float64)
    rc = _load().oracle_knn_exact(_p(xq), nq, _p(xb), xb.shape[0], d, k, metric, _p(D), _p(I), _p(S), id_offset)
    if rc != 0:
        raise ValueError("oracle_knn_exact: bad arguments")
    return D, I, S


def merge(S_parts, I_parts, k, metric):
    S_parts = np.ascontiguousarray(S_parts, np.float64)
    I_parts = np.ascontiguousarray(I_parts, np.int64)
    nparts, nq, _ = S_parts.shape
    D = np.empty((nq, k), np.float32)
    I = np.empty((nq, k), np.int64)
    S = np.empty((nq, k), np.float64)
    _load().oracle_topk_merge(_p(S_parts), _p(I_parts), nparts, nq, k, metric, _p(D), _p(I), _p(S))
    return D, I, S


def numpy_search(xq, xb, k, metric):
    """Independent float64 restatement (lexsort on (-goodness, id))."""
    q = np.asarray(xq, np.float64)
    x = np.asarray(xb, np.float64)
    if metric == METRIC_IP:
        g = q @ x.T
    else:
        g = -(((q[:, None, :] - x[None, :, :]) ** 2).sum(-1))
    ids = np.arange(x.shape[0])
    I = np.empty((q.shape[0], k), np.int64)
    for i in range(q.shape[0]):
        order = np.lexsort((ids, -g[i]))[:k]
        I[i, : len(order)] = order
        I[i, len(order):] = -1
    S = np.take_along_axis(g, np.maximum(I, 0), 1)
    return (S if metric == METRIC_IP else -S), I


def faiss_port(xq, xb, k, metric, bs_x=4096, bs_y=1024):
    """faiss-cpu flat search restated (blocked fp32 BLAS + per-query top-k)."""
    xq = np.ascontiguousarray(xq, np.float32)
    xb = np.ascontiguousarray(xb, np.float32)
    nq = xq.shape[0]
    best_s = np.full((nq, k), -np.inf if metric == METRIC_IP else np.inf, np.float32)
    best_i = np.full((nq, k), -1, np.int64)
    yn = (xb * xb).sum(1) if metric == METRIC_L2 else None
    for i0 in range(0, nq, bs_x):
        q = xq[i0:i0 + bs_x]
        qn = (q * q).sum(1)[:, None] if metric == METRIC_L2 else None
        cs = best_s[i0:i0 + bs_x]
        ci = best_i[i0:i0 + bs_x]
        for j0 in range(0, xb.shape[0], bs_y * 64):
            y = xb[j0:j0 + bs_y * 64]
            ip = q @ y.T
            s = ip if metric == METRIC_IP else (qn + yn[j0:j0 + y.shape[0]][None, :] - 2 * ip)
            ids = np.broadcast_to(np.arange(j0, j0 + y.shape[0]), s.shape)
            allv = np.concatenate([cs, s], 1)
            alli = np.concatenate([ci, ids], 1)
            kk = min(k, allv.shape[1])
            part = np.argpartition(-allv if metric == METRIC_IP else allv, kk - 1, axis=1)[:, :kk]
            cs = np.take_along_axis(allv, part, 1)
            ci = np.take_along_axis(alli, part, 1)
        order = np.argsort(-cs if metric == METRIC_IP else cs, axis=1, kind="stable")
        best_s[i0:i0 + bs_x] = np.take_along_axis(cs, order, 1)
        best_i[i0:i0 + bs_x] = np.take_along_axis(ci, order, 1)
    return best_s, best_i
