"""ctypes binding of libnrk.so (the C-ABI in include/nrk.h).

This is the binding a maintainer of the reference would add (the reference is
Python calling native code through faiss's SWIG layer and torch's ATen): plain
pointers, sizes and a hipStream_t.  There is no CPU fallback — a product call
without the library, or with host tensors, raises.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NRK_LIB") or os.path.join(_HERE, "libnrk.so")  # NRK_LIB: A/B builds only

NRK_METRIC_INNER_PRODUCT = 0
NRK_METRIC_L2 = 1
NRK_DTYPE_F32 = 0
NRK_DTYPE_BF16 = 1

c_p = ctypes.c_void_p
c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_f32 = ctypes.c_float
c_size = ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/nrk.h exactly (tests check both ways)
SIGNATURES = {
    "nrk_last_error": (ctypes.c_char_p, []),
    "nrk_version": (ctypes.c_int, []),
    "nrk_padded_dim": (ctypes.c_int, [c_i32]),
    "nrk_knn_flat_main_pass": (ctypes.c_int, [c_i64, c_i64, c_i32, c_i32, c_i32, ctypes.c_char_p, c_size]),
    "nrk_flat_prepare": (ctypes.c_int, [c_p, c_i64, c_i32, c_p, c_p, c_p, c_p]),
    "nrk_knn_flat_workspace": (ctypes.c_int, [c_i64, c_i64, c_i32, c_i32, ctypes.POINTER(c_size)]),
    "nrk_knn_flat": (ctypes.c_int, [c_p, c_i64, c_p, c_p, c_p, c_p, c_i64, c_i32, c_i32, c_i32, c_p, c_p, c_p, c_i64,
                                    c_p, c_p, c_size, c_p, c_p]),
    "nrk_knn_exact": (ctypes.c_int, [c_p, c_i64, c_p, c_i64, c_i32, c_i32, c_i32, c_p, c_p, c_p, c_i64, c_p]),
    "nrk_topk_merge": (ctypes.c_int, [c_p, c_p, c_i32, c_i64, c_i32, c_i32, c_p, c_p, c_p, c_p]),
    "nrk_group_by_list_workspace": (ctypes.c_int, [c_i64, c_i32, ctypes.POINTER(c_size)]),
    "nrk_group_by_list": (ctypes.c_int, [c_p, c_i64, c_i32, c_p, c_p, c_p, c_p, c_p, c_size, c_p]),
    "nrk_ivf_pack": (ctypes.c_int, [c_p, c_i64, c_i32, c_p, c_p, c_p, c_p, c_p]),
    "nrk_kmeans_update": (ctypes.c_int, [c_p, c_i32, c_p, c_p, c_i32, c_p, c_p]),
    "nrk_ivf_search_workspace": (ctypes.c_int, [c_i64, c_i32, c_i32, c_i64, c_i32, c_i32, ctypes.POINTER(c_size)]),
    "nrk_ivf_search": (ctypes.c_int, [c_p, c_i64, c_p, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i32, c_i64, c_i64,
                                      c_i32, c_i32, c_i32, c_p, c_p, c_p, c_i64, c_p, c_p, c_size, c_p, c_p]),
    "nrk_ivf_search_status": (ctypes.c_int, [c_p, c_size, c_p, c_p]),
    "nrk_din_head_workspace": (ctypes.c_int, [c_i32, c_i32, c_i32, ctypes.POINTER(c_size)]),
    "nrk_din_head_train": (ctypes.c_int, [c_p, c_p, c_i64, c_p, c_i32, c_i32, c_i32, c_f32, c_f32, c_f32,
                                          ctypes.c_uint64, c_p, c_p, c_p, c_p, c_p, c_p, c_size, c_p]),
    "nrk_clip_adam_workspace": (ctypes.c_int, [c_i64, ctypes.POINTER(c_size)]),
    "nrk_clip_adam": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_i64, c_p, c_f32, c_p, c_f32, c_f32, c_f32, c_f32, c_f32,
                                     c_p, c_size, c_p]),
    "nrk_din_attn_fwd": (ctypes.c_int, [c_p, c_p, c_i64, c_i32, c_p, c_p, c_p, c_f32, c_i32, c_i32, c_i32, c_i32,
                                        c_p, c_p, c_p]),
    "nrk_din_attn_bwd_workspace": (ctypes.c_int, [c_i32, c_i32, c_i32, ctypes.POINTER(c_size)]),
    "nrk_din_attn_bwd": (ctypes.c_int, [c_p, c_p, c_i64, c_i32, c_p, c_p, c_p, c_f32, c_i32, c_i32, c_i32, c_i32,
                                        c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_size, c_p]),
    "nrk_din_attn_bwd_params": (ctypes.c_int, [c_p, c_p, c_i64, c_i32, c_p, c_p, c_p, c_p, c_i32, c_i32, c_i32, c_i32,
                                               c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_size, c_p]),
    "nrk_din_attn_bwd_params_head": (ctypes.c_int, [c_p, c_p, c_i64, c_i32, c_p, c_p, c_p, c_p, c_i32, c_i32, c_i32,
                                                    c_i32, c_p, c_p, c_i32, c_p, c_p, c_size, c_p, c_p, c_p, c_p, c_i64,
                                                    c_p, c_p, c_size, c_p]),
    "nrk_clip_adam_partials": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_i64, c_p, c_f32, c_p, c_f32, c_f32, c_f32, c_f32,
                                              c_f32, c_p, c_i32, c_p, c_size, c_p]),
    "nrk_din_head_ws_views": (ctypes.c_int, [c_i32, c_i32, c_i32, c_p, c_size, c_p, c_p, c_p]),
    "nrk_din_batch_u": (ctypes.c_int, [c_p, c_i32, c_i32, c_p, c_p, c_i32, c_p, c_p, c_p]),
    "nrk_din_batch": (ctypes.c_int, [c_p, c_i32, c_p, c_p, c_p, c_i64, c_i32, c_p, c_i64, c_i32, c_i32, c_p, c_p,
                                     c_i32, c_p, c_p, c_p, c_p, c_p, c_p]),
    "nrk_din_rerank_workspace": (ctypes.c_int, [ctypes.POINTER(c_size)]),
    "nrk_din_rerank": (ctypes.c_int, [c_p, c_i64, c_i32, c_p, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_i32, c_i32,
                                      c_i32, c_p, c_p, c_size, c_p]),
    "nrk_din_rerank_project": (ctypes.c_int, [c_p, c_i64, c_i32, c_p, c_i64, c_i32, c_i32, c_i32, c_p, c_p, c_p]),
    "nrk_din_rerank_project_hist": (ctypes.c_int, [c_p, c_i64, c_i32, c_p, c_i64, c_i32, c_i32, c_i32, c_p, c_p, c_p]),
    "nrk_din_rerank_max_history": (ctypes.c_int, [c_i32, c_i32, ctypes.POINTER(c_i32)]),
    "nrk_din_rerank_projected": (ctypes.c_int, [c_p, c_i64, c_i32, c_p, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p, c_p,
                                                c_i32, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p, c_size, c_p]),
    "nrk_rerank_user_stats": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_i32, c_p, c_p, c_p, c_p]),
    "nrk_embed_workspace": (ctypes.c_int, [c_i32, c_i32, c_i32, ctypes.POINTER(c_size)]),
    "nrk_embed": (ctypes.c_int, [c_p, c_i64, c_i64, c_i32, c_p, c_p, c_i32, c_p, c_p, c_i32, c_p, c_p, c_size, c_p]),
    "nrk_gather_rows": (ctypes.c_int, [c_p, c_i64, c_i32, c_p, c_i64, c_i32, c_p, c_p]),
    "nrk_train_samples": (ctypes.c_int, [c_p, c_i64, c_p, c_i64, c_i32, c_p, c_i64, c_p, c_p, c_p, c_p]),
    "nrk_triplet_samples": (ctypes.c_int, [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p]),
}



class RerankParams(ctypes.Structure):
    """nrk_din_rerank_params (include/nrk.h): device pointers of the folded,
    hi/lo-split eval model (pipeline.rerank_params)."""
    _fields_ = [(n, c_p) for n in ("W1q_hi", "W1q_lo", "W1k_hi", "W1k_lo", "b1", "w2", "H1q_hi", "H1q_lo", "H1p_hi",
                                   "H1p_lo", "c1", "H2_hi", "H2_lo", "c2", "h3")] + [("c3", c_f32)]


_lib = None


class NrkError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load libnrk.so.  torch is imported first so that its bundled HIP runtime
    is the one the library's libamdhip64.so.7 dependency resolves to."""
    global _lib
    if _lib is None:
        if not os.path.exists(path):
            raise NrkError(f"{path} is missing: build it with `python -m newsrecommend_amd.build` "
                           "(there is no CPU fallback for the HIP path)")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("NRK_LIB") and not hasattr(lib, name):
                continue  # an A/B build of an older library: entry points it lacks stay unbound
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().nrk_last_error().decode(errors="replace")
        raise NrkError(f"{what or 'libnrk'} failed (code {rc}): {msg}")


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def stream(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(*tensors, what: str = "libnrk") -> torch.device:
    dev = None
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise NrkError(f"{what}: tensors must live on the GPU (got {t.device}); the HIP path has no CPU fallback")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise NrkError(f"{what}: tensors on different devices ({dev} vs {t.device})")
    return dev


# ------------------------------------------------ HIP events (bench timing) --
_hip = None


def _hiprt():
    """The HIP runtime torch loaded (same process-wide libamdhip64.so.7)."""
    global _hip
    if _hip is None:
        import torch  # noqa: F401
        h = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
        h.hipEventCreate.argtypes = [ctypes.POINTER(c_p)]
        h.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), c_p, c_p]
        h.hipEventSynchronize.argtypes = [c_p]
        h.hipEventDestroy.argtypes = [c_p]
        _hip = h
    return _hip


class StageEvents:
    """NRK_KNN_STAGES+1 hipEvent_t for nrk_knn_flat's stage_events."""

    N = 5

    def __init__(self):
        h = _hiprt()
        self.ev = (c_p * self.N)()
        for i in range(self.N):
            e = c_p()
            if h.hipEventCreate(ctypes.byref(e)) != 0:
                raise NrkError("hipEventCreate failed")
            self.ev[i] = e

    def elapsed_ms(self):
        h = _hiprt()
        h.hipEventSynchronize(self.ev[self.N - 1])
        out = []
        for i in range(self.N - 1):
            t = ctypes.c_float(0)
            h.hipEventElapsedTime(ctypes.byref(t), self.ev[i], self.ev[i + 1])
            out.append(t.value)
        return out

    def __del__(self):
        try:
            h = _hiprt()
            for i in range(self.N):
                h.hipEventDestroy(self.ev[i])
        except Exception:
            pass
