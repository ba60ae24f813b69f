"""ctypes binding of libpardis.so (the C ABI in include/pardis.h).

This is the only way the package computes anything: there is no CPU or
PyTorch fallback.  If the library is missing or no ROCm GPU is visible the
calls raise.  ``torch`` is imported first so the process has exactly one HIP
runtime (torch's libamdhip64.so.7, which libpardis then binds to).
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PYPARDIS_LIB") or os.path.join(HERE, "libpardis.so")   # (override: A/B builds)

PD_F32, PD_F64 = 0, 1
PD_EUCLIDEAN, PD_CITYBLOCK = 0, 1
PD_OPT_TIMING, PD_OPT_FULL_COUNTS, PD_OPT_SEQUENTIAL_MOMENTS = 1, 2, 3
PD_OPT_XSUB, PD_OPT_FP32_SCREEN = 6, 7
PD_OPT_SWEEP_STATS = 8
PD_OPT_DENSE_PRUNE = 11
PD_OPT_COUNT_ROTATE = 12
PD_OPT_CENTRE_WINDOW = 13
PD_OPT_DIR_BUDGET = 14
PD_OPT_LABEL_BUCKETS = 15
PD_OPT_DIR_PAGED = 17
PD_OPT_DENSE_SCREEN = 18
PD_OPT_SHARD_CORE_BIT = 19
PD_OPT_COUNT_REPLAY = 24
PD_OPT_HALO_PASSES = 25
PD_OPT_HALO_CAP = 26
PD_OPT_KD_FUSE = 27
PD_OPT_VERIFY_FUSED = 28
PD_OPT_HALO_TREE = 29
PD_OPT_KD_REPLAY = 30
# retired in round 5 (pardis.h): set_option raises for them
PD_OPT_RETIRED = (4, 5, 9, 10, 16, 20, 21, 22, 23)
TIMING_SLOTS = ["halo", "sort", "gather", "cells", "count", "link", "merge", "roots", "border",
                "label", "total", "records", "cells_n", "grid_cells", "key_bits", "core_records",
                "s_count_cand", "s_link_cand", "s_link_hit", "s_link_core", "s_link_same",
                "s_link_find_same", "s_link_unions", "s_verify_pairs", "grid_grow",
                "count_kernel", "dir_paged", "dir_words", "s_count_batches", "s_count_staged",
                "halo_fallback"]

# every symbol include/pardis.h declares (tests/test_abi.py checks the .so)
EXPORTS = ["pd_abi_version", "pd_last_error", "pd_ctx_create", "pd_ctx_destroy",
           "pd_ctx_set_option", "pd_ctx_timings", "pd_bbox", "pd_kd_moments", "pd_kd_counts",
           "pd_kd_split", "pd_halo_members", "pd_cluster", "pd_train", "pd_kd_moments_dd",
           "pd_route", "pd_pack", "pd_train_begin", "pd_train_exports", "pd_merge_exports",
           "pd_train_end", "pd_select_roots", "pd_sort_pairs", "pd_sort_u32", "pd_rank_labels",
           "pd_kd_radix_hist", "pd_kd_pass", "pd_owned_results", "pd_scatter_results",
           "pd_comm_unique_id", "pd_comm_init", "pd_comm_init_all", "pd_comm_destroy",
           "pd_comm_all_reduce", "pd_comm_all_gather_v", "pd_comm_all_to_all_v",
           "pd_comm_broadcast", "pd_dense_count", "pd_dense_link", "pd_dense_border",
           "pd_dense_finish", "pd_kd_build", "pd_kd_labels", "pd_train_tree", "pd_kdx_begin", "pd_kdx_moments",
           "pd_kdx_axes", "pd_kdx_counts", "pd_kdx_boundary", "pd_kdx_end", "pd_route2",
           "pd_pack2", "pd_results", "pd_results_scatter", "pd_comm_exchange", "pd_comm_abort",
           "pd_comm_self_check", "pd_comm_size"]


class PardisError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libpardis error {code}: {msg}")
        self.code = code


_lib = None
_lock = threading.Lock()
_tls = threading.local()


def load():
    """Load the in-tree library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -m pypardis_amd.build` "
                "(hipcc --offload-arch=gfx950).  There is no CPU fallback.")
        lib = ctypes.CDLL(LIB_PATH)
        P, I32, I64, D = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
        U32 = ctypes.c_uint32
        sig = {
            "pd_abi_version": ([], I32),
            "pd_last_error": ([], ctypes.c_char_p),
            "pd_ctx_create": ([I32, ctypes.POINTER(P)], I32),
            "pd_ctx_destroy": ([P], I32),
            "pd_ctx_set_option": ([P, I32, I64], I32),
            "pd_ctx_timings": ([P, P, I32], I32),
            "pd_bbox": ([P, P, I32, I64, I32, P, P, P], I32),
            "pd_kd_moments": ([P, P, I32, I64, I32, P, I32, P, P, P], I32),
            "pd_kd_counts": ([P, P, I32, I64, I32, P, I32, P, P, P, P, P], I32),
            "pd_kd_split": ([P, P, I32, I64, I32, P, I32, P, P, P, P, P], I32),
            "pd_halo_members": ([P, P, I32, I64, I32, I32, P, P, P, I64, P], I32),
            "pd_cluster": ([P, P, I32, I64, I32, D, I32, I32, P, P, P, P, P], I32),
            "pd_train": ([P, P, I32, I64, I32, D, I32, I32, I32, P, P, P, P, P, P, P, P], I32),
            "pd_kd_moments_dd": ([P, P, I32, I64, I32, P, I32, P, P, P], I32),
            "pd_route": ([P, P, I32, I64, I32, I32, P, P, I32, P, P, P], I32),
            "pd_pack": ([P, P, I32, I64, I32, P, I32, P, I32, P, P, U32, P, P, P, P, I64, P, P],
                        I32),
            "pd_train_begin": ([P, P, I32, I64, I32, D, I32, I32, I32, P, P, P, P, P, P, P], I32),
            "pd_train_exports": ([P, P, P, I64, P], I32),
            "pd_merge_exports": ([P, P, P, I64, P, P, P, P], I32),
            "pd_train_end": ([P, I64, P, P, I64, P, P, P], I32),
            "pd_select_roots": ([P, P, P, I64, P, P, P], I32),
            "pd_sort_u32": ([P, P, I64, P], I32),
            "pd_sort_pairs": ([P, P, I32, P, I64, I32, P], I32),
            "pd_rank_labels": ([P, P, I64, P, I64, P, P], I32),
            "pd_kd_radix_hist": ([P, P, I32, I64, I32, P, I32, P, P, P, I32, P, P], I32),
            "pd_kd_pass": ([P, P, I32, I64, I32, P, I32, I32, P, P, P, P, I32, P, P, P, P, P],
                           I32),
            "pd_owned_results": ([P, I64, P, P, P, P, I32, P, P, I64, P, P, P], I32),
            "pd_scatter_results": ([P, P, I64, U32, I64, P, P, P], I32),
            "pd_comm_unique_id": ([P], I32),
            "pd_comm_init": ([P, I32, I32, P, ctypes.POINTER(P)], I32),
            "pd_comm_init_all": ([I32, P, P], I32),
            "pd_comm_destroy": ([P], I32),
            "pd_comm_all_reduce": ([P, P, P, I64, I32, I32, P], I32),
            "pd_comm_all_gather_v": ([P, P, P, P, I32, P], I32),
            "pd_comm_all_to_all_v": ([P, P, P, P, P, I32, P], I32),
            "pd_comm_broadcast": ([P, P, I64, I32, I32, P], I32),
            "pd_dense_count": ([P, P, I32, I64, I32, D, I32, I32, P, I32, I32, P, P], I32),
            "pd_dense_link": ([P, P, P, P, P], I32),
            "pd_dense_border": ([P, P, I32, P, P, P], I32),
            "pd_dense_finish": ([P, P, P, P, P, P, P], I32),
            "pd_kd_build": ([P, P, I32, I64, I32, P, I32, P, P, P, I32, P, P, P, P], I32),
            "pd_kd_labels": ([P, P, I32, I64, I32, P, I32, P, P, P, P, P, P], I32),
            "pd_train_tree": ([P, P, I32, I64, I32, D, I32, I32, I32, P, P, I32, P, P, P, P, P, P, P,
                               P, P, P], I32),
            "pd_kdx_begin": ([P, I32, I32, P, P, P, P], I32),
            "pd_kdx_moments": ([P, P, I32, I64, I32, P, I32, P, P], I32),
            "pd_kdx_axes": ([P, P, I32, I32, P], I32),
            "pd_kdx_counts": ([P, P, I32, I64, I32, P, I32, P, P], I32),
            "pd_kdx_boundary": ([P, P, I32, P], I32),
            "pd_kdx_end": ([P, P, I32, I64, I32, P, I32, P, P, P, P], I32),
            "pd_route2": ([P, P, I32, I64, I32, I32, P, P, P, I32, P, P], I32),
            "pd_pack2": ([P, P, I32, I64, I32, P, I32, P, P, U32, I32, P, P, P, P, P], I32),
            "pd_results": ([P, I64, P, P, P, P, P, I64, I64, U32, I64, I32, I32, P, I64, P, P, P,
                            P], I32),
            "pd_results_scatter": ([P, P, I64, U32, I64, P, P, P], I32),
            "pd_comm_exchange": ([P, I32, P, P, P, P, P, P, P, I32, P], I32),
            "pd_comm_abort": ([P], I32),
            "pd_comm_self_check": ([P], I32),
            "pd_comm_size": ([P, P, P], I32),
        }
        for name, (args, res) in sig.items():
            f = getattr(lib, name)
            f.argtypes = args
            f.restype = res
        _lib = lib
        return lib


def _check(rc):
    if rc != 0:
        raise PardisError(rc, load().pd_last_error().decode(errors="replace"))


class Context:
    """One pd_ctx per (host thread, device)."""

    def __init__(self, device):
        self.device = int(device)
        self.ptr = ctypes.c_void_p()
        _check(load().pd_ctx_create(self.device, ctypes.byref(self.ptr)))

    def __del__(self):
        try:
            if self.ptr:
                load().pd_ctx_destroy(self.ptr)
        except Exception:
            pass

    def set_option(self, opt, value):
        _check(load().pd_ctx_set_option(self.ptr, opt, int(value)))

    def timings(self):
        out = np.zeros(len(TIMING_SLOTS), np.float64)
        _check(load().pd_ctx_timings(self.ptr, out.ctypes.data, len(out)))
        return dict(zip(TIMING_SLOTS, out.tolist()))


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("pypardis_amd needs a ROCm GPU (MI355X / gfx950); none is visible. "
                           "There is no CPU fallback.")


def context(device=None):
    require_gpu()
    load()
    dev = torch.cuda.current_device() if device is None else int(device)
    cache = getattr(_tls, "ctx", None)
    if cache is None:
        cache = _tls.ctx = {}
    if dev not in cache:
        cache[dev] = Context(dev)
    return cache[dev]


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _dtype_code(t):
    if t.dtype == torch.float32:
        return PD_F32
    if t.dtype == torch.float64:
        return PD_F64
    raise TypeError(f"coordinates must be float32 or float64, got {t.dtype}")


def _check_points(X):
    if not isinstance(X, torch.Tensor) or not X.is_cuda:
        raise TypeError("X must be a CUDA (ROCm) torch tensor")
    if X.dim() != 2 or not X.is_contiguous():
        raise ValueError("X must be a contiguous (n, d) tensor")
    return _dtype_code(X)


def metric_code(metric):
    if callable(metric):
        metric = getattr(metric, "__name__", repr(metric))
    m = str(metric).lower()
    if m in ("euclidean", "l2", "minkowski"):
        return PD_EUCLIDEAN
    if m in ("cityblock", "manhattan", "l1"):
        return PD_CITYBLOCK
    raise ValueError(f"metric {metric!r}: only euclidean and cityblock keep the 2*eps box "
                     "expansion exact (R:dbscan/dbscan.py:88-91)")


# ----------------------------------------------------------------- stages
def bbox(X, ctx=None):
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    d = X.shape[1]
    out = np.zeros(2 * d, np.float64)
    bad = np.zeros(1, np.int64)
    _check(load().pd_bbox(ctx.ptr, X.data_ptr(), dt, X.shape[0], d, out.ctypes.data,
                          bad.ctypes.data, _stream(X.device)))
    return out[:d], out[d:], int(bad[0])


def kd_moments(X, labels, sel, sequential=False, ctx=None):
    """sequential=True: the reference's left-to-right fold (bit-identical
    boundaries, slow); default: correctly rounded double-double sums."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    d = X.shape[1]
    sel = np.ascontiguousarray(sel, np.int32)
    out = np.zeros((len(sel), 3, d), np.float64)
    if sequential:
        ctx.set_option(PD_OPT_SEQUENTIAL_MOMENTS, 1)
    try:
        _check(load().pd_kd_moments(ctx.ptr, X.data_ptr(), dt, X.shape[0], d, labels.data_ptr(),
                                    len(sel), sel.ctypes.data, out.ctypes.data,
                                    _stream(X.device)))
    finally:
        if sequential:
            ctx.set_option(PD_OPT_SEQUENTIAL_MOMENTS, 0)
    return out


def kd_counts(X, labels, sel, axis, bounds, ctx=None):
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    sel = np.ascontiguousarray(sel, np.int32)
    axis = np.ascontiguousarray(axis, np.int32)
    bounds = np.ascontiguousarray(bounds, np.float64).reshape(len(sel), 7)
    out = np.zeros((len(sel), 8), np.int64)
    _check(load().pd_kd_counts(ctx.ptr, X.data_ptr(), dt, X.shape[0], X.shape[1],
                               labels.data_ptr(), len(sel), sel.ctypes.data, axis.ctypes.data,
                               bounds.ctypes.data, out.ctypes.data, _stream(X.device)))
    return out


def kd_split(X, labels, sel, axis, boundary, new, ctx=None):
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    sel = np.ascontiguousarray(sel, np.int32)
    axis = np.ascontiguousarray(axis, np.int32)
    boundary = np.ascontiguousarray(boundary, np.float64)
    new = np.ascontiguousarray(new, np.int32)
    _check(load().pd_kd_split(ctx.ptr, X.data_ptr(), dt, X.shape[0], X.shape[1],
                              labels.data_ptr(), len(sel), sel.ctypes.data, axis.ctypes.data,
                              boundary.ctypes.data, new.ctypes.data, _stream(X.device)))


def kd_pass(X, labels, split=None, sel=(), labels_zero=False, bbox=False, ctx=None):
    """One fused KD level pass (pd_kd_pass): apply ``split`` = (sel, axes,
    boundary, new) of the previous level to ``labels`` in place, then the
    double-double moment partials (len(sel), 1 + 4d) of the labels ``sel``;
    with ``bbox`` (first level: labels_zero, one label) also (lo, hi, bad).
    Returns dd, or (dd, lo, hi, bad)."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n, d = X.shape
    sel = np.ascontiguousarray(sel, np.int32)
    out = np.zeros((len(sel), 1 + 4 * d), np.float64)
    ns = 0
    ss = sa = sb = sn = None
    if split is not None:
        ss = np.ascontiguousarray(split[0], np.int32)
        sa = np.ascontiguousarray(split[1], np.int32)
        sb = np.ascontiguousarray(split[2], np.float64)
        sn = np.ascontiguousarray(split[3], np.int32)
        ns = len(ss)
    lohi = np.zeros(2 * d, np.float64) if bbox else None
    bad = np.zeros(1, np.int64)
    ptr = (lambda a: a.ctypes.data if a is not None else None)
    _check(load().pd_kd_pass(ctx.ptr, X.data_ptr(), dt, n, d, labels.data_ptr(),
                             1 if labels_zero else 0, ns, ptr(ss), ptr(sa), ptr(sb), ptr(sn),
                             len(sel), sel.ctypes.data if len(sel) else None,
                             out.ctypes.data if len(sel) else None, ptr(lohi), bad.ctypes.data,
                             _stream(X.device)))
    if bbox:
        return out, lohi[:d], lohi[d:], int(bad[0])
    return out


PD_EUNSUPPORTED = -5
KD_TRACE = 13


def kd_build(X, labels, levels, final_split=True, ctx=None):
    """pd_kd_build: the whole min_var BFS in one launch chain.  levels: the
    BFS schedule (lists of (cur, new) label pairs).  final_split: True / 1
    apply the last split to `labels`, False / 0 leave it, 2 the labels are
    not needed (the passes replay the splits; kd_labels recovers them).
    Returns (lo, hi, bad, trace (n_splits, 13)); raises
    PardisError(PD_EUNSUPPORTED) when the fused path does not apply."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n, d = X.shape
    sizes = np.array([len(lv) for lv in levels], np.int32)
    cur = np.array([c for lv in levels for c, _ in lv], np.int32)
    new = np.array([nl for lv in levels for _, nl in lv], np.int32)
    trace = np.zeros((len(cur), KD_TRACE), np.float64)
    lohi = np.zeros(2 * d, np.float64)
    bad = np.zeros(1, np.int64)
    _check(load().pd_kd_build(ctx.ptr, X.data_ptr(), dt, n, d, labels.data_ptr(), len(sizes),
                              sizes.ctypes.data, cur.ctypes.data, new.ctypes.data,
                              2 if final_split == 2 else int(bool(final_split)),
                              trace.ctypes.data, lohi.ctypes.data, bad.ctypes.data,
                              _stream(X.device)))
    return lohi[:d], lohi[d:], int(bad[0]), trace


def kd_labels(X, labels, tree, ctx=None):
    """pd_kd_labels: every point's KD label by replaying a finished split
    tree (sizes, cur, axis, boundary, new) — KDPartitioner.split_tree()."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n, d = X.shape
    sizes, cur, axis, bound, new = (np.ascontiguousarray(a) for a in tree)
    sizes, cur, axis, new = (a.astype(np.int32) for a in (sizes, cur, axis, new))
    bound = bound.astype(np.float64)
    _check(load().pd_kd_labels(ctx.ptr, X.data_ptr(), dt, n, d, labels.data_ptr() if n else None,
                               len(sizes), sizes.ctypes.data, cur.ctypes.data, axis.ctypes.data,
                               bound.ctypes.data, new.ctypes.data, _stream(X.device)))
    return labels


def round_dd(dd):
    """(S, 1 + 4d) double-double partials of one device -> (S, 3, d) moments
    {count, sum v, sum v^2}, each rounded once (hi + lo)."""
    dd = np.asarray(dd, np.float64)
    S, G = dd.shape
    d = (G - 1) // 4
    mom = np.empty((S, 3, d))
    mom[:, 0, :] = dd[:, :1]
    mom[:, 1, :] = dd[:, 1:1 + 2 * d:2] + dd[:, 2:2 + 2 * d:2]
    mom[:, 2, :] = dd[:, 1 + 2 * d::2] + dd[:, 2 + 2 * d::2]
    return mom


def kd_radix_hist(X, labels, sel, axis, prefix, shift, ctx=None):
    """One radix-select pass (pd_kd_radix_hist): (n_sel, 256) int64 digit
    histogram of the order keys of v[axis] under each slot's prefix."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    sel = np.ascontiguousarray(sel, np.int32)
    axis = np.ascontiguousarray(axis, np.int32)
    prefix = np.ascontiguousarray(prefix, np.uint64)
    out = np.zeros((len(sel), 256), np.int64)
    _check(load().pd_kd_radix_hist(ctx.ptr, X.data_ptr(), dt, X.shape[0], X.shape[1],
                                   labels.data_ptr(), len(sel), sel.ctypes.data,
                                   axis.ctypes.data, prefix.ctypes.data, int(shift),
                                   out.ctypes.data, _stream(X.device)))
    return out


def halo_members(X, ebox, ctx=None):
    """ebox: (P, 2, d) fp64.  Returns (counts[P], members int64 device tensor)."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    ebox = np.ascontiguousarray(ebox, np.float64)
    P = ebox.shape[0]
    counts = np.zeros(P, np.int64)
    lib = load()
    _check(lib.pd_halo_members(ctx.ptr, X.data_ptr(), dt, X.shape[0], X.shape[1], P,
                               ebox.ctypes.data, counts.ctypes.data, None, 0, _stream(X.device)))
    total = int(counts.sum())
    members = torch.empty(max(total, 1), dtype=torch.int64, device=X.device)
    _check(lib.pd_halo_members(ctx.ptr, X.data_ptr(), dt, X.shape[0], X.shape[1], P,
                               ebox.ctypes.data, counts.ctypes.data, members.data_ptr(), total,
                               _stream(X.device)))
    return counts, members[:total]


def cluster(X, eps, min_samples, metric=PD_EUCLIDEAN, want_counts=False, ctx=None):
    """sklearn fit_predict semantics on one point set (device tensors out)."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n = X.shape[0]
    labels = torch.empty(n, dtype=torch.int32, device=X.device)
    core = torch.empty(n, dtype=torch.uint8, device=X.device)
    counts = torch.empty(n, dtype=torch.int32, device=X.device) if want_counts else None
    ncl = np.zeros(1, np.int64)
    _check(load().pd_cluster(ctx.ptr, X.data_ptr(), dt, n, X.shape[1], float(eps),
                             int(min_samples), int(metric), labels.data_ptr(), core.data_ptr(),
                             counts.data_ptr() if counts is not None else None,
                             ncl.ctypes.data, _stream(X.device)))
    return labels, core, counts, int(ncl[0])


def train(X, eps, min_samples, metric, ebox, owner=None, data_box=None, want_counts=False,
          out=None, ctx=None):
    """The fused per-device pipeline (pd_train).  ebox: (P, 2, d) fp64."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n, d = X.shape
    ebox = np.ascontiguousarray(ebox, np.float64)
    P = ebox.shape[0]
    if out is None:
        labels = torch.empty(n, dtype=torch.int32, device=X.device)
        core = torch.empty(n, dtype=torch.uint8, device=X.device)
    else:
        labels, core = out
    counts = torch.empty(n, dtype=torch.int32, device=X.device) if want_counts else None
    dbox = None
    if data_box is not None:
        dbox = np.ascontiguousarray(data_box, np.float64).reshape(2 * d)
    ncl = np.zeros(1, np.int64)
    _check(load().pd_train(ctx.ptr, X.data_ptr(), dt, n, d, float(eps), int(min_samples),
                           int(metric), P, ebox.ctypes.data,
                           dbox.ctypes.data if dbox is not None else None,
                           owner.data_ptr() if owner is not None else None, labels.data_ptr(),
                           core.data_ptr(), counts.data_ptr() if counts is not None else None,
                           ncl.ctypes.data, _stream(X.device)))
    return labels, core, counts, int(ncl[0])


def train_tree(X, eps, min_samples, metric, ebox, tree, data_box=None, want_counts=False,
               ctx=None):
    """pd_train_tree: pd_train with the KD split tree (sizes, cur, axis,
    boundary, new) replayed per point instead of owner labels."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n, d = X.shape
    ebox = np.ascontiguousarray(ebox, np.float64)
    sizes, cur, axis, bound, new = (np.ascontiguousarray(tree[0], np.int32),
                                    np.ascontiguousarray(tree[1], np.int32),
                                    np.ascontiguousarray(tree[2], np.int32),
                                    np.ascontiguousarray(tree[3], np.float64),
                                    np.ascontiguousarray(tree[4], np.int32))
    labels = torch.empty(n, dtype=torch.int32, device=X.device)
    core = torch.empty(n, dtype=torch.uint8, device=X.device)
    counts = torch.empty(n, dtype=torch.int32, device=X.device) if want_counts else None
    dbox = None if data_box is None else np.ascontiguousarray(data_box, np.float64).reshape(2 * d)
    ncl = np.zeros(1, np.int64)
    _check(load().pd_train_tree(ctx.ptr, X.data_ptr(), dt, n, d, float(eps), int(min_samples),
                                int(metric), ebox.shape[0], ebox.ctypes.data,
                                dbox.ctypes.data if dbox is not None else None, len(sizes),
                                sizes.ctypes.data, cur.ctypes.data, axis.ctypes.data,
                                bound.ctypes.data, new.ctypes.data, labels.data_ptr(),
                                core.data_ptr(), counts.data_ptr() if counts is not None else None,
                                ncl.ctypes.data, _stream(X.device)))
    return labels, core, counts, int(ncl[0])


# ------------------------------------------------------- sharded train stages
# u32 ids/keys live in int32 tensors (same bits; 0xFFFFFFFF reads as -1), the
# u64 route mask in an int64 tensor: both move through torch.distributed as is.
KEY_NONE = -1


def kd_moments_dd(X, labels, sel, ctx=None):
    """(n_sel, 1 + 4d) unrounded double-double partials (pd_kd_moments_dd)."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    d = X.shape[1]
    sel = np.ascontiguousarray(sel, np.int32)
    out = np.zeros((len(sel), 1 + 4 * d), np.float64)
    _check(load().pd_kd_moments_dd(ctx.ptr, X.data_ptr(), dt, X.shape[0], d, labels.data_ptr(),
                                   len(sel), sel.ctypes.data, out.ctypes.data, _stream(X.device)))
    return out


def route(X, ebox, part_rank, n_ranks, ctx=None):
    """Returns (mask int64[n] device, counts int64[n_ranks] host)."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n, d = X.shape
    ebox = np.ascontiguousarray(ebox, np.float64)
    part_rank = np.ascontiguousarray(part_rank, np.int32)
    mask = torch.empty(max(n, 1), dtype=torch.int64, device=X.device)
    counts = np.zeros(n_ranks, np.int64)
    _check(load().pd_route(ctx.ptr, X.data_ptr(), dt, n, d, ebox.shape[0], ebox.ctypes.data,
                           part_rank.ctypes.data, int(n_ranks), mask.data_ptr(),
                           counts.ctypes.data, _stream(X.device)))
    return mask[:n], counts


def pack(X, mask, dest, kdlab, part_rank, local_index, gid_base, out, ctx=None):
    """Fill out = (coords (m, d), gid int32[m], owner int32[m], xr uint8[m]) views
    with the points routed to `dest`; returns m."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n, d = X.shape
    coords, gid, owner, xr = out
    cap = gid.shape[0]
    part_rank = np.ascontiguousarray(part_rank, np.int32)
    local_index = np.ascontiguousarray(local_index, np.int32)
    m = np.zeros(1, np.int64)
    ptr = (lambda t: t.data_ptr() if t.numel() else None)
    _check(load().pd_pack(ctx.ptr, X.data_ptr() if n else None, dt, n, d,
                          mask.data_ptr() if n else None, int(dest),
                          kdlab.data_ptr() if n else None, len(part_rank),
                          part_rank.ctypes.data, local_index.ctypes.data, int(gid_base),
                          ptr(coords), ptr(gid), ptr(owner), ptr(xr), cap, m.ctypes.data,
                          _stream(X.device)))
    return int(m[0])


# ---- device-decided sharded KD (pd_kdx_*): tensors stay on the device
def _ptr(t):
    return t.data_ptr() if t is not None and t.numel() else None


def kdx_begin(d, levels, device, ctx=None):
    ctx = ctx or context(device)
    sizes = np.array([len(lv) for lv in levels], np.int32)
    cur = np.array([c for lv in levels for c, _ in lv], np.int32)
    new = np.array([nl for lv in levels for _, nl in lv], np.int32)
    _check(load().pd_kdx_begin(ctx.ptr, int(d), len(levels), sizes.ctypes.data, cur.ctypes.data,
                               new.ctypes.data, _stream(device)))


def kdx_part_len(S, d, level):
    return S * (1 + 4 * d) + (2 * d + 1 if level == 0 else 0)


def kdx_moments(X, labels, level, S, ctx=None):
    """This slice's moment partials of level `level` (device float64)."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n, d = X.shape
    out = torch.empty(kdx_part_len(S, d, level), dtype=torch.float64, device=X.device)
    _check(load().pd_kdx_moments(ctx.ptr, X.data_ptr() if n else None, dt, n, d, _ptr(labels),
                                 int(level), out.data_ptr(), _stream(X.device)))
    return out


def kdx_axes(gathered, n_ranks, level, ctx=None):
    g = gathered.contiguous()
    ctx = ctx or context(g.device.index)
    _check(load().pd_kdx_axes(ctx.ptr, g.data_ptr(), int(n_ranks), int(level), _stream(g.device)))


def kdx_counts(X, labels, level, S, ctx=None):
    """This slice's n_less / n per split of the level (device int64, S x 8)."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n, d = X.shape
    out = torch.empty(8 * S, dtype=torch.int64, device=X.device)
    _check(load().pd_kdx_counts(ctx.ptr, X.data_ptr() if n else None, dt, n, d, _ptr(labels),
                                int(level), out.data_ptr(), _stream(X.device)))
    return out


def kdx_boundary(counts, level, ctx=None):
    c = counts.contiguous()
    ctx = ctx or context(c.device.index)
    _check(load().pd_kdx_boundary(ctx.ptr, c.data_ptr(), int(level), _stream(c.device)))


def kdx_end(X, labels, n_splits, final_split, ctx=None):
    """-> (trace (n_splits, 13), lo, hi, non-finite count) on the host."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n, d = X.shape
    trace = np.zeros((n_splits, 13), np.float64)
    lohi = np.zeros(2 * d, np.float64)
    bad = np.zeros(1, np.int64)
    _check(load().pd_kdx_end(ctx.ptr, X.data_ptr() if n else None, dt, n, d, _ptr(labels),
                             1 if final_split else 0, trace.ctypes.data, lohi.ctypes.data,
                             bad.ctypes.data, _stream(X.device)))
    return trace, lohi[:d].copy(), lohi[d:].copy(), int(bad[0])


def route2(X, ebox, part_rank, kdlab, n_ranks, ctx=None):
    """Destination masks (kept in the context for pack2) and per rank
    (points routed there, of which it owns) — int64 (n_ranks, 2), host."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n, d = X.shape
    ebox = np.ascontiguousarray(ebox, np.float64)
    part_rank = np.ascontiguousarray(part_rank, np.int32)
    counts = np.zeros((n_ranks, 2), np.int64)
    _check(load().pd_route2(ctx.ptr, X.data_ptr() if n else None, dt, n, d, ebox.shape[0],
                            ebox.ctypes.data, part_rank.ctypes.data, _ptr(kdlab), int(n_ranks),
                            counts.ctypes.data, _stream(X.device)))
    return counts


def pack2(X, kdlab, part_rank, local_index, gid_base, outs, ctx=None):
    """outs[r] = (coords (m_r, d), gid int32[m_r], owner int32[m_r], xr uint8[m_r])
    device views, one per rank (after route2 on the same context)."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n, d = X.shape
    W = len(outs)
    part_rank = np.ascontiguousarray(part_rank, np.int32)
    local_index = np.ascontiguousarray(local_index, np.int32)
    tabs = [np.array([_ptr(o[f]) or 0 for o in outs], np.uint64) for f in range(4)]
    _check(load().pd_pack2(ctx.ptr, X.data_ptr() if n else None, dt, n, d, _ptr(kdlab),
                           len(part_rank), part_rank.ctypes.data, local_index.ctypes.data,
                           int(gid_base), W, tabs[0].ctypes.data, tabs[1].ctypes.data,
                           tabs[2].ctypes.data, tabs[3].ctypes.data, _stream(X.device)))


def results(keys, core, owner, gid, roots, n_total, gid_base, n_local, n_ranks, rank, src_off,
            expect_remote, device, ctx=None):
    """Labels / core flags of this rank's points from the owned records of its
    own block; the other owned records as (gid, (label + 1) | core << 31)
    pairs, block by block.  -> (labels int32[n_local], core uint8[n_local],
    pairs int32 (expect_remote, 2)), all on the device."""
    ctx = ctx or context(device)
    nr = keys.shape[0]
    labels = torch.empty(max(n_local, 1), dtype=torch.int32, device=device)
    core_out = torch.empty(max(n_local, 1), dtype=torch.uint8, device=device)
    pairs = torch.empty((max(expect_remote, 1), 2), dtype=torch.int32, device=device)
    src = np.ascontiguousarray(src_off, np.int64)
    _check(load().pd_results(ctx.ptr, nr, _ptr(keys), _ptr(core), _ptr(owner), _ptr(gid),
                             _ptr(roots), roots.shape[0], int(n_total), int(gid_base),
                             int(n_local), int(n_ranks), int(rank), src.ctypes.data,
                             int(expect_remote), labels.data_ptr(), core_out.data_ptr(),
                             pairs.data_ptr(), _stream(device)))
    return labels[:n_local], core_out[:n_local], pairs[:expect_remote]


def results_scatter(pairs, gid_base, labels, core, ctx=None):
    device = labels.device
    ctx = ctx or context(device.index)
    m = pairs.shape[0]
    p = pairs.contiguous()
    _check(load().pd_results_scatter(ctx.ptr, _ptr(p), m, int(gid_base), labels.shape[0],
                                     _ptr(labels), _ptr(core), _stream(device)))


def train_begin(X, eps, min_samples, metric, ebox, owner, gid, xr, data_box, ctx=None):
    """Phase A of a sharded train; returns the number of exports."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n, d = X.shape
    ebox = np.ascontiguousarray(ebox, np.float64).reshape(-1, 2, d)
    dbox = np.ascontiguousarray(data_box, np.float64).reshape(2 * d)
    ne = np.zeros(1, np.int64)
    _check(load().pd_train_begin(ctx.ptr, X.data_ptr() if n else None, dt, n, d, float(eps),
                                 int(min_samples), int(metric), ebox.shape[0], ebox.ctypes.data,
                                 dbox.ctypes.data, owner.data_ptr() if n else None,
                                 _ptr(gid) if n else None, _ptr(xr) if n else None,
                                 ne.ctypes.data, _stream(X.device)))
    return int(ne[0])


def train_exports(m, device, ctx=None):
    """(gid int32[m], key int32[m]) device tensors of the last train_begin."""
    ctx = ctx or context(device)
    gid = torch.empty(max(m, 1), dtype=torch.int32, device=device)
    key = torch.empty(max(m, 1), dtype=torch.int32, device=device)
    _check(load().pd_train_exports(ctx.ptr, gid.data_ptr(), key.data_ptr(), m, _stream(device)))
    return gid[:m], key[:m]


def merge_exports(gid, key, ctx=None):
    """Union of all devices' exports: (ids, keys) int32 device tensors — the
    distinct ids named, ascending (u32 order), and each one's global key."""
    device = gid.device
    ctx = ctx or context(device.index)
    m = gid.shape[0]
    ids = torch.empty(max(2 * m, 1), dtype=torch.int32, device=device)
    keys = torch.empty(max(2 * m, 1), dtype=torch.int32, device=device)
    u = np.zeros(1, np.int64)
    _check(load().pd_merge_exports(ctx.ptr, gid.data_ptr() if m else None,
                                   key.data_ptr() if m else None, m, ids.data_ptr(),
                                   keys.data_ptr(), u.ctypes.data, _stream(device)))
    return ids[:int(u[0])], keys[:int(u[0])]


def train_end(n, keymap, device, ctx=None):
    """Phase B: (keys int32[n], core uint8[n]) device tensors (owned points).
    keymap: (ids, keys) from merge_exports, or None."""
    ctx = ctx or context(device)
    keys = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    core = torch.empty(max(n, 1), dtype=torch.uint8, device=device)
    ids, mk = keymap if keymap is not None else (None, None)
    nm = 0 if ids is None else ids.shape[0]
    _check(load().pd_train_end(ctx.ptr, n, ids.data_ptr() if nm else None,
                               mk.data_ptr() if nm else None, nm, keys.data_ptr(),
                               core.data_ptr(), _stream(device)))
    return keys[:n], core[:n]


def select_roots(keys, gid, ctx=None):
    device = keys.device
    ctx = ctx or context(device.index)
    n = keys.shape[0]
    roots = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    m = np.zeros(1, np.int64)
    _check(load().pd_select_roots(ctx.ptr, keys.data_ptr() if n else None,
                                  _ptr(gid) if n else None, n, roots.data_ptr(),
                                  m.ctypes.data, _stream(device)))
    return roots[:int(m[0])]


def sort_u32(data, ctx=None):
    """In-place ascending sort (u32 order) of an int32 device tensor."""
    ctx = ctx or context(data.device.index)
    n = data.shape[0]
    _check(load().pd_sort_u32(ctx.ptr, data.data_ptr() if n else None, n, _stream(data.device)))
    return data


def sort_pairs(keys, vals, key_bits, ctx=None):
    """pd_sort_pairs: stable in-place sort of (keys, vals) by key bits [0,
    key_bits) — the train's record sort.  keys: int32 / int64 device tensor
    (unsigned order), vals: int32 device tensor of the same length."""
    ctx = ctx or context(keys.device.index)
    n = keys.shape[0]
    if vals.shape[0] != n or vals.dtype != torch.int32 or keys.dtype not in (torch.int32, torch.int64):
        raise TypeError("keys int32/int64 and vals int32 of one length")
    _check(load().pd_sort_pairs(ctx.ptr, keys.data_ptr() if n else None, keys.element_size(),
                                vals.data_ptr() if n else None, n, int(key_bits),
                                _stream(keys.device)))
    return keys, vals


def rank_labels(keys, roots, ctx=None):
    device = keys.device
    ctx = ctx or context(device.index)
    n, nr = keys.shape[0], roots.shape[0]
    labels = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    _check(load().pd_rank_labels(ctx.ptr, keys.data_ptr() if n else None, n,
                                 roots.data_ptr() if nr else None, nr, labels.data_ptr(),
                                 _stream(device)))
    return labels[:n]


def owned_results(owner, gid, labels, core, gid_offsets, ctx=None):
    """(pairs int32[m, 2] device, counts int64[W] host): the owned records as
    (gid, (label + 1) | core << 31), grouped by the device holding the point."""
    device = gid.device
    ctx = ctx or context(device.index)
    n = gid.shape[0]
    off = np.ascontiguousarray(gid_offsets, np.int64)
    W = len(off) - 1
    out = torch.empty((max(n, 1), 2), dtype=torch.int32, device=device)
    counts = np.zeros(W, np.int64)
    m = np.zeros(1, np.int64)
    ptr = (lambda t: t.data_ptr() if t is not None and n else None)
    _check(load().pd_owned_results(ctx.ptr, n, ptr(owner), ptr(gid), ptr(labels), ptr(core), W,
                                   off.ctypes.data, out.data_ptr(), n, counts.ctypes.data,
                                   m.ctypes.data, _stream(device)))
    return out[:int(m[0])], counts


def scatter_results(pairs, gid_base, n, device, ctx=None):
    """(labels int32[n], core uint8[n]) of this device's input points."""
    ctx = ctx or context(device.index)
    labels = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    core = torch.empty(max(n, 1), dtype=torch.uint8, device=device)
    m = pairs.shape[0]
    _check(load().pd_scatter_results(ctx.ptr, pairs.data_ptr() if m else None, m, int(gid_base),
                                     n, labels.data_ptr(), core.data_ptr(), _stream(device)))
    return labels[:n], core[:n]


# ------------------------------------------------------------------ RCCL
PD_COMM_ID_BYTES = 128
# ------------------------------------------------ sharded dense train (d > 4)
def dense_count(X, eps, min_samples, metric, data_box, rank, world, ctx=None):
    """Stage 1 (pd_dense_count): int32[n] counts of this rank's rows, 0 elsewhere.
    X (all n points) must stay alive until dense_finish."""
    dt = _check_points(X)
    ctx = ctx or context(X.device.index)
    n, d = X.shape
    dbox = np.ascontiguousarray(data_box, np.float64).reshape(2 * d)
    counts = torch.empty(max(n, 1), dtype=torch.int32, device=X.device)
    _check(load().pd_dense_count(ctx.ptr, X.data_ptr() if n else None, dt, n, d, float(eps),
                                 int(min_samples), int(metric), dbox.ctypes.data, int(rank),
                                 int(world), counts.data_ptr(), _stream(X.device)))
    return counts[:n]


def dense_link(counts, ctx=None):
    """Stage 2 (pd_dense_link): this rank's forest over the core rows, int32[n_core]."""
    device = counts.device
    ctx = ctx or context(device.index)
    n = counts.shape[0]
    forest = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    mc = np.zeros(1, np.int64)
    _check(load().pd_dense_link(ctx.ptr, counts.contiguous().data_ptr() if n else None,
                                forest.data_ptr(), mc.ctypes.data, _stream(device)))
    return forest[:int(mc[0])]


def dense_border(forests, n_forests, n, ctx=None):
    """Stage 3 (pd_dense_border): int32[n_border] smallest adjacent core key per
    border candidate (INT32_MAX: none, or not this rank's row)."""
    device = forests.device
    ctx = ctx or context(device.index)
    best = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    mb = np.zeros(1, np.int64)
    f = forests.contiguous()
    _check(load().pd_dense_border(ctx.ptr, f.data_ptr() if f.numel() else None, int(n_forests),
                                  best.data_ptr(), mb.ctypes.data, _stream(device)))
    return best[:int(mb[0])]


def dense_finish(best, n, device, want_counts=False, ctx=None):
    """Stage 4 (pd_dense_finish): (labels int32[n], core uint8[n], counts or
    None, n_clusters) over all points."""
    ctx = ctx or context(device)
    labels = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    core = torch.empty(max(n, 1), dtype=torch.uint8, device=device)
    counts = torch.empty(max(n, 1), dtype=torch.int32, device=device) if want_counts else None
    ncl = np.zeros(1, np.int64)
    b = best.contiguous()
    _check(load().pd_dense_finish(ctx.ptr, b.data_ptr() if b.numel() else None,
                                  labels.data_ptr(), core.data_ptr(),
                                  counts.data_ptr() if counts is not None else None,
                                  ncl.ctypes.data, _stream(device)))
    return labels[:n], core[:n], (counts[:n] if counts is not None else None), int(ncl[0])


PD_R_SUM, PD_R_MAX, PD_R_MIN = 0, 1, 2
_ELEM = {torch.uint8: 0, torch.bool: 0, torch.int32: 1, torch.int64: 3, torch.float32: 5,
         torch.float64: 6}


def comm_unique_id():
    buf = (ctypes.c_uint8 * PD_COMM_ID_BYTES)()
    _check(load().pd_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p)))
    return bytes(buf)


class Comm:
    """One rank of an RCCL communicator (pd_comm_*).  Device tensors in and
    out, on this rank's device and the current stream."""

    def __init__(self, ptr, device, n_ranks, rank):
        self.ptr = ptr
        self.device = torch.device("cuda", int(device))
        self.world = int(n_ranks)
        self.rank = int(rank)

    @classmethod
    def init(cls, n_ranks, rank, uid, device):
        ctx = context(device)
        buf = (ctypes.c_uint8 * PD_COMM_ID_BYTES).from_buffer_copy(uid)
        ptr = ctypes.c_void_p()
        _check(load().pd_comm_init(ctx.ptr, int(n_ranks), int(rank),
                                   ctypes.cast(buf, ctypes.c_void_p), ctypes.byref(ptr)))
        return cls(ptr, device, n_ranks, rank)

    @classmethod
    def init_all(cls, devices):
        devs = np.ascontiguousarray(devices, np.int32)
        ptrs = (ctypes.c_void_p * len(devs))()
        require_gpu()
        _check(load().pd_comm_init_all(len(devs), devs.ctypes.data,
                                       ctypes.cast(ptrs, ctypes.c_void_p)))
        return [cls(ctypes.c_void_p(ptrs[i]), int(devs[i]), len(devs), i)
                for i in range(len(devs))]

    def destroy(self):
        if self.ptr:
            load().pd_comm_destroy(self.ptr)
            self.ptr = None

    def _elem(self, t):
        if t.dtype not in _ELEM:
            raise TypeError(f"no RCCL element type for {t.dtype}")
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("RCCL buffers must be contiguous device tensors")
        return _ELEM[t.dtype]

    def all_reduce(self, t, op=PD_R_SUM):
        """In place."""
        _check(load().pd_comm_all_reduce(self.ptr, t.data_ptr(), t.data_ptr(), t.numel(),
                                         self._elem(t), int(op), _stream(self.device)))
        return t

    def all_gather_v(self, t, counts):
        """Concatenation over ranks of counts[r] rows of t's row shape."""
        row = int(np.prod(t.shape[1:])) if t.dim() > 1 else 1
        c = np.ascontiguousarray(np.asarray(counts, np.int64) * row)
        out = torch.empty((int(np.sum(counts)),) + tuple(t.shape[1:]), dtype=t.dtype,
                          device=self.device)
        if out.numel() == 0:
            return out
        _check(load().pd_comm_all_gather_v(self.ptr, t.data_ptr() if t.numel() else None,
                                           out.data_ptr(), c.ctypes.data, self._elem(out),
                                           _stream(self.device)))
        return out

    def all_to_all_v(self, send, send_counts, recv_counts):
        """send rows grouped by destination; returns rows grouped by source."""
        row = int(np.prod(send.shape[1:])) if send.dim() > 1 else 1
        sc = np.ascontiguousarray(np.asarray(send_counts, np.int64) * row)
        rc = np.ascontiguousarray(np.asarray(recv_counts, np.int64) * row)
        out = torch.empty((int(np.sum(recv_counts)),) + tuple(send.shape[1:]), dtype=send.dtype,
                          device=self.device)
        _check(load().pd_comm_all_to_all_v(self.ptr, send.data_ptr() if send.numel() else None,
                                           sc.ctypes.data,
                                           out.data_ptr() if out.numel() else None,
                                           rc.ctypes.data, self._elem(send),
                                           _stream(self.device)))
        return out

    def exchange(self, sends, recvs, send_counts, recv_counts, skip_self=True):
        """Fields exchanged in one group: sends[f] rows grouped by destination
        (send_counts), recvs[f] rows grouped by source (recv_counts); with
        skip_self the self block is already in place in recvs[f]."""
        W = self.world
        sc = np.ascontiguousarray(send_counts, np.int64)
        rc = np.ascontiguousarray(recv_counts, np.int64)
        # send buffers hold the other ranks' blocks only when the self block
        # was packed in place
        se = sc.copy()
        if skip_self:
            se[self.rank] = 0
        so = np.ascontiguousarray(np.concatenate([[0], np.cumsum(se)[:-1]]), np.int64)
        ro = np.ascontiguousarray(np.concatenate([[0], np.cumsum(rc)[:-1]]), np.int64)
        rb = np.array([t.element_size() * (int(np.prod(t.shape[1:])) if t.dim() > 1 else 1)
                       for t in recvs], np.int64)
        sp = np.array([_ptr(t) or 0 for t in sends], np.uint64)
        rp = np.array([_ptr(t) or 0 for t in recvs], np.uint64)
        if len(sends) != len(recvs) or len(sc) != W or len(rc) != W:
            raise ValueError("exchange: one send and one recv per field, counts per rank")
        _check(load().pd_comm_exchange(self.ptr, len(sends), sp.ctypes.data, rp.ctypes.data,
                                       rb.ctypes.data, sc.ctypes.data, so.ctypes.data,
                                       rc.ctypes.data, ro.ctypes.data, 1 if skip_self else 0,
                                       _stream(self.device)))

    def abort(self):
        if self.ptr:
            load().pd_comm_abort(self.ptr)

    def self_check(self):
        _check(load().pd_comm_self_check(self.ptr))

    def broadcast(self, t, root=0):
        _check(load().pd_comm_broadcast(self.ptr, t.data_ptr(), t.numel(), self._elem(t),
                                        int(root), _stream(self.device)))
        return t

    def size(self):
        """(n_ranks, rank) as RCCL reports them (ncclCommCount / ncclCommUserRank)."""
        n, r = ctypes.c_int32(0), ctypes.c_int32(-1)
        _check(load().pd_comm_size(self.ptr, ctypes.byref(n), ctypes.byref(r)))
        return int(n.value), int(r.value)
