"""Ingestion: every input form the reference's ``train`` / ``KDPartitioner``
would be fed, turned into one device-resident point set.

The reference takes an RDD of ``(key, k-dim vector)`` (R:dbscan/dbscan.py:104-109,
R:dbscan/partition.py:111-121).  Accepted here:
  * an RDD-like object (anything with ``collect()``, e.g. a pyspark RDD),
  * an iterable of ``(key, vector)`` pairs,
  * a numpy array or torch tensor of shape (n, d) — keys are 0..n-1,
  * a ``(keys, X)`` tuple,
  * a ``PointSet`` (passed through).
float32 inputs stay float32, float64 stay float64 (the predicate is exact for
either); anything else becomes float64.
"""
from __future__ import annotations

from operator import itemgetter

import numpy as np
import torch


class PointSet:
    """keys (host numpy, or None meaning 0..n-1) + X (CUDA tensor, (n, d))."""

    def __init__(self, X, keys=None):
        self.X = X
        self.keys = keys

    @property
    def n(self):
        return int(self.X.shape[0])

    @property
    def d(self):
        return int(self.X.shape[1])

    def key_array(self):
        return np.arange(self.n, dtype=np.int64) if self.keys is None else self.keys

    def vectors(self, idx=None):
        """Host copies of the vectors (API views only, never the hot path)."""
        X = self.X if idx is None else self.X[idx]
        return X.cpu().numpy()


def _device(device):
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(device) if not isinstance(device, torch.device) else device


def _to_tensor(X, device):
    if isinstance(X, torch.Tensor):
        t = X
    else:
        a = np.asarray(X)
        if a.dtype not in (np.float32, np.float64):
            a = a.astype(np.float64)
        t = torch.from_numpy(np.ascontiguousarray(a))
    if t.dtype not in (torch.float32, torch.float64):
        t = t.to(torch.float64)
    if t.dim() == 1:
        t = t.reshape(-1, 1)
    if t.dim() != 2:
        raise ValueError(f"expected (n, d) points, got shape {tuple(t.shape)}")
    return t.to(device).contiguous()


def _keys(keys):
    if isinstance(keys, torch.Tensor):
        keys = keys.detach().cpu().numpy()
    try:
        a = np.asarray(keys)
        if a.dtype.kind in "iu":
            return a.astype(np.int64)
    except Exception:
        pass
    a = np.empty(len(keys), dtype=object)
    a[:] = list(keys)
    return a


def _is_keys_and_matrix(data):
    """A ``(keys, X)`` pair: X is an array/tensor of points (ndim 1 or 2) and
    keys a sequence of scalars of the same length.  A tuple of two (key,
    vector) records is not one: its second element is a record, not a
    matrix."""
    if not (isinstance(data, tuple) and len(data) == 2):
        return False
    keys, X = data
    if not isinstance(X, (np.ndarray, torch.Tensor)) or X.ndim not in (1, 2):
        return False
    if isinstance(keys, (np.ndarray, torch.Tensor)):
        # a 1-D key array (its elements are 0-d arrays / tensors, not scalars)
        return keys.ndim == 1 and len(keys) == len(X)
    try:
        return len(keys) == len(X) and all(np.isscalar(k) for k in keys[:8])
    except TypeError:
        return False


def as_points(data, device=None):
    if isinstance(data, PointSet):
        return data
    dev = _device(device)
    if isinstance(data, (torch.Tensor, np.ndarray)):
        return PointSet(_to_tensor(data, dev))
    if _is_keys_and_matrix(data):
        keys, X = data
        return PointSet(_to_tensor(X, dev), _keys(keys))
    recs = data.collect() if hasattr(data, "collect") else data
    if not isinstance(recs, (list, tuple)):
        recs = list(recs)
    if not recs:
        raise ValueError("no points")
    got = _unzip_native(recs)
    if got is not None:
        X, k = got
        return PointSet(_to_tensor(X, dev), _dense_or(k))
    # unzip of the (key, vector) records: itemgetter maps (an order of
    # magnitude faster than zip(*recs)), one concatenate for equal-length
    # vectors
    keys = list(map(itemgetter(0), recs))
    vecs = list(map(itemgetter(1), recs))
    X = None
    if np.ndim(vecs[0]) == 1 and len(set(map(len, vecs))) == 1:
        try:
            X = np.concatenate(vecs).reshape(len(vecs), -1)
        except (ValueError, TypeError):
            X = None
    if X is None:
        X = np.asarray(vecs)
        if X.dtype == object or X.ndim not in (1, 2):
            X = np.stack([np.asarray(v) for v in vecs])
    # float32 stays float32 only if every vector is float32 (np.asarray of
    # a mixed list already promotes); anything else becomes float64
    if X.dtype not in (np.float32, np.float64):
        X = X.astype(np.float64)
    return PointSet(_to_tensor(X, dev), _dense_or(_keys(keys)))


def _dense_or(k):
    """None for the keys 0..n-1 (the implicit key array), else k."""
    if k.dtype == np.int64 and len(k) and k[0] == 0 and np.array_equal(k, np.arange(len(k))):
        return None
    return k


def _unzip_native(recs):
    """(X, keys) from csrc/ingest.cpp's one-pass unzip, or None when the
    extension is not built or the records are not uniform (key, 1-D vector)
    pairs — the numpy path below then handles (or rejects) them."""
    try:
        from . import _ingest
    except ImportError:
        return None
    try:
        v0 = recs[0][1]
        if np.ndim(v0) != 1:
            return None
        d = len(v0)
        if d < 1:
            return None
        n = len(recs)
        K = np.empty(n, dtype=np.int64)
        f64 = 0 if getattr(v0, "dtype", None) == np.float32 else 1
        X = np.empty((n, d), dtype=np.float64 if f64 else np.float32)
        st = _ingest.unzip(recs, X, K, d, f64)
        if st == 2:   # a non-float32 vector: the set is float64
            X = np.empty((n, d), dtype=np.float64)
            st = _ingest.unzip(recs, X, K, d, 1)
    except (TypeError, ValueError, IndexError):
        return None
    keys = K if st & 1 else _keys(list(map(itemgetter(0), recs)))
    return X, keys
