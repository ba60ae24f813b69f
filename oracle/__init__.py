"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's hot path, used as the checker by tests/,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg.  The
product package (``pypardis_amd``) never imports it and has no CPU fallback.

Pieces (each cites the reference line it restates):

* ``dbscan``      — sklearn ``DBSCAN.fit`` semantics, in C (dbscan_oracle.c).
* ``kd_partition``— ``KDPartitioner`` + ``min_var_split``/``mean_var_split``
  (R:dbscan/partition.py:33-183) in numpy, with the reference's sequential
  fp64 sums so split boundaries match the shim-run reference bit for bit.
* ``halo``        — ``DBSCAN._create_neighborhoods`` (R:dbscan/dbscan.py:136-151).
* ``pipeline``    — KD → halo → per-neighbourhood DBSCAN → owner-rule merge;
  its labels equal global sklearn DBSCAN's exactly (pinned by the goldens).

Pinning: tests/test_oracle.py checks every function here against the
fixtures in tests/golden/ (made by tests/golden/make_golden.py from the
reference run under an RDD stand-in, and from scikit-learn 1.7.2).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

METRICS = {"euclidean": 0, "cityblock": 1, "manhattan": 1, "l2": 0, "l1": 1}


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE], stdout=sys.stderr)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        lib.oracle_counts.argtypes = [P, ctypes.c_int64, ctypes.c_int32, ctypes.c_double,
                                      ctypes.c_int32, P]
        lib.oracle_counts.restype = ctypes.c_int
        lib.oracle_neighbors.argtypes = [P, ctypes.c_int64, ctypes.c_int32, ctypes.c_double,
                                         ctypes.c_int32, P, P]
        lib.oracle_neighbors.restype = ctypes.c_int
        lib.oracle_dbscan.argtypes = [P, ctypes.c_int64, ctypes.c_int32, ctypes.c_double,
                                      ctypes.c_int64, ctypes.c_int32, P, P, P]
        lib.oracle_dbscan.restype = ctypes.c_int64
        lib.oracle_counts_capped.argtypes = [P, ctypes.c_int64, P, ctypes.c_int64, ctypes.c_int32,
                                             ctypes.c_double, ctypes.c_int32, ctypes.c_int64, P]
        lib.oracle_counts_capped.restype = ctypes.c_int
        _lib = lib
    return _lib


def metric_id(metric):
    if callable(metric):
        name = getattr(metric, "__name__", "")
        metric = {"euclidean": "euclidean", "cityblock": "cityblock"}.get(name, name)
    if metric not in METRICS:
        raise ValueError(f"metric {metric!r} not supported (euclidean / cityblock)")
    return METRICS[metric]


def _as64(X):
    X = np.asarray(X)
    if X.ndim == 1:
        X = X[:, None]
    return np.ascontiguousarray(X, dtype=np.float64)


def counts(X, eps, metric="euclidean"):
    X = _as64(X)
    out = np.zeros(len(X), np.int64)
    rc = _load().oracle_counts(X.ctypes.data, len(X), X.shape[1], float(eps),
                               metric_id(metric), out.ctypes.data)
    assert rc == 0
    return out


def counts_capped(Q, C, eps, cap, metric="euclidean"):
    """min(#points of C within eps of each query, cap) by brute force (cap <= 0:
    exact counts).  With C holding every point within eps of the queries (the
    queries themselves included) this is the count sklearn's core test uses."""
    Q, C = _as64(Q), _as64(C)
    out = np.zeros(len(Q), np.int64)
    rc = _load().oracle_counts_capped(Q.ctypes.data, len(Q), C.ctypes.data, len(C), Q.shape[1],
                                      float(eps), metric_id(metric), int(cap), out.ctypes.data)
    assert rc == 0
    return out


def neighbors(X, eps, metric="euclidean"):
    """CSR neighbourhoods (self included, rows sorted)."""
    X = _as64(X)
    c = counts(X, eps, metric)
    off = np.zeros(len(X) + 1, np.int64)
    np.cumsum(c, out=off[1:])
    nbr = np.empty(max(int(off[-1]), 1), np.int64)
    rc = _load().oracle_neighbors(X.ctypes.data, len(X), X.shape[1], float(eps),
                                  metric_id(metric), off.ctypes.data, nbr.ctypes.data)
    assert rc == 0
    return off, nbr[: off[-1]]


def dbscan(X, eps, min_samples, metric="euclidean"):
    """sklearn DBSCAN(algorithm='kd_tree').fit → (labels int64, core uint8,
    counts int64, n_clusters)."""
    X = _as64(X)
    n = len(X)
    labels = np.empty(n, np.int64)
    core = np.empty(n, np.uint8)
    cnt = np.empty(n, np.int64)
    nc = _load().oracle_dbscan(X.ctypes.data, n, X.shape[1], float(eps), int(min_samples),
                               metric_id(metric), labels.ctypes.data, core.ctypes.data,
                               cnt.ctypes.data)
    assert nc >= 0
    return labels, core, cnt, int(nc)


# ---------------------------------------------------------------------------
# KD partition: R:dbscan/partition.py
# ---------------------------------------------------------------------------
FLT_MAX = sys.float_info.max
FLT_MIN = sys.float_info.min


def root_box(X):
    """``data.aggregate(BoundingBox(k=k), union, union)`` (R:dbscan/partition.py:135-137)
    with the empty-box sentinels of R:dbscan/geometry.py:28-29: lower starts at
    float_info.max and upper at float_info.min (+2.2e-308, not -max)."""
    X = np.asarray(X)
    k = X.shape[1]
    lo = np.full(k, FLT_MAX)
    hi = np.full(k, FLT_MIN)
    if len(X):
        lo = np.minimum(lo, X.min(axis=0).astype(np.float64))
        hi = np.maximum(hi, X.max(axis=0).astype(np.float64))
    return lo, hi


def split_schedule(max_partitions):
    """The BFS of R:dbscan/partition.py:159-183 as a list of levels; each level
    is a list of (current_label, next_label).  Left child keeps the label."""
    levels, todo, done, nxt = [], [0], [], 1
    cur_level = []
    while nxt < max_partitions:
        if todo:
            cur = todo.pop(0)
            cur_level.append((cur, nxt))
            done += [cur, nxt]
            nxt += 1
        else:
            levels.append(cur_level)
            cur_level = []
            todo, done = done, []
    if cur_level:
        levels.append(cur_level)
    return levels


def mean_var_bounds(mean, variance):
    """R:dbscan/partition.py:58-59 (same fp64 expression order)."""
    std = np.sqrt(np.float64(max(variance, 0.0)))   # var<0 clamped: see DESIGN.md
    return np.array([mean + (i - 3) * 0.3 * std for i in range(7)])


def min_var_moments(V, sums="sequential"):
    """R:dbscan/partition.py:86-89: fp64 sums of [1, v, v**2] with v**2 taken
    in the input precision (numpy squares fp32 vectors in fp32).

    sums='sequential': the reference's left-to-right fold (single Spark slice)
    — bit-exact with the shim-run reference.
    sums='exact': correctly rounded sums (math.fsum), the order-independent
    value the GPU's double-double reduction produces."""
    import math
    if len(V) == 0:
        return np.zeros((3, V.shape[1]))
    sq = (V * V).astype(np.float64)
    V64 = V.astype(np.float64)
    m0 = float(len(V))
    if sums == "exact":
        m1 = np.array([math.fsum(V64[:, j]) for j in range(V.shape[1])])
        m2 = np.array([math.fsum(sq[:, j]) for j in range(V.shape[1])])
    else:
        m1 = np.cumsum(V64, axis=0)[-1]
        m2 = np.cumsum(sq, axis=0)[-1]
    return np.stack([np.full(V.shape[1], m0), m1, m2])


def kd_partition(X, max_partitions=None, split_method="min_var", sums="sequential"):
    """KDPartitioner (R:dbscan/partition.py:111-183).

    Returns dict(owner=int64[n] KD label per point, box_lo/box_hi (P,k) fp64,
    splits=[(cur, new, axis, cand, n_left, n_right, mean, var, boundary)])."""
    X = np.asarray(X)
    if X.ndim == 1:
        X = X[:, None]
    n, k = X.shape
    P = int(max_partitions) if max_partitions is not None else 4 ** k
    lo, hi = root_box(X)
    boxes = {0: (lo.copy(), hi.copy())}
    owner = np.zeros(n, np.int64)
    splits = []
    axis_rot = 0
    for level in split_schedule(P):
        for cur, new in level:
            idx = np.nonzero(owner == cur)[0]        # key order, as the RDD keeps it
            V = X[idx]
            if split_method == "min_var":
                mom = min_var_moments(V, sums)
                with np.errstate(invalid="ignore", divide="ignore"):
                    means = mom[1] / mom[0]
                    var = mom[2] / mom[0] - means ** 2
                axis = int(np.argmax(var))
                bounds = mean_var_bounds(means[axis], var[axis])
                col = V[:, axis].astype(np.float64)
                cnt = np.array([np.sum(2 * (col < b).astype(np.float64) - 1) for b in bounds])
                cand = int(np.argmin(np.abs(cnt)))
                boundary = bounds[cand]
                mean_a, var_a = float(means[axis]), float(var[axis])
            else:   # 'rotation' → median_search_split (R:dbscan/partition.py:8-30)
                axis = axis_rot
                col = np.sort(V[:, axis].astype(np.float64))
                boundary = col[len(col) // 2] if len(col) else np.nan
                cand, mean_a, var_a = -1, np.nan, np.nan
            right = X[idx, axis].astype(np.float64) >= boundary
            owner[idx[right]] = new
            blo, bhi = boxes[cur]
            l_hi = bhi.copy()
            l_hi[axis] = boundary
            r_lo = blo.copy()
            r_lo[axis] = boundary
            boxes[cur] = (blo.copy(), l_hi)
            boxes[new] = (r_lo, bhi.copy())
            splits.append((cur, new, axis, cand, int((~right).sum()), int(right.sum()),
                           mean_a, var_a, float(boundary)))
        axis_rot = (axis_rot + 1) % k
    P_eff = len(boxes)
    box_lo = np.array([boxes[i][0] for i in range(P_eff)]).reshape(P_eff, k)
    box_hi = np.array([boxes[i][1] for i in range(P_eff)]).reshape(P_eff, k)
    return dict(owner=owner, box_lo=box_lo, box_hi=box_hi, splits=splits)


def halo(X, box_lo, box_hi, eps):
    """R:dbscan/dbscan.py:136-151 with BoundingBox.expand/contains
    (R:dbscan/geometry.py:73-96): membership[L] = indices inside box L grown
    by 2·eps, inclusive on every axis."""
    X = np.asarray(X)
    if X.ndim == 1:
        X = X[:, None]
    X64 = X.astype(np.float64)
    elo = box_lo - 2 * eps
    ehi = box_hi + 2 * eps
    members = []
    for L in range(len(box_lo)):
        m = np.all(elo[L] <= X64, axis=1) & np.all(ehi[L] >= X64, axis=1)
        members.append(np.nonzero(m)[0])
    return elo, ehi, members


class _UF:
    def __init__(self, n):
        self.p = list(range(n))

    def find(self, x):
        p = self.p
        while p[x] != x:
            p[x] = p[p[x]]
            x = p[x]
        return x

    def union(self, a, b):
        ra, rb = self.find(a), self.find(b)
        if ra != rb:
            if ra < rb:
                ra, rb = rb, ra
            self.p[ra] = rb


def pipeline(X, eps, min_samples, max_partitions=None, metric="euclidean"):
    """KD → halo → per-neighbourhood DBSCAN → owner-rule merge.

    The merge implements what R:dbscan/aggregator.py:9-73 intends (SURVEY.md
    §8(a) A12 lists why its literal behaviour is not reproduced): local
    clusters are linked through points that are core in two neighbourhoods;
    every point takes its value from its owner KD partition; cluster ids are
    numbered by their smallest core index and a border point joins the
    adjacent cluster with the smallest id — which is exactly sklearn's
    depth-first labelling (SK:cluster/_dbscan_inner.pyx:19-41) of the whole
    data set.  Returns dict(labels, core, kd, members, local)."""
    X = np.asarray(X)
    if X.ndim == 1:
        X = X[:, None]
    n = len(X)
    kd = kd_partition(X, max_partitions)
    elo, ehi, members = halo(X, kd["box_lo"], kd["box_hi"], eps)
    P = len(members)
    local = []
    node_base = [0]
    for L in range(P):
        lab, core, _, ncl = dbscan(X[members[L]], eps, min_samples, metric)
        local.append((lab, core))
        node_base.append(node_base[-1] + ncl)
    uf = _UF(node_base[-1])
    first_node = np.full(n, -1, np.int64)
    core_any = np.zeros(n, bool)
    for L in range(P):
        lab, core = local[L]
        for i, c, is_core in zip(members[L], lab, core):
            if is_core:
                node = node_base[L] + int(c)
                core_any[i] = True
                if first_node[i] < 0:
                    first_node[i] = node
                else:
                    uf.union(first_node[i], node)
    nroot = np.array([uf.find(v) for v in range(node_base[-1])], np.int64)
    gmin = np.full(node_base[-1], np.iinfo(np.int64).max, np.int64)
    for L in range(P):
        lab, core = local[L]
        m = core.astype(bool)
        np.minimum.at(gmin, nroot[node_base[L] + lab[m]], members[L][m])
    key = np.full(n, -1, np.int64)
    is_core = np.zeros(n, np.uint8)
    owner = kd["owner"]
    for L in range(P):
        lab, core = local[L]
        mem = members[L]
        own = owner[mem] == L
        if not np.any(own):
            continue
        pos = np.nonzero(own)[0]
        cm = core[pos].astype(bool)
        key[mem[pos[cm]]] = gmin[nroot[node_base[L] + lab[pos[cm]]]]
        is_core[mem[pos[cm]]] = 1
        border = pos[~cm]
        if len(border):
            off, nbr = neighbors(X[mem], eps, metric)
            for b in border:
                js = nbr[off[b]:off[b + 1]]
                js = js[core[js].astype(bool)]
                if len(js):
                    key[mem[b]] = gmin[nroot[node_base[L] + lab[js]]].min()
    uniq = np.unique(key[key >= 0])
    labels = np.full(n, -1, np.int64)
    labels[key >= 0] = np.searchsorted(uniq, key[key >= 0])
    return dict(labels=labels, core=is_core, kd=kd, members=members, local=local,
                box_elo=elo, box_ehi=ehi)
