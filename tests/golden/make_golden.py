#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ (test infrastructure).

Runs ONLY in the build container, where the reference is mounted read-only at
/root/reference.  It never writes there (PYTHONDONTWRITEBYTECODE is forced) and
nothing from the reference is copied into the repo: only the numeric
inputs/outputs below are saved, as small .npz files.

Two sources of truth:

1. The reference pipeline itself (R:dbscan/*.py), imported unmodified and run
   over an in-memory stand-in for the handful of pyspark RDD methods it calls
   (pyspark/Java are absent).  The stand-in is written here
   from the RDD semantics, not taken from anywhere.  From it we record, per
   dataset: every KD split (R:dbscan/partition.py:33-95), the bounding and
   expanded boxes (R:dbscan/dbscan.py:136-151), the halo membership of every
   neighbourhood, and every neighbourhood's ``dbscan_partition`` output
   (R:dbscan/dbscan.py:12-34) — core flags and local labels.  The final
   ``assignments()`` are stored as an artefact only (they are hash-seed
   dependent).

2. scikit-learn 1.7.2 (the reference's arithmetic dependency, not vendored):
   global ``DBSCAN(algorithm='kd_tree')`` labels / core flags / neighbour counts
   on the fp64 upcast of each dataset, and the known-answer cases of
   SK:cluster/tests/test_dbscan.py:297-305, 376-403.

Usage:  PYTHONHASHSEED=0 python tests/golden/make_golden.py [dataset ...]
"""
from __future__ import annotations

import builtins
import collections
import copy
import os
import sys
import types

sys.dont_write_bytecode = True
os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)


# --------------------------------------------------------------------------
# In-memory RDD stand-in: just the surface R:dbscan/*.py touches.
# --------------------------------------------------------------------------
class _Py2Dict(dict):
    def iteritems(self):
        return iter(list(self.items()))

    def itervalues(self):
        return iter(list(self.values()))


class _Py2DefaultDict(collections.defaultdict):
    def iteritems(self):
        return iter(list(self.items()))


def _apply(f, rec):
    # Python-2 tuple-parameter lambdas (lambda (k, v): ...) were rewritten as
    # two-argument lambdas in the reference; Spark would pass one record.
    if f.__code__.co_argcount == 2 and isinstance(rec, tuple) and len(rec) == 2:
        return f(*rec)
    return f(rec)


class _Broadcast:
    def __init__(self, value):
        self.value = value


class FakeContext:
    def __init__(self, slices=1):
        self.slices = slices

    def emptyRDD(self):
        return FakeRDD(self, [])

    def broadcast(self, v):
        return _Broadcast(copy.deepcopy(v))

    def parallelize(self, data, n=None):
        data = list(data)
        n = n or self.slices
        L = len(data)
        return FakeRDD(self, [data[i * L // n:(i + 1) * L // n] for i in range(n)])


class FakeRDD:
    def __init__(self, ctx, parts):
        self.context = ctx
        self.parts = parts

    def _new(self, parts):
        return FakeRDD(self.context, parts)

    def cache(self):
        return self

    def first(self):
        for p in self.parts:
            for x in p:
                return x
        raise ValueError("empty RDD")

    def collect(self):
        return [x for p in self.parts for x in p]

    def map(self, f):
        return self._new([[_apply(f, x) for x in p] for p in self.parts])

    def filter(self, f):
        return self._new([[x for x in p if _apply(f, x)] for p in self.parts])

    def union(self, other):
        return self._new(self.parts + other.parts)

    def sortBy(self, f):
        return self._new([sorted(self.collect(), key=lambda x: _apply(f, x))])

    def sortByKey(self):
        return self._new([sorted(self.collect(), key=lambda kv: kv[0])])

    def mapPartitions(self, f):
        return self._new([list(f(iter(p))) for p in self.parts])

    def partitionBy(self, n):
        out = [[] for _ in range(n)]
        for p in self.parts:
            for k, v in p:
                out[hash(k) % n].append((k, v))
        return self._new(out)

    def groupByKey(self):
        d = collections.OrderedDict()
        for p in self.parts:
            for k, v in p:
                d.setdefault(k, []).append(v)
        return self._new([list(d.items())])

    def aggregate(self, zero, seq, comb):
        partials = []
        for p in self.parts:
            acc = copy.deepcopy(zero)
            for x in p:
                acc = seq(acc, x)
            partials.append(acc)
        acc = zero
        for r in partials:
            if hasattr(r, "rev"):
                r.rev = _Py2DefaultDict(set, r.rev)
            acc = comb(acc, r)
        return acc


def load_reference():
    builtins.xrange = range
    sys.maxint = sys.maxsize
    mod = types.ModuleType("pyspark")
    mod.RDD = FakeRDD
    mod.SparkContext = FakeContext
    sys.modules["pyspark"] = mod
    sys.path.insert(0, REF)
    import dbscan as ref  # noqa: E402  (the reference package)
    from dbscan import partition as refpart
    from dbscan import dbscan as refdb
    sys.path.remove(REF)

    class KDP(ref.KDPartitioner):
        # only wraps the dicts the unmodified split loop builds, so the later
        # Python-2 iteritems()/itervalues() calls resolve
        def _create_partitions(self, data, box):
            super()._create_partitions(data, box)
            self.partitions = _Py2Dict(self.partitions)
            self.bounding_boxes = _Py2Dict(self.bounding_boxes)

    refdb.KDPartitioner = KDP
    return ref, refpart, refdb, KDP


# --------------------------------------------------------------------------
def run_reference(X, eps, min_samples, max_partitions, metric="euclidean"):
    ref, refpart, refdb, KDP = load_reference()
    trace = []
    orig_mvs = refpart.mean_var_split

    def traced(partition, k, axis, next_label, mean, variance):
        p1, p2, boundary = orig_mvs(partition, k, axis, next_label, mean, variance)
        std = np.sqrt(variance)
        bounds = np.array([mean + (i - 3) * 0.3 * std for i in range(7)])
        cand = int(np.where(bounds == boundary)[0][0]) if np.any(bounds == boundary) else 0
        n_part = len(partition.collect())
        cur = partition.first()[0][1] if n_part else -1
        trace.append(dict(cur=cur, new=next_label, axis=int(axis), mean=float(mean),
                          var=float(variance), boundary=float(boundary), cand=cand,
                          n_left=len(p1.collect()), n_right=len(p2.collect())))
        return p1, p2, boundary

    refpart.mean_var_split = traced
    try:
        ctx = FakeContext(1)
        rows = [(i, X[i]) for i in range(len(X))]
        rdd = ctx.parallelize(rows)
        metric_obj = metric
        if metric == "callable":
            from scipy.spatial.distance import euclidean
            metric_obj = euclidean
        m = ref.DBSCAN(eps=eps, min_samples=min_samples, metric=metric_obj,
                       max_partitions=max_partitions)
        m.train(rdd)
        assign = m.assignments()
    finally:
        refpart.mean_var_split = orig_mvs

    P = len(m.bounding_boxes)
    d = X.shape[1]
    lo = np.array([m.bounding_boxes[i].lower for i in range(P)], dtype=np.float64).reshape(P, d)
    hi = np.array([m.bounding_boxes[i].upper for i in range(P)], dtype=np.float64).reshape(P, d)
    elo = np.array([m.expanded_boxes[i].lower for i in range(P)], dtype=np.float64).reshape(P, d)
    ehi = np.array([m.expanded_boxes[i].upper for i in range(P)], dtype=np.float64).reshape(P, d)
    # halo membership: (label, key) pairs, sorted
    halo = []
    for lab in range(P):
        for (key, l2), _v in m.neighbors[lab].collect():
            halo.append((lab, key))
    halo = np.array(sorted(halo), dtype=np.int64).reshape(-1, 2)
    # per-neighbourhood dbscan_partition output: (label, key, local cid, core)
    part_out = []
    for key, s in m.data.collect():
        p, rest = s.split(":")
        core = 0 if rest.endswith("*") else 1
        part_out.append((int(p), int(key), int(rest.rstrip("*")), core))
    part_out = np.array(sorted(part_out), dtype=np.int64).reshape(-1, 4)
    # owner partition of each point (the KD value filters)
    owner = np.full(len(X), -1, dtype=np.int64)
    kdp = KDP(ctx.parallelize([(i, X[i]) for i in range(len(X))]), max_partitions)
    for lab, prdd in kdp.partitions.items():
        for (key, _l), _v in prdd.collect():
            owner[key] = lab
    ref_assign = np.array([(k, v) for k, v in assign], dtype=np.int64).reshape(-1, 2)
    splits = np.array([[t["cur"], t["new"], t["axis"], t["cand"], t["n_left"], t["n_right"]]
                       for t in trace], dtype=np.int64).reshape(-1, 6)
    split_f = np.array([[t["mean"], t["var"], t["boundary"]] for t in trace],
                       dtype=np.float64).reshape(-1, 3)
    return dict(P=np.int64(P), box_lo=lo, box_hi=hi, ebox_lo=elo, ebox_hi=ehi,
                halo=halo, part_out=part_out, owner=owner, ref_assign=ref_assign,
                splits=splits, split_f=split_f)


def run_sklearn(X, eps, min_samples, metric="euclidean"):
    from sklearn.cluster import DBSCAN
    from sklearn.neighbors import NearestNeighbors
    X64 = np.asarray(X, dtype=np.float64)
    db = DBSCAN(eps=eps, min_samples=min_samples, metric=metric,
                algorithm="kd_tree").fit(X64)
    core = np.zeros(len(X), np.uint8)
    core[db.core_sample_indices_] = 1
    nn = NearestNeighbors(radius=eps, algorithm="kd_tree", metric=metric).fit(X64)
    counts = np.array([len(a) for a in nn.radius_neighbors(X64, return_distance=False)],
                      dtype=np.int64)
    # the same fit on the raw (possibly fp32) array: checks that sklearn
    # upcasts before the predicate (KDTree is KDTree64)
    db_raw = DBSCAN(eps=eps, min_samples=min_samples, metric=metric,
                    algorithm="kd_tree").fit(X)
    assert np.array_equal(db_raw.labels_, db.labels_), "fp32 vs fp64 sklearn mismatch"
    return dict(sk_labels=db.labels_.astype(np.int64), sk_core=core, sk_counts=counts)


def datasets():
    from pypardis_amd import synth
    out = {}
    X0, _ = synth.make_config("C0")
    out["c0"] = (X0, 0.3, 10, None, "euclidean")
    out["c0_callable"] = (X0, 0.3, 10, None, "callable")
    out["c0_p3"] = (X0, 0.3, 10, 3, "euclidean")
    out["c0_p5_cityblock"] = (X0, 0.3, 10, 5, "cityblock")
    X2 = synth.blobs_noise(20000, 2, side=20.0, n_centers=12, sigma=0.6,
                           noise_frac=0.1, seed=11)
    out["b2d_20k"] = (X2, 0.12, 10, 8, "euclidean")
    X3 = synth.blobs_noise(20000, 3, side=12.0, n_centers=10, sigma=0.7,
                           noise_frac=0.15, seed=12)
    out["b3d_20k"] = (X3, 0.25, 10, 8, "euclidean")
    # all-negative coordinates (BoundingBox float_info.min quirk, A1)
    Xn = synth.blobs_noise(3000, 2, side=10.0, n_centers=4, sigma=0.5,
                           noise_frac=0.1, seed=13) - np.float32(50.0)
    out["neg_3k"] = (Xn, 0.2, 6, 4, "euclidean")
    # zero-variance data (A5): 40 identical points, 2 partitions
    Xz = np.full((40, 2), 0.7, dtype=np.float64)
    out["ident_40"] = (Xz, 0.1, 5, 2, "euclidean")
    # exact ties on an fp32 lattice (A4): spacing f32(0.05), eps = f32(0.05)
    g = np.arange(30, dtype=np.float32) * np.float32(0.05)
    Xl = np.stack(np.meshgrid(g, g, indexing="ij"), -1).reshape(-1, 2).astype(np.float32)
    out["lattice_900"] = (Xl, float(np.float32(0.05)), 5, 4, "euclidean")
    # duplicates + 1-D
    rng = np.random.default_rng(14)
    Xd = np.repeat(rng.uniform(0, 5, size=(200, 1)).astype(np.float32), 3, axis=0)
    rng.shuffle(Xd)
    out["dup_1d"] = (Xd, 0.05, 4, 4, "euclidean")
    # 64-D unit embeddings (config C3 at 5k points: 10 clusters of ~50)
    X6, c6 = synth.make_config("C3", n=5000)
    out["c3_5k"] = (X6, c6["eps"], c6["min_samples"], 2, "euclidean")
    return out


def sklearn_kats():
    """SK:cluster/tests/test_dbscan.py:376-403 and :297-305."""
    from sklearn.cluster import dbscan
    res = {}
    X = np.array([[0], [2], [3], [4], [6], [8], [10]], dtype=np.float64)
    exp = {1: ([0, 1, 2, 3, 4, 5, 6], [0, 1, 1, 1, 2, 3, 4]),
           2: ([1, 2, 3], [-1, 0, 0, 0, -1, -1, -1]),
           3: ([2], [-1, 0, 0, 0, -1, -1, -1]),
           4: ([], [-1] * 7)}
    for ms, (core, lab) in exp.items():
        c, l = dbscan(X, eps=1, min_samples=ms, algorithm="kd_tree")
        assert list(c) == core and list(l) == lab
        res[f"toy_ms{ms}_labels"] = np.array(lab, np.int64)
        res[f"toy_ms{ms}_core"] = np.array(core, np.int64)
    res["toy_X"] = X
    # boundaries: eps inclusive, min_samples counts the point itself
    res["bnd_a_X"] = np.array([[0], [1]], np.float64)
    res["bnd_a_core"] = dbscan(res["bnd_a_X"], eps=2, min_samples=2)[0].astype(np.int64)
    res["bnd_b_X"] = np.array([[0], [1], [1]], np.float64)
    res["bnd_b_core_eps1"] = dbscan(res["bnd_b_X"], eps=1, min_samples=2)[0].astype(np.int64)
    res["bnd_b_core_eps099"] = dbscan(res["bnd_b_X"], eps=0.99, min_samples=2)[0].astype(np.int64)
    # generate_clustered_data (SK:cluster/tests/common.py:12-37), eps 0.8, ms 10
    from sklearn.cluster.tests.common import generate_clustered_data
    Xc = generate_clustered_data(n_clusters=3)
    c, l = dbscan(Xc, eps=0.8, min_samples=10, metric="euclidean", algorithm="kd_tree")
    res["clustered_X"] = Xc
    res["clustered_labels"] = l.astype(np.int64)
    res["clustered_core"] = c.astype(np.int64)
    # no core samples (SK:.../test_dbscan.py:148-157)
    rng = np.random.RandomState(0)
    Xn = rng.rand(40, 10)
    Xn[Xn < 0.8] = 0
    c, l = dbscan(Xn, min_samples=6, algorithm="kd_tree")
    assert len(c) == 0 and np.all(l == -1)
    res["nocore_X"] = Xn
    return res


def main(only=()):
    if os.environ.get("PYTHONHASHSEED") != "0":
        print("warning: run with PYTHONHASHSEED=0 for a reproducible ref_assign artefact")
    if not only:
        np.savez_compressed(os.path.join(HERE, "sklearn_kat.npz"), **sklearn_kats())
    for name, (X, eps, ms, P, metric) in datasets().items():
        if only and name not in only:
            continue
        sk_metric = "euclidean" if metric == "callable" else metric
        rec = dict(X=X, eps=np.float64(eps), min_samples=np.int64(ms),
                   max_partitions=np.int64(-1 if P is None else P),
                   metric=np.array(metric))
        rec.update(run_sklearn(X, eps, ms, sk_metric))
        rec.update(run_reference(X, eps, ms, P, metric))
        np.savez_compressed(os.path.join(HERE, f"ref_{name}.npz"), **rec)
        n_core = int(rec["sk_core"].sum())
        n_cl = int(rec["sk_labels"].max() + 1)
        print(f"{name}: n={len(X)} d={X.shape[1]} P={int(rec['P'])} cores={n_core} "
              f"clusters={n_cl} halo_records={len(rec['halo'])} splits={len(rec['splits'])}")


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))
