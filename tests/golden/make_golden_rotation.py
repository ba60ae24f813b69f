#!/usr/bin/env python3
"""Golden vectors for KDPartitioner(split_method='rotation') (test infrastructure).

Runs ONLY in the build container (reference mounted read-only at
/root/reference), with the same in-memory RDD stand-in as make_golden.py.
The reference's median_search_split indexes ``sorted_values[len / 2]``
(R:dbscan/partition.py:25-26), which is an integer index under Python 2; the
stand-in's ``collect()`` therefore returns a list that accepts integral float
indices, as the Python-2 runtime the code was written for would.  Nothing else
is changed; only numeric inputs/outputs are saved (rot_*.npz).

Usage:  PYTHONHASHSEED=0 python tests/golden/make_golden_rotation.py
"""
from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402


class _Py2List(list):
    """list indexed by ``len / 2`` as Python 2 evaluates it (floor division):
    Python 3 hands over the true quotient, e.g. 187.5 for 375 values."""

    def __getitem__(self, i):
        if isinstance(i, float) and i >= 0:
            i = int(i)   # == len // 2 for i == len / 2
        return super().__getitem__(i)


class _RDD(mg.FakeRDD):
    def _new(self, parts):
        return _RDD(self.context, parts)

    def collect(self):
        return _Py2List(super().collect())


class _Ctx(mg.FakeContext):
    def parallelize(self, data, n=None):
        r = super().parallelize(data, n)
        return _RDD(self, r.parts)


def run(X, P):
    ref, refpart, refdb, KDP = mg.load_reference()
    trace = []
    orig = refpart.median_search_split

    def traced(partition, axis, next_part):
        p1, p2, median = orig(partition, axis, next_part)
        cur = partition.first()[0][1]
        trace.append((cur, next_part, axis, len(p1.collect()), len(p2.collect()), median))
        return p1, p2, median

    refpart.median_search_split = traced
    try:
        ctx = _Ctx(1)
        kdp = KDP(ctx.parallelize([(i, X[i]) for i in range(len(X))]), P,
                  split_method="rotation")
    finally:
        refpart.median_search_split = orig
    d = X.shape[1]
    Pn = len(kdp.bounding_boxes)
    lo = np.array([kdp.bounding_boxes[i].lower for i in range(Pn)], np.float64).reshape(Pn, d)
    hi = np.array([kdp.bounding_boxes[i].upper for i in range(Pn)], np.float64).reshape(Pn, d)
    owner = np.full(len(X), -1, np.int64)
    for lab, prdd in kdp.partitions.items():
        for (key, _l), _v in prdd.collect():
            owner[key] = lab
    splits = np.array([t[:5] for t in trace], np.int64).reshape(-1, 5)
    medians = np.array([t[5] for t in trace], np.float64)
    return dict(X=X, max_partitions=np.int64(P), box_lo=lo, box_hi=hi, owner=owner,
                splits=splits, medians=medians)


def datasets():
    from pypardis_amd import synth
    out = {}
    X0, _ = synth.make_config("C0")
    out["c0_p16"] = (X0, 16)
    out["c0_p5"] = (X0, 5)
    X3 = synth.blobs_noise(20000, 3, side=12.0, n_centers=10, sigma=0.7,
                           noise_frac=0.15, seed=12)
    out["b3d_p8"] = (X3, 8)
    # duplicated values: the median index lands inside runs of equal values
    rng = np.random.default_rng(21)
    Xd = np.round(rng.normal(size=(3001, 2)), 1).astype(np.float32)
    out["dup2d_p6"] = (Xd, 6)
    return out


def main():
    for name, (X, P) in datasets().items():
        rec = run(X, P)
        np.savez_compressed(os.path.join(HERE, f"rot_{name}.npz"), **rec)
        print(f"rot_{name}: n={len(X)} d={X.shape[1]} P={P} splits={len(rec['splits'])}")


if __name__ == "__main__":
    main()
