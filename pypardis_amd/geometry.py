"""Axis-aligned boxes in fp64 on the host — same semantics as the
reference's ``BoundingBox`` (R:dbscan/geometry.py:5-100), including its
empty-box sentinels: ``BoundingBox(k=k)`` starts at lower = float_info.max and
upper = float_info.min (+2.2e-308, *not* -max; R:dbscan/geometry.py:28-29), so
a union over all-negative data keeps upper = 2.2e-308 on that axis.

Boxes are tiny (2·k doubles) and only ever touched a few times per train, so
they stay numpy; every per-point test against them runs on the GPU
(``pd_halo_members`` / ``pd_train``).
"""
from __future__ import annotations

import sys

import numpy as np


class BoundingBox(object):
    """:lower: / :upper: fp64 bounds, inclusive on every axis."""

    def __init__(self, lower=None, upper=None, k=None, all_space=False):
        if lower is not None:
            self.lower = np.array(lower)
            self.upper = np.array(upper) if upper is not None else self.lower
        elif k is not None:
            big, tiny = sys.float_info.max, sys.float_info.min
            self.lower = np.full(k, tiny if all_space else big)
            self.upper = np.full(k, big if all_space else tiny)
        else:
            self.lower = None
            self.upper = None

    @property
    def k(self):
        return None if self.lower is None else int(np.size(self.lower))

    def intersection(self, other):
        """R:dbscan/geometry.py:34-43"""
        return BoundingBox(lower=np.maximum(self.lower, other.lower),
                           upper=np.minimum(self.upper, other.upper))

    def union(self, other):
        """R:dbscan/geometry.py:45-54"""
        return BoundingBox(lower=np.minimum(self.lower, other.lower),
                           upper=np.maximum(self.upper, other.upper))

    @classmethod
    def _own(cls, lower, upper):
        # fresh arrays the new box owns (no second copy; the train's host path
        # builds a few dozen boxes per call)
        b = cls.__new__(cls)
        b.lower = lower
        b.upper = upper
        return b

    def split(self, dim, value):
        """R:dbscan/geometry.py:56-71: left keeps [lower, value], right [value, upper]."""
        left_up = self.upper.copy()
        left_up[dim] = value
        right_lo = self.lower.copy()
        right_lo[dim] = value
        return (BoundingBox._own(self.lower.copy(), left_up),
                BoundingBox._own(right_lo, self.upper.copy()))

    def expand(self, eps=0, how='add'):
        """R:dbscan/geometry.py:73-87 ('add' grows by eps, 'multiply' by eps·span)."""
        if how == 'add':
            return BoundingBox._own(self.lower - eps, self.upper + eps)
        if how == 'multiply':
            span = self.upper - self.lower
            return BoundingBox(self.lower - eps * span, self.upper + eps * span)
        return None

    def contains(self, vector):
        """R:dbscan/geometry.py:89-96: inclusive on every axis."""
        return bool(np.all(self.lower <= vector) and np.all(self.upper >= vector))

    def as_array(self):
        """(2, k) fp64 [lower; upper] — the layout the C ABI takes."""
        return np.array((self.lower, self.upper), np.float64)

    def __eq__(self, other):
        return (isinstance(other, BoundingBox) and np.array_equal(self.lower, other.lower)
                and np.array_equal(self.upper, other.upper))

    def __repr__(self):
        return 'BoundingBox(lower=%s\n\tupper=%s)' % (str(self.lower), str(self.upper))
