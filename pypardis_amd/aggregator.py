"""String-label compatibility layer for callers
that consume ``dbscan_partition``'s ``"p:c[*]"`` records directly.

``ClusterAggregator`` keeps the reference's interface (R:dbscan/aggregator.py:
9-73): ``fwd`` (partition-level label → global id), ``rev`` (global id → set
of labels), ``next_global_id``, ``agg + (key, labels)``, ``agg + other``,
``agg[label] = gid``.  It implements what that code intends, not its bugs
(SURVEY.md §8(a) A12): a point links every CORE label it carries (no ``*``,
no ``-1``), whatever the set iteration order, and combining two aggregators
unions their groups instead of re-testing an arbitrary first element.  The
production path does not use this: ``pd_train`` merges on the device.
"""
from __future__ import annotations

import sys
from collections import defaultdict


def default_value():
    """R:dbscan/aggregator.py:5-6 (``sys.maxint`` on Python 2)."""
    return sys.maxsize


class ClusterAggregator(object):
    def __init__(self):
        self.fwd = defaultdict(default_value)
        self.rev = defaultdict(set)
        self.next_global_id = 0

    def _link(self, labels):
        core = [l for l in labels if '*' not in l and '-1' not in l]
        if not core:
            return
        known = {self.fwd[l] for l in core if l in self.fwd}
        gid = min(known) if known else self.next_global_id
        if not known:
            self.next_global_id += 1
        for other in known:
            if other != gid:
                for l in self.rev.pop(other, ()):
                    self[l] = gid
        for l in core:
            self[l] = gid

    def __add__(self, other):
        if isinstance(other, ClusterAggregator):
            for labels in list(other.rev.values()):
                self._link(list(labels))
        else:
            _index, pl_ids = other
            self._link(list(set(pl_ids)))
        return self

    def __setitem__(self, a, b):
        old = self.fwd.get(a)
        if old is not None and old != b and a in self.rev.get(old, ()):
            self.rev[old].discard(a)
            if not self.rev[old]:
                del self.rev[old]
        self.fwd[a] = b
        self.rev[b].add(a)
