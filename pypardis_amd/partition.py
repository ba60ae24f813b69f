"""KD partitioner — R:dbscan/partition.py:8-183, with the per-point passes
on the GPU.

Host side keeps exactly the reference's scalar arithmetic (mean, variance,
the seven candidate bounds ``mean + (i - 3) * 0.3 * std``, first argmin,
left-keeps-label / right-gets-next_label, BFS label order).  The passes over
the points run as HIP kernels through the C ABI:

    moments  Σ[1, v, v²] per label    pd_kd_moments   (R:dbscan/partition.py:86-89)
    counts   Σ 2·[v < b_i] − 1        pd_kd_counts    (R:dbscan/partition.py:60-63)
    split    v >= boundary → relabel  pd_kd_split     (R:dbscan/partition.py:66-68)
    bbox     union of all points      pd_bbox         (R:dbscan/partition.py:135-137)
    median   sorted v[axis][len/2]    pd_kd_radix_hist (R:dbscan/partition.py:23-26;
             split_method='rotation': MSD radix select, one histogram pass
             per 8-bit digit of the order key, all splits of a level at once)

All splits of one BFS level run in the same passes (each split only reads its
own label's points, so batching cannot change a result).  The sums are
correctly rounded (double-double, order independent — the same on one device
or summed over many, pypardis_amd/distributed.py); ``sums='sequential'``
reproduces the reference's left-to-right fold bit for bit instead.

Deliberate deviation: a variance that round-off makes negative is clamped to
0 before the sqrt; the reference takes sqrt(<0) = NaN there and silently
drops every point of that partition.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _native
from ._data import PointSet, as_points
from .geometry import BoundingBox


def _split_schedule(max_partitions):
    """The todo/done queue walk of R:dbscan/partition.py:159-183 as BFS levels
    of (current_label, next_label) pairs."""
    levels, todo, done, nxt, cur_level = [], [0], [], 1, []
    while nxt < max_partitions:
        if todo:
            cur = todo.pop(0)
            cur_level.append((cur, nxt))
            done += [cur, nxt]
            nxt += 1
        else:
            levels.append(cur_level)
            cur_level, todo, done = [], done, []
    if cur_level:
        levels.append(cur_level)
    return levels


# KDPartitioner's exact min_var path: the level decisions on the device
# (pd_kd_build, one host sync per partition) instead of one host round trip
# per pass; False forces the per-pass path (same splits; tests compare them).
DEVICE_DECISIONS = True


def _bounds(mean, variance):
    """R:dbscan/partition.py:58-59, same expression order in fp64."""
    std_dev = np.sqrt(np.float64(variance) if variance >= 0 else np.float64(0.0)) \
        if not np.isnan(variance) else np.float64(np.nan)
    return np.array([mean + (i - 3) * 0.3 * std_dev for i in range(7)])


class PartitionView(object):
    """The points currently carrying one KD label — what the reference keeps
    as the RDD ``((key, label), vector)`` of that partition."""

    def __init__(self, points, labels, label):
        self.points = points
        self._labels = labels   # tensor, or the partitioner (labels on first use)
        self.label = int(label)

    @property
    def labels(self):
        return self._labels.labels if isinstance(self._labels, KDPartitioner) else self._labels

    def indices(self):
        return torch.nonzero(self.labels == self.label).flatten()

    def count(self):
        return int((self.labels == self.label).sum().item())

    def keys(self):
        return self.points.key_array()[self.indices().cpu().numpy()]

    def collect(self):
        idx = self.indices()
        keys = self.points.key_array()[idx.cpu().numpy()]
        vecs = self.points.vectors(idx)
        return [((k, self.label), v) for k, v in zip(keys.tolist(), vecs)]

    def __len__(self):
        return self.count()

    def __repr__(self):
        return f"PartitionView(label={self.label})"


class _Union(object):
    """``KDPartitioner.result``: the union of every partition."""

    def __init__(self, parts):
        self.parts = parts

    def collect(self):
        out = []
        for L in sorted(self.parts):
            out += self.parts[L].collect()
        return out

    def count(self):
        return sum(p.count() for p in self.parts.values())


def _labels_of(partition):
    if not isinstance(partition, PartitionView):
        raise TypeError("expected a PartitionView (from KDPartitioner.partitions)")
    return partition.points.X, partition.labels


def mean_var_split(partition, k, axis, next_label, mean, variance):
    """R:dbscan/partition.py:33-69.  Returns (part1, part2, boundary); part1
    keeps the label (v < boundary), part2 becomes ``next_label``.  The split
    is applied to the partition's shared label array in place."""
    X, labels = _labels_of(partition)
    bounds = _bounds(mean, variance)
    cnt = _native.kd_counts(X, labels, [partition.label], [axis], bounds[None])[0]
    counts = np.abs(2.0 * cnt[:7].astype(np.float64) - float(cnt[7]))
    boundary = bounds[int(np.argmin(counts))]
    _native.kd_split(X, labels, [partition.label], [axis], [boundary], [next_label])
    return (partition, PartitionView(partition.points, labels, next_label), boundary)


def min_var_split(partition, k, next_label, sums='exact'):
    """R:dbscan/partition.py:72-95: split on the axis of largest variance."""
    X, labels = _labels_of(partition)
    mom = _native.kd_moments(X, labels, [partition.label], sequential=(sums == 'sequential'))[0]
    with np.errstate(invalid="ignore", divide="ignore"):
        means = mom[1] / mom[0]
        variances = mom[2] / mom[0] - means ** 2
    axis = int(np.argmax(variances))
    return mean_var_split(partition, k, axis, next_label, means[axis], variances[axis]), axis


def _from_key(key):
    """Inverse of the device's order key (kd.hip order_key) -> fp64 value."""
    key = int(key)
    bits = key & 0x7FFFFFFFFFFFFFFF if key >> 63 else (~key) & 0xFFFFFFFFFFFFFFFF
    return np.array([bits], np.uint64).view(np.float64)[0]


def level_medians(hist_fn, S, fp32):
    """Radix select of sorted_values[len // 2] for the S splits of a level
    (R:dbscan/partition.py:23-26).  hist_fn(prefix, shift) -> (S, 256) digit
    histograms (pd_kd_radix_hist, or its all-reduced sum over devices).
    Returns (median fp64 values, #points strictly below each median, #points).
    fp32 inputs widen to doubles whose low 29 mantissa bits are zero, so their
    select stops after the digit at bit 24.  An empty partition raises
    IndexError, as the reference's list index does."""
    less = np.zeros(S, np.int64)
    prefix = np.zeros(S, np.uint64)
    last = 24 if fp32 else 0
    totals = target = None
    for shift in range(56, last - 1, -8):
        h = np.asarray(hist_fn(prefix, shift), np.int64).reshape(S, 256)
        if totals is None:   # the top digit has no prefix condition: all points
            totals = h.sum(axis=1)
            if np.any(totals == 0):
                raise IndexError("list index out of range (median of an empty partition, "
                                 "R:dbscan/partition.py:25-26)")
            target = totals // 2
        cum = np.cumsum(h, axis=1)
        b = np.argmax(cum > target[:, None], axis=1)
        below = np.where(b > 0, cum[np.arange(S), b - 1], 0)
        less += below
        target -= below
        prefix = (prefix << np.uint64(8)) | b.astype(np.uint64)
    # the undecided low bits are zero in the value: zeros in the key of a
    # positive value, ones in the (complemented) key of a negative one
    low = (1 << last) - 1
    keys = [(int(p) << last) | (low if not (int(p) << last) >> 63 else 0) for p in prefix]
    return np.array([_from_key(k) for k in keys]), less, totals


def median_search_split(partition, axis, next_part):
    """R:dbscan/partition.py:8-30 (split_method='rotation'): split at the
    value of index len/2 of the sorted v[axis] (radix select on the GPU,
    pd_kd_radix_hist); part1 = v < median keeps the label, part2 = v >= median
    becomes ``next_part``.  Returns (part1, part2, median)."""
    X, labels = _labels_of(partition)
    med, _, _ = level_medians(
        lambda prefix, shift: _native.kd_radix_hist(X, labels, [partition.label], [axis],
                                                    prefix, shift),
        1, X.dtype == torch.float32)
    _native.kd_split(X, labels, [partition.label], [axis], [med[0]], [next_part])
    return (partition, PartitionView(partition.points, labels, next_part), float(med[0]))


def level_axes(mom):
    """Per split of one BFS level, from its moments (S, 3, d) = {count, Σv,
    Σv²}: the largest-variance axis (first argmax), its mean and variance and
    the seven candidate bounds (R:dbscan/partition.py:86-95, 58-59)."""
    axes, means, vars_, bounds = [], [], [], []
    for s in range(mom.shape[0]):
        with np.errstate(invalid="ignore", divide="ignore"):
            m = mom[s, 1] / mom[s, 0]
            v = mom[s, 2] / mom[s, 0] - m ** 2
        a = int(np.argmax(v))
        axes.append(a)
        means.append(m[a])
        vars_.append(v[a])
        bounds.append(_bounds(m[a], v[a]))
    return axes, means, vars_, np.array(bounds).reshape(len(axes), 7)


def level_boundaries(cnt, bounds):
    """First bound minimising |#left − #right| (R:dbscan/partition.py:60-65);
    cnt (S, 8) = #points below each bound, #points."""
    boundary, cand = [], []
    for s in range(cnt.shape[0]):
        c = np.abs(2.0 * cnt[s, :7].astype(np.float64) - float(cnt[s, 7]))
        i = int(np.argmin(c))
        cand.append(i)
        boundary.append(bounds[s, i])
    return boundary, cand


def apply_level(boxes, splits, level, axes, means, vars_, cnt, cand, boundary):
    """Split the boxes of one level (R:dbscan/partition.py:151-152,
    R:dbscan/geometry.py:51-71) and record the split trace."""
    for s, (cur, nl) in enumerate(level):
        left, right = boxes[cur].split(axes[s], boundary[s])
        boxes[cur] = left
        boxes[nl] = right
        n_tot = int(cnt[s, 7])
        # left child = points with v < boundary: counts of the chosen bound
        n_left = int(cnt[s, cand[s]])
        splits.append((cur, nl, axes[s], cand[s], n_left, n_tot - n_left,
                       float(means[s]), float(vars_[s]), float(boundary[s])))


def apply_rotation_level(boxes, splits, level, axes, medians, less, totals):
    """Box splits of one 'rotation' level (R:dbscan/partition.py:168-176);
    trace entries as apply_level's with cand = -1 and mean = var = NaN."""
    for s, (cur, nl) in enumerate(level):
        left, right = boxes[cur].split(axes[s], medians[s])
        boxes[cur] = left
        boxes[nl] = right
        splits.append((cur, nl, axes[s], -1, int(less[s]), int(totals[s] - less[s]),
                       float('nan'), float('nan'), float(medians[s])))


class KDPartitioner(object):
    """R:dbscan/partition.py:98-183.

    :partitions: label -> PartitionView
    :bounding_boxes: label -> BoundingBox
    :result: union of the partitions
    :labels: device int32 tensor, the KD label of every point
    :splits: per split (cur, new, axis, cand, n_left, n_right, mean, var, boundary)

    ``sums`` (extension): 'exact' (default) takes each label's moments as
    correctly rounded, order-independent sums; 'sequential' folds them in
    point order exactly as the reference's single-slice aggregate does, so
    boundaries are bit-identical to it (one GPU lane per moment: slow, a
    compatibility mode).  The two differ only where the reference's choice is
    decided by round-off (e.g. StandardScaler data: all variances are 1).
    """

    def __init__(self, data, max_partitions=None, k=None, split_method='min_var', sums='exact'):
        self.split_method = split_method if split_method in ['min_var', 'rotation'] else 'min_var'
        if sums not in ('exact', 'sequential'):
            raise ValueError("sums must be 'exact' or 'sequential'")
        self.sums = sums
        self.points = as_points(data)
        X = self.points.X
        self.k = int(k) if k is not None else self.points.d
        self.max_partitions = int(max_partitions) if max_partitions is not None else 4 ** self.k
        if self.max_partitions < 1:
            raise ValueError("max_partitions must be >= 1")
        if self.max_partitions > 1 << 16:
            # the reference's default 4**k (R:dbscan/partition.py:132-133) is
            # astronomically large in high dimension; it would never finish
            raise ValueError(f"max_partitions={self.max_partitions} (> 65536; the default is "
                             "4**k): pass max_partitions explicitly")
        self._pending = None    # the last level's split, applied on first use
        self._tree = None       # (sizes, cur, axis, boundary, new): pd_train_tree
        levels = _split_schedule(self.max_partitions)
        device_kd = bool(levels) and self._fused() and DEVICE_DECISIONS
        # pd_kd_build writes every label from its second level on (no fill)
        self._labels = (torch.empty if device_kd and len(levels) >= 2 else torch.zeros)(
            self.points.n, dtype=torch.int32, device=X.device)
        first = None
        trace = None
        if device_kd:
            # the whole BFS in one launch chain (pd_kd_build): the level
            # decisions run on the device, bit-identical to the host's
            try:
                # final mode 2: the labels are not written (the passes replay
                # the splits; the labels property replays the finished tree)
                lo, hi, bad, trace = _native.kd_build(X, self._labels, levels,
                                                      final_split=2)
            except _native.PardisError as e:
                if e.code != _native.PD_EUNSUPPORTED:
                    raise
                self._labels.zero_()   # the host-level passes start from label 0
        if trace is not None:
            if bad:
                raise ValueError("Input contains NaN or infinity.")
            self.data_box = (lo, hi)
            self.splits = []
            self._apply_trace(BoundingBox(k=self.k).union(BoundingBox(lo, hi)), levels, trace)
            last = trace[len(trace) - len(levels[-1]):]
            self._pending = ([c for c, _ in levels[-1]], last[:, 0].astype(np.int32).tolist(),
                             last[:, 12].tolist(), [nl for _, nl in levels[-1]])
            self._tree = (np.array([len(lv) for lv in levels], np.int32),
                          np.array([c for lv in levels for c, _ in lv], np.int32),
                          trace[:, 0].astype(np.int32), trace[:, 12].copy(),
                          np.array([nl for lv in levels for _, nl in lv], np.int32))
            self.partitions = {L: PartitionView(self.points, self, L)
                               for L in sorted(self.bounding_boxes)}
            self.result = _Union(self.partitions)
            return
        if levels and self._fused():
            # the bbox rides on the first level's moments pass (one read of X)
            first, lo, hi, bad = _native.kd_pass(X, self._labels, sel=[0], labels_zero=True,
                                                 bbox=True)
        else:
            lo, hi, bad = _native.bbox(X)
        if bad:
            raise ValueError("Input contains NaN or infinity.")
        self.data_box = (lo, hi)     # tight box: the engine clips its grids to it
        box = BoundingBox(k=self.k).union(BoundingBox(lo, hi))
        self.splits = []
        self._create_partitions(box, levels, first)
        self.partitions = {L: PartitionView(self.points, self._labels, L)
                           for L in sorted(self.bounding_boxes)}
        self.result = _Union(self.partitions)

    @property
    def labels(self):
        """KD label of every point (device int32, input order), computed on
        first use by replaying the split tree (pd_kd_labels)."""
        if self._pending is not None:
            self._pending = None
            _native.kd_labels(self.points.X, self._labels, self._tree)
        return self._labels

    def split_tree(self):
        """The BFS split tree for pd_train_tree (device-decided path), else None."""
        return self._tree

    def _apply_trace(self, box, levels, trace):
        """Boxes and split trace from pd_kd_build's per-split records."""
        self.bounding_boxes = {0: box}
        k = 0
        for level in levels:
            t = trace[k:k + len(level)]
            k += len(level)
            apply_level(self.bounding_boxes, self.splits, level, t[:, 0].astype(np.int64).tolist(),
                        t[:, 1], t[:, 2], t[:, 3:11].astype(np.int64),
                        t[:, 11].astype(np.int64).tolist(), t[:, 12])

    def _fused(self):
        return self.split_method == 'min_var' and self.sums == 'exact'

    def _create_partitions(self, box, levels, first=None):
        X, labels = self.points.X, self._labels
        self.bounding_boxes = {0: box}
        if self._fused():
            # per level two streaming passes: pd_kd_pass (the previous
            # level's split + this level's moments) and pd_kd_counts; the
            # last level's split runs alone
            pending = None
            for depth, level in enumerate(levels):
                sel = [c for c, _ in level]
                new = [nl for _, nl in level]
                dd = first if depth == 0 and first is not None else \
                    _native.kd_pass(X, labels, split=pending, sel=sel)
                axes, means, vars_, bounds = level_axes(_native.round_dd(dd))
                cnt = _native.kd_counts(X, labels, sel, axes, bounds)
                boundary, cand = level_boundaries(cnt, bounds)
                pending = (sel, axes, boundary, new)
                apply_level(self.bounding_boxes, self.splits, level, axes, means, vars_, cnt,
                            cand, boundary)
            if pending is not None:
                _native.kd_split(X, labels, *pending)
            return
        for depth, level in enumerate(levels):
            sel = [c for c, _ in level]
            new = [nl for _, nl in level]
            if self.split_method == 'rotation':
                # the axis cycles once per BFS level (R:dbscan/partition.py:152,180-183)
                axes = [depth % self.k] * len(sel)
                med, less, tot = level_medians(
                    lambda prefix, shift: _native.kd_radix_hist(X, labels, sel, axes, prefix,
                                                                shift),
                    len(sel), X.dtype == torch.float32)
                _native.kd_split(X, labels, sel, axes, med, new)
                apply_rotation_level(self.bounding_boxes, self.splits, level, axes, med, less, tot)
                continue
            mom = _native.kd_moments(X, labels, sel, sequential=(self.sums == 'sequential'))
            axes, means, vars_, bounds = level_axes(mom)
            cnt = _native.kd_counts(X, labels, sel, axes, bounds)
            boundary, cand = level_boundaries(cnt, bounds)
            _native.kd_split(X, labels, sel, axes, boundary, new)
            apply_level(self.bounding_boxes, self.splits, level, axes, means, vars_, cnt, cand,
                        boundary)

    def box_array(self):
        """(P, 2, k) fp64 boxes in label order."""
        return np.stack([self.bounding_boxes[L].as_array() for L in sorted(self.bounding_boxes)])
