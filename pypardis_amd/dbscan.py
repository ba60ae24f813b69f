"""``DBSCAN`` driver — the surface of R:dbscan/dbscan.py:56-165 on MI355X.

What ``train`` does, stage by stage, against the reference:

    KDPartitioner(data, max_partitions)      R:dbscan/dbscan.py:110   GPU passes (partition.py)
    _create_neighborhoods: box.expand(2·eps)  R:dbscan/dbscan.py:136-151
    partitionBy + mapPartitions(dbscan_partition)
                                              R:dbscan/dbscan.py:116-124
    _remap_cluster_ids (+ ClusterAggregator)  R:dbscan/dbscan.py:153-165
        └── the last three fused into ONE device call, pd_train (engine.hip):
            halo records → (neighbourhood, eps-cell) sort → neighbour count /
            core flags → union-find on core–core edges → merge of the copies
            of each halo point → border attach → global labels.

The labels are the ones sklearn's ``DBSCAN(eps, min_samples).fit_predict``
gives on the whole data set (what the reference's merge intends; its literal
merge is hash-order dependent), and are independent of
``max_partitions``.
"""
from __future__ import annotations

import numpy as np
import torch
from scipy.spatial.distance import euclidean

from . import _native
from ._data import PointSet, as_points
from .partition import KDPartitioner


def dbscan_partition(iterable, params):
    """R:dbscan/dbscan.py:12-34: cluster one neighbourhood.

    :param iterable: ((key, partition), vector) records of one neighbourhood
    :param params: {'eps', 'min_samples', 'metric'}
    :return: yields (key, '%i:%i%s' % (partition, cluster_id, '' or '*'))
    Runs ``pd_cluster`` (sklearn fit_predict semantics) on the GPU.  An empty
    neighbourhood yields nothing (the reference raises IndexError, :24).
    """
    data = list(iterable)
    if not data:
        return
    (key, part), vector = data[0]
    X = np.array([v for (_, __), v in data])
    y = [k for (k, _), __ in data]
    pts = as_points(X)
    labels, core, _, _ = _native.cluster(pts.X, params['eps'], params['min_samples'],
                                         _native.metric_code(params.get('metric', 'euclidean')))
    c = labels.cpu().numpy()
    cores = core.cpu().numpy()
    for i in range(len(c)):
        flag = '' if cores[i] else '*'
        yield (y[i], '%i:%i%s' % (part, c[i], flag))


def map_cluster_id(x, broadcast_dict):
    """R:dbscan/dbscan.py:37-53 (string-label compatibility): first label of
    the group, '*' stripped; -1 if it is noise or unmapped."""
    key, cluster_id = x
    cluster_id = next(iter(cluster_id)).strip('*')
    cluster_dict = getattr(broadcast_dict, 'value', broadcast_dict)
    if '-1' not in cluster_id and cluster_id in cluster_dict:
        return key, cluster_dict[cluster_id]
    return key, -1


class _Neighborhood(object):
    """``neighbors[label]``: points inside the 2·eps-expanded box of one KD
    partition (membership computed on the GPU by pd_halo_members)."""

    def __init__(self, owner, label):
        self._owner = owner
        self.label = label

    def indices(self):
        return self._owner._members(self.label)

    def keys(self):
        return self._owner.points.key_array()[self.indices()]

    def collect(self):
        idx = self.indices()
        vecs = self._owner.points.vectors(torch.from_numpy(idx).to(self._owner.points.X.device))
        return [((k, self.label), v) for k, v in zip(self.keys().tolist(), vecs)]

    def count(self):
        return len(self.indices())

    __len__ = count


class _Neighborhoods(dict):
    def __init__(self, points, expanded, ebox=None):
        super().__init__()
        self.points = points
        self._ebox = ebox if ebox is not None else \
            np.array([expanded[L].as_array() for L in sorted(expanded)], np.float64)
        self._cache = None
        for L in sorted(expanded):
            self[L] = _Neighborhood(self, L)

    def _members(self, L):
        if self._cache is None:
            counts, members = _native.halo_members(self.points.X, self._ebox)
            m = members.cpu().numpy()
            off = np.concatenate([[0], np.cumsum(counts)])
            self._cache = [m[off[i]:off[i + 1]] for i in range(len(counts))]
        return self._cache[L]

    def iteritems(self):
        return iter(self.items())


def _partition_records(X, keys, n_parts, members, cluster, params):
    """The reference's per-partition records (R:dbscan/dbscan.py:116-125 with
    dbscan_partition, :12-34): for each neighbourhood L (partitionBy order)
    and each of its points in input order, ``(key, 'L:c')`` or ``(key,
    'L:c*')`` — c the neighbourhood's own sklearn label of the point, '*' a
    non-core point.  members(L) -> ascending point indices of neighbourhood
    L; cluster(X_L, eps, min_samples, metric) -> (labels, core) numpy."""
    recs = []
    metric = _native.metric_code(params.get('metric', 'euclidean'))
    for L in range(n_parts):
        idx = np.asarray(members(L), np.int64)
        if not len(idx):
            continue
        XL = X[torch.from_numpy(idx).to(X.device)].contiguous()
        lab, core = cluster(XL, params['eps'], params['min_samples'], metric)
        recs.extend((k, '%i:%i%s' % (L, c, '' if f else '*'))
                    for k, c, f in zip(keys[idx].tolist(), np.asarray(lab).tolist(),
                                       np.asarray(core).tolist()))
    return recs


def _device_cluster(X, eps, min_samples, metric):
    lab, core, _, _ = _native.cluster(X, eps, min_samples, metric)
    return lab.cpu().numpy(), core.cpu().numpy()


class _PartitionRecords(object):
    """``DBSCAN.data`` after ``train`` (R:dbscan/dbscan.py:116-125): the
    records of the per-partition clustering (_partition_records).  Built
    lazily on first use, one pd_cluster per neighbourhood; the global labels
    never depend on it."""

    def __init__(self, neighbors, params):
        self.neighbors = neighbors
        self.params = params
        self._recs = None

    def _build(self):
        if self._recs is None:
            nb = self.neighbors
            self._recs = _partition_records(nb.points.X, nb.points.key_array(), len(nb),
                                            lambda L: nb[L].indices(), _device_cluster,
                                            self.params)
        return self._recs

    def collect(self):
        return list(self._build())

    def count(self):
        return sum(len(nb) for nb in self.neighbors.values())

    def take(self, k):
        return self._build()[:k]

    def __iter__(self):
        return iter(self._build())


class _ShardedPartitionRecords(_PartitionRecords):
    """``DBSCAN.data`` after a sharded train: the same records as one device
    would give for the union of every rank's slice (global input order =
    rank order), like the reference's one RDD over all executors.  The
    neighbourhoods span ranks, so ``collect()`` / ``take()`` / iteration are
    collectives (every rank calls them): the slices are all-gathered (keys and
    coordinates, the reference's ``collect`` to the driver), then each
    neighbourhood is clustered on this rank's device (``ops``: pd_halo_members
    + pd_cluster).  ``count()`` all-reduces the neighbourhood sizes of the
    local slices (a collective too)."""

    def __init__(self, points, gid_base, ebox, params, group, ops):
        self.points = points
        self.gid_base = gid_base
        self.ebox = np.ascontiguousarray(ebox, np.float64)
        self.params = params
        self.group = group
        self.ops = ops
        self._recs = None

    def _local_keys(self):
        if self.points.keys is None:
            return self.gid_base + np.arange(self.points.n, dtype=np.int64)
        return np.asarray(self.points.key_array())

    def _build(self):
        if self._recs is None:
            import torch.distributed as dist
            parts = [None] * dist.get_world_size(self.group)
            dist.all_gather_object(parts, (self._local_keys(), self.points.X.cpu().numpy()),
                                   group=self.group)
            keys = np.concatenate([p[0] for p in parts])
            X = torch.from_numpy(np.ascontiguousarray(np.concatenate([p[1] for p in parts])))
            X = X.to(self.ops.device)
            counts, members = self.ops.halo_members(X, self.ebox)
            off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
            self._recs = _partition_records(X, keys, len(self.ebox),
                                            lambda L: members[off[L]:off[L + 1]],
                                            self.ops.cluster, self.params)
        return self._recs

    def count(self):
        import torch.distributed as dist
        counts, _ = self.ops.halo_members(self.points.X.to(self.ops.device), self.ebox)
        t = torch.tensor([int(np.sum(counts))], dtype=torch.int64)
        dist.all_reduce(t, group=self.group)
        return int(t.item())


class _Assignments(object):
    """``DBSCAN.result``: (key, cluster id) pairs sorted by key
    (``.sortByKey()``, R:dbscan/dbscan.py:162-164)."""

    def __init__(self, points, labels):
        self.points = points
        self.labels = labels

    def labels_by_key(self):
        lab = self.labels.cpu().numpy().astype(np.int64)
        keys = self.points.key_array()
        if self.points.keys is None:
            return keys, lab
        order = np.argsort(keys, kind="stable")
        return keys[order], lab[order]

    def collect(self):
        keys, lab = self.labels_by_key()
        return list(zip(keys.tolist(), lab.tolist()))

    def count(self):
        return self.points.n


class _ShardedAssignments(object):
    """``DBSCAN.result`` of a sharded train: this rank holds the (key, label)
    pairs of its input slice, like one partition of the reference's result
    RDD.  ``collect()`` / ``count()`` are collectives (every rank calls them)
    and return the whole, sorted by key (R:dbscan/dbscan.py:162-164)."""

    def __init__(self, points, labels, gid_base, n_total, group):
        self.points = points
        self.labels = labels
        self.gid_base = gid_base
        self.n_total = n_total
        self.group = group

    def local(self):
        lab = self.labels.cpu().numpy().astype(np.int64)
        if self.points.keys is None:
            return self.gid_base + np.arange(self.points.n, dtype=np.int64), lab
        return self.points.keys, lab

    def collect(self):
        import torch.distributed as dist
        keys, lab = self.local()
        parts = [None] * dist.get_world_size(self.group)
        dist.all_gather_object(parts, (keys, lab), group=self.group)
        keys = np.concatenate([p[0] for p in parts])
        lab = np.concatenate([p[1] for p in parts])
        order = np.argsort(keys, kind="stable")
        return list(zip(keys[order].tolist(), lab[order].tolist()))

    def count(self):
        return self.n_total


class DBSCAN(object):
    """
    :eps: nearest neighbor radius
    :min_samples: minimum number of samples within radius eps
    :metric: distance metric (euclidean or cityblock, string or scipy callable)
    :max_partitions: maximum number of partitions used by KDPartitioner
    :data: before ``train`` None; after it the reference's per-partition
        records ``(key, 'L:c[*]')`` as an RDD-like object (``collect``,
        ``count``, ``take``, iteration; R:dbscan/dbscan.py:116-125) — after a
        sharded train the same records over all ranks, its calls collectives
    :result: (key, cluster label) pairs, sorted by key, via ``collect()``
    :bounding_boxes: label -> BoundingBox of each KD partition
    :expanded_boxes: label -> BoundingBox grown by 2·eps
    :neighbors: label -> points inside the expanded box
    :cluster_dict: kept for API parity; the reference never assigns it

    MI355X additions: ``labels_`` (device int32, input order),
    ``core_sample_mask_`` (device uint8), ``n_clusters_``.

    ``kd_sums``: KD moment summation.  'exact' (default): correctly rounded,
    order-independent double-double sums — the same boxes on one device or
    many; 'sequential': the reference's left-to-right fold, bit-identical to
    its boxes (on C0 a split the reference decides by round-off differs
    otherwise), single device only.  Never changes the labels.

    Multi-GPU (the reference's fan-out over executors, R:dbscan/dbscan.py:
    104-126) is opt-in:
      * ``group=`` a torch.distributed process group (or ``'world'``), one
        process per GPU (e.g. torchrun): ``train(slice)`` clusters the union
        of every rank's slice; each rank passes its own slice and gets
        ``labels_`` / ``core_sample_mask_`` for it (input order), the global
        ``n_clusters_``, the same ``bounding_boxes`` / ``expanded_boxes``,
        ``neighbors`` over its slice, and a ``result`` whose ``collect()`` (a
        collective) returns every (key, label).  Keys of array input are
        global indices (rank offset + row).  Collectives run on RCCL through
        libpardis (pd_comm_*) for an "nccl" group;
      * ``n_gpus=N > 1`` without a group: this process drives GPUs 0..N-1
        itself (one thread per device, pd_comm_init_all), the input split by
        index;
      * neither: one device — also inside an initialised process group (each
        rank clusters its own data, the reference's single-driver behaviour).
    ``device``: where the points go (default: the current CUDA device).
    ``keep_shard_records``: a sharded train keeps the records each rank owns
    (``shard.gid`` / ``shard.labels`` / ``shard.core``: diagnostics, ~13 B
    of HBM per received record); off by default.
    """

    def __init__(self, eps=0.5, min_samples=5, metric=euclidean, max_partitions=None,
                 kd_sums='exact', n_gpus=None, device=None, group=None, keep_shard_records=False):
        self.eps = eps
        self.keep_shard_records = keep_shard_records
        self.kd_sums = kd_sums
        self.n_gpus = n_gpus
        self.device = device
        self.group = group
        self.min_samples = int(min_samples)
        self.metric = metric
        self.max_partitions = max_partitions
        self.data = None
        self.result = None
        self.bounding_boxes = None
        self.expanded_boxes = None
        self.neighbors = None
        self.cluster_dict = None
        self.labels_ = None
        self.core_sample_mask_ = None
        self.n_clusters_ = None
        self.partitioner = None
        self.shard = None

    def _process_group(self):
        """The process group of an opt-in sharded train: ``group=`` (a
        torch.distributed group, or 'world'), else None — a rank of a
        torchrun / DDP job that does not ask for it clusters its own data on
        its own device, as the reference's ``train`` would."""
        if self.group is None:
            return None
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            raise ValueError("group= needs an initialised torch.distributed process group")
        group = dist.group.WORLD if isinstance(self.group, str) and self.group == "world" \
            else self.group
        if self.n_gpus not in (None, dist.get_world_size(group)):
            raise ValueError(f"n_gpus={self.n_gpus} inside a process group of "
                             f"{dist.get_world_size(group)} ranks")
        return group

    def train(self, data):
        """
        :param data: RDD-like / iterable of (key, vector), or (n, d) array/tensor
        Train the model (R:dbscan/dbscan.py:104-126).
        """
        if not (self.eps > 0):
            raise ValueError("eps must be > 0")
        if self.min_samples < 1:
            raise ValueError("min_samples must be >= 1")
        metric = _native.metric_code(self.metric)
        group = self._process_group()
        if group is not None:
            return self._train_group(data, group, metric)
        if self.n_gpus is not None and int(self.n_gpus) > 1:
            return self._train_devices(data, metric)
        points = as_points(data, self.device)
        parts = KDPartitioner(points, self.max_partitions, sums=self.kd_sums)
        self.partitioner = parts
        self.bounding_boxes = parts.bounding_boxes
        self.expanded_boxes = {L: box.expand(2 * self.eps)
                               for L, box in sorted(parts.bounding_boxes.items())}
        ebox = np.array([self.expanded_boxes[L].as_array() for L in sorted(self.expanded_boxes)],
                        np.float64)
        self.neighbors = _Neighborhoods(points, self.expanded_boxes, ebox)
        # the reference's self.data after train: the per-partition records
        self.data = _PartitionRecords(self.neighbors, {'eps': self.eps,
                                                       'min_samples': self.min_samples,
                                                       'metric': self.metric})
        lo, hi = parts.data_box
        tree = parts.split_tree() if len(ebox) > 1 and points.d <= 4 else None
        if tree is not None:
            # the owner of each point is found by replaying the KD splits in
            # the halo pass (no owner array, no final split pass)
            labels, core, _, ncl = _native.train_tree(points.X, self.eps, self.min_samples, metric,
                                                      ebox, tree, data_box=np.stack([lo, hi]))
        else:
            owner = parts.labels if len(ebox) > 1 else None
            labels, core, _, ncl = _native.train(points.X, self.eps, self.min_samples, metric,
                                                 ebox, owner=owner, data_box=np.stack([lo, hi]))
        self.labels_ = labels
        self.core_sample_mask_ = core
        self.n_clusters_ = ncl
        self.result = _Assignments(points, labels)
        return self

    # ------------------------------------------------------------ multi-GPU
    def _sharded_checks(self, points):
        if self.kd_sums != 'exact':
            raise ValueError("kd_sums='sequential' is single-device (the fold order of one "
                             "slice); the multi-GPU train uses the exact sums")
        P = self.max_partitions if self.max_partitions is not None else 4 ** points.d
        return int(P)

    def _set_sharded(self, points, labels, core, res, result, group=None, ops=None):
        ebox = np.ascontiguousarray(res.boxes, np.float64)
        params = {'eps': self.eps, 'min_samples': self.min_samples, 'metric': self.metric}
        if group is not None:
            self.data = _ShardedPartitionRecords(points, res.gid_base, ebox, params, group, ops)
        else:   # one process holds every slice: the single-device records
            self.data = None
        self.labels_ = labels
        self.core_sample_mask_ = core
        self.n_clusters_ = res.n_clusters
        self.bounding_boxes = res.bounding_boxes
        self.expanded_boxes = {L: box.expand(2 * self.eps)
                               for L, box in sorted(res.bounding_boxes.items())}
        self.neighbors = _Neighborhoods(points, self.expanded_boxes)
        if group is None:
            self.data = _PartitionRecords(self.neighbors, params)
        self.result = result
        self.shard = res
        return self

    def _train_group(self, data, group, metric):
        from . import distributed
        points = as_points(data, self.device)
        P = self._sharded_checks(points)
        res = distributed.train_sharded(points.X, self.eps, self.min_samples, metric=metric,
                                        max_partitions=P, group=group,
                                        keep_owned=self.keep_shard_records)
        result = _ShardedAssignments(points, res.local_labels, res.gid_base, res.n_total, group)
        ops = distributed.NativeOps(points.X.device)
        return self._set_sharded(points, res.local_labels, res.local_core, res, result,
                                 group, ops)

    def _train_devices(self, data, metric):
        from . import distributed
        W = int(self.n_gpus)
        _native.require_gpu()
        if torch.cuda.device_count() < W:
            raise ValueError(f"n_gpus={W} but {torch.cuda.device_count()} GPU(s) are visible")
        points = as_points(data, self.device)
        P = self._sharded_checks(points)
        n = points.n
        cuts = [r * n // W for r in range(W + 1)]
        # a slice moved to another device is a fresh allocation already; one
        # left on its device is a view at an offset, which train_sharded
        # realigns (copies once) when it is not 16-byte aligned — no second
        # full copy of every slice here (transient 2x HBM at C4 scale)
        slices = [points.X[cuts[r]:cuts[r + 1]].to(torch.device("cuda", r)) for r in range(W)]
        torch.cuda.synchronize(points.X.device)
        comms = distributed.device_comms(range(W))
        ops = [distributed.NativeOps(torch.device("cuda", r)) for r in range(W)]
        res = distributed.train_threads(slices, self.eps, self.min_samples, comms, ops,
                                        metric=metric, max_partitions=P,
                                        keep_owned=self.keep_shard_records)
        dev = points.X.device
        labels = torch.cat([r.local_labels.to(dev) for r in res])
        core = torch.cat([r.local_core.to(dev) for r in res])
        return self._set_sharded(points, labels, core, res[0], _Assignments(points, labels))

    def assignments(self):
        """
        :rtype: list
        :return: list of (key, cluster_id), sorted by key
        """
        return self.result.collect()
