"""Sharded train: one process per GPU, torch.distributed for the exchanges.

The reference spreads its work over Spark executors: the KD partitioner's
aggregates run over every RDD slice (R:dbscan/partition.py:60-63,86-89), the
halo records are shuffled with ``partitionBy(max_partitions)``
(R:dbscan/dbscan.py:114-118), every partition is clustered where it lands
(R:dbscan/dbscan.py:12-34) and the driver merges the cluster ids
(R:dbscan/dbscan.py:153-165, R:dbscan/aggregator.py:9-73).  Here each rank
holds a slice of the points in its GPU's HBM and the same steps are:

  1. bbox: one all-reduce (min / max / non-finite count);
  2. KD levels: per level one all-gather of the double-double moment partials
     (added exactly, so the split axes and bounds equal the single-device
     ones bit for bit) and one all-reduce of the seven-bound counts;
  3. routing: neighbourhood L goes to rank ``L * world // P``; every point
     travels once to each rank whose neighbourhoods' 2·eps boxes hold it
     (pd_route / pd_pack), one all-to-all-v per field;
  4. phase A on each rank (pd_train_begin): grid, counts, union-find, local
     component keys; export (global id, key) of core points that also live on
     another rank;
  5. one all-gather of the exports; every rank builds the same global key map
     (pd_merge_exports) — the RCCL label merge;
  6. phase B (pd_train_end): border attach with global keys;
  7. labels: all-gather of the cluster roots (one id per cluster), sorted, and
     each key's rank is its label (pd_select_roots / pd_sort_u32 /
     pd_rank_labels) — sklearn's numbering, as the single-device pd_train.

Result: each rank returns the global ids and labels of the points it owns
(every point is owned by exactly one rank: the one holding its KD partition).

d > 4 (the dense tile path) shares steps 1-2 (the KD boxes of the API) and
then all-gathers the slices: the distance tiles need every point on every
GPU, and each rank computes its share of the tile rows (``_train_dense``).

The device work goes through an ``ops`` object (``NativeOps``: libpardis on
this rank's GPU).  Collectives run on ``comm_device``: the GPU under RCCL
("nccl"), the host under gloo.
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.distributed as dist

from . import _native
from .geometry import BoundingBox
from .partition import (_split_schedule, apply_level, apply_rotation_level, level_axes,
                        level_boundaries, level_medians)


class NativeOps(object):
    """The per-rank device stages (libpardis through the C ABI)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.ctx = _native.context(self.device.index)

    # -- buffers
    def empty(self, n, dtype, d=None):
        shape = (n, d) if d is not None else (n,)
        return torch.empty(shape, dtype=dtype, device=self.device)

    def zeros(self, n, dtype):
        return torch.zeros(n, dtype=dtype, device=self.device)

    # -- KD passes
    def bbox(self, X):
        return _native.bbox(X, ctx=self.ctx)

    def moments_dd(self, X, labels, sel):
        return _native.kd_moments_dd(X, labels, sel, ctx=self.ctx)

    def level_pass(self, X, labels, split, sel, labels_zero=False, bbox=False):
        return _native.kd_pass(X, labels, split=split, sel=sel, labels_zero=labels_zero,
                               bbox=bbox, ctx=self.ctx)

    def counts(self, X, labels, sel, axes, bounds):
        return _native.kd_counts(X, labels, sel, axes, bounds, ctx=self.ctx)

    def radix_hist(self, X, labels, sel, axes, prefix, shift):
        return _native.kd_radix_hist(X, labels, sel, axes, prefix, shift, ctx=self.ctx)

    def split(self, X, labels, sel, axes, boundary, new):
        _native.kd_split(X, labels, sel, axes, boundary, new, ctx=self.ctx)

    # -- routing
    def route(self, X, ebox, part_rank, world):
        return _native.route(X, ebox, part_rank, world, ctx=self.ctx)

    def pack(self, X, mask, dest, kdlab, part_rank, local_index, gid_base, out):
        return _native.pack(X, mask, dest, kdlab, part_rank, local_index, gid_base, out,
                            ctx=self.ctx)

    # -- clustering phases
    def train_begin(self, X, eps, min_samples, metric, ebox, owner, gid, xr, data_box):
        return _native.train_begin(X, eps, min_samples, metric, ebox, owner, gid, xr, data_box,
                                   ctx=self.ctx)

    def exports(self, m):
        return _native.train_exports(m, self.device, ctx=self.ctx)

    def merge(self, gid, key):
        return _native.merge_exports(gid, key, ctx=self.ctx)

    def train_end(self, n, keymap):
        return _native.train_end(n, keymap, self.device, ctx=self.ctx)

    def select_roots(self, keys, gid):
        return _native.select_roots(keys, gid, ctx=self.ctx)

    def sort(self, data):
        return _native.sort_u32(data, ctx=self.ctx)

    def rank_labels(self, keys, roots):
        return _native.rank_labels(keys, roots, ctx=self.ctx)

    def owned_results(self, owner, gid, labels, core, gid_offsets):
        return _native.owned_results(owner, gid, labels, core, gid_offsets, ctx=self.ctx)

    def scatter_results(self, pairs, gid_base, n):
        return _native.scatter_results(pairs, gid_base, n, self.device, ctx=self.ctx)

    # -- dense (d > 4) stages
    def dense_count(self, X, eps, min_samples, metric, data_box, rank, world):
        return _native.dense_count(X, eps, min_samples, metric, data_box, rank, world,
                                   ctx=self.ctx)

    def dense_link(self, counts):
        return _native.dense_link(counts, ctx=self.ctx)

    def dense_border(self, forests, n_forests, n):
        return _native.dense_border(forests, n_forests, n, ctx=self.ctx)

    def dense_finish(self, best, n):
        labels, core, _, ncl = _native.dense_finish(best, n, self.device, ctx=self.ctx)
        return labels, core, ncl

    def timings(self):
        return self.ctx.timings()


# ------------------------------------------------------------------ helpers
def _two_sum(a, b):
    s = a + b
    bb = s - a
    return s, (a - (s - bb)) + (b - bb)


def dd_combine(parts):
    """Add per-rank double-double partials (W, S, 1 + 4d) in rank order and
    round once: (S, 3, d) moments = {count, Σv, Σv²} (kd.hip dd_add)."""
    parts = np.asarray(parts, np.float64)
    W, S, G = parts.shape
    d = (G - 1) // 4
    cnt = np.zeros(S)
    hs = np.zeros((S, 2 * d))
    ls = np.zeros((S, 2 * d))
    for w in range(W):
        p = parts[w]
        cnt = cnt + p[:, 0]
        bh = p[:, 1::2]
        bl = p[:, 2::2]
        s, e = _two_sum(hs, bh)
        e = e + (ls + bl)
        hi = s + e
        ls = e - (hi - s)
        hs = hi
    tot = hs + ls
    mom = np.empty((S, 3, d))
    mom[:, 0, :] = cnt[:, None]
    mom[:, 1, :] = tot[:, :d]
    mom[:, 2, :] = tot[:, d:]
    return mom


def partition_ranks(P, world):
    """Neighbourhood -> rank (contiguous blocks of KD labels) and each
    neighbourhood's index among its rank's neighbourhoods."""
    part_rank = np.array([L * world // P for L in range(P)], np.int32)
    local_index = np.zeros(P, np.int32)
    for r in range(world):
        idx = np.nonzero(part_rank == r)[0]
        local_index[idx] = np.arange(len(idx), dtype=np.int32)
    return part_rank, local_index


_TORCH_OPS = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}


class _TorchComm(object):
    """Collectives through a torch.distributed process group (gloo on the
    host: the CPU tests; any backend without device buffers)."""

    def __init__(self, group, device):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        backend = dist.get_backend(group)
        self.device = torch.device(device) if backend == "nccl" else torch.device("cpu")

    def to(self, t):
        return t.to(self.device)

    def all_reduce(self, arr, op):
        t = torch.as_tensor(np.ascontiguousarray(arr)).to(self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM,
                        group=self.group)
        return t.cpu().numpy()

    def all_reduce_t(self, t, op):
        """Element-wise reduction ("sum", "min", "max") of a tensor over the
        ranks; returns the result on the collective's device."""
        r = self.to(t).contiguous().clone()
        dist.all_reduce(r, op=_TORCH_OPS[op], group=self.group)
        return r

    def all_gather_np(self, arr):
        t = torch.as_tensor(np.ascontiguousarray(arr)).to(self.device)
        outs = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(outs, t, group=self.group)
        return np.stack([o.cpu().numpy() for o in outs])

    def all_gather_var(self, t):
        """Concatenate tensors of different lengths (dim 0) from every rank."""
        sizes = self.all_gather_np(np.array([t.shape[0]], np.int64))[:, 0]
        mx = max(int(sizes.max()), 1)
        buf = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=self.device)
        buf[:t.shape[0]] = self.to(t)
        outs = [torch.empty_like(buf) for _ in range(self.world)]
        dist.all_gather(outs, buf, group=self.group)
        return torch.cat([o[:int(s)] for o, s in zip(outs, sizes)])

    def all_to_all_v(self, send, send_counts, recv_counts):
        """Rows of `send` grouped by destination -> rows grouped by source."""
        row = tuple(send.shape[1:])
        w = int(np.prod(row)) if row else 1
        recv = torch.empty(int(sum(recv_counts)) * w, dtype=send.dtype, device=self.device)
        dist.all_to_all_single(recv, self.to(send.reshape(-1)),
                               output_split_sizes=[int(c) * w for c in recv_counts],
                               input_split_sizes=[int(c) * w for c in send_counts],
                               group=self.group)
        return recv.reshape((-1,) + row)


class RcclComm(object):
    """Collectives through libpardis's RCCL communicator (pd_comm_*): device
    buffers on this rank's GPU, grouped point-to-point sends for the
    variable-size exchanges.  torch.distributed only hands the 128-byte
    RCCL id from rank 0 to the others."""

    def __init__(self, comm):
        self.comm = comm
        self.world = comm.world
        self.rank = comm.rank
        self.device = comm.device

    @classmethod
    def from_group(cls, group, device):
        device = torch.device(device)
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        uid = _native.comm_unique_id() if rank == 0 else bytes(_native.PD_COMM_ID_BYTES)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        if dist.get_backend(group) == "nccl":
            t = t.to(device)
        dist.broadcast(t, dist.get_global_rank(group, 0) if group is not None else 0,
                       group=group)
        return cls(_native.Comm.init(world, rank, bytes(t.cpu().tolist()), device.index))

    def to(self, t):
        return t.to(self.device)

    def all_reduce(self, arr, op):
        t = torch.as_tensor(np.ascontiguousarray(arr)).to(self.device)
        self.comm.all_reduce(t, _native.PD_R_MAX if op == "max" else _native.PD_R_SUM)
        return t.cpu().numpy()

    def all_reduce_t(self, t, op):
        r = self.to(t).contiguous().clone()
        code = {"sum": _native.PD_R_SUM, "min": _native.PD_R_MIN, "max": _native.PD_R_MAX}[op]
        self.comm.all_reduce(r, code)
        return r

    def all_gather_np(self, arr):
        a = np.ascontiguousarray(arr)
        t = torch.as_tensor(a.reshape(1, -1) if a.ndim == 0 else a[None]).to(self.device)
        out = self.comm.all_gather_v(t, [1] * self.world)
        return out.cpu().numpy()

    def all_gather_var(self, t):
        sizes = self.all_gather_np(np.array([t.shape[0]], np.int64))[:, 0]
        return self.comm.all_gather_v(self.to(t).contiguous(), sizes)

    def all_to_all_v(self, send, send_counts, recv_counts):
        return self.comm.all_to_all_v(self.to(send).contiguous(), send_counts, recv_counts)


_rccl_cache = {}


def make_comm(group, device):
    """RCCL (pd_comm) for an "nccl" group on GPU ranks, torch.distributed
    otherwise.  The RCCL communicator is built once per (group, device)."""
    device = torch.device(device)
    if dist.get_backend(group) == "nccl" and device.type == "cuda":
        key = (id(group), device.index)
        if key not in _rccl_cache:
            _rccl_cache[key] = RcclComm.from_group(group, device)
        return _rccl_cache[key]
    return _TorchComm(group, device)


class ShardedResult(object):
    """Per-rank output of ``train_sharded``.

    :gid: global ids of the points this rank owns (ascending)
    :labels: their DBSCAN labels (sklearn numbering over all points, -1 noise)
    :core: their core flags
    :local_labels, local_core: labels / core flags of this rank's INPUT
        points in input order (returned by the owners; None when
        ``return_local`` was off)
    :gid_base: global id of this rank's first input point
    :n_total: points over all ranks
    :n_clusters: number of clusters over all points
    :splits: the KD trace (identical on every rank)
    :bounding_boxes: label -> BoundingBox of each KD partition
    :boxes: (P, 2, d) expanded boxes
    """

    def __init__(self, **kw):
        self.__dict__.update(kw)


def train_sharded(X, eps, min_samples, metric=_native.PD_EUCLIDEAN, max_partitions=None,
                  group=None, ops=None, split_method='min_var', comm=None, return_local=True):
    """Sharded DBSCAN train over the ranks of ``group`` (default: world).

    X: this rank's (n_i, d) slice (float32/float64, on this rank's GPU for
    NativeOps); the global id of row j is sum(n_0 .. n_{i-1}) + j.
    ``max_partitions`` defaults to the world size (one KD partition per GPU).
    ``split_method``: 'min_var' (default) or 'rotation' (KDPartitioner's).
    ``comm``: a collective layer (make_comm(group, device) by default: RCCL
    through libpardis for an "nccl" group, torch.distributed otherwise).
    """
    if split_method not in ('min_var', 'rotation'):
        split_method = 'min_var'   # the reference's fallback (R:dbscan/partition.py:129-130)
    if X.dim() != 2:
        raise ValueError("X must be an (n, d) tensor")
    ops = ops or NativeOps(X.device)
    comm = comm or make_comm(group, getattr(ops, "device", X.device))
    W, rank = comm.world, comm.rank
    n, d = X.shape
    P = int(max_partitions) if max_partitions is not None else W
    if P < 1:
        raise ValueError("max_partitions must be >= 1")
    if P > 64 * 1024:
        raise ValueError("max_partitions too large")
    metric = _native.metric_code(metric) if not isinstance(metric, int) else metric
    stats = {}
    clock = [time.perf_counter()]

    def lap(name):   # host wall time per phase (each phase ends in a host sync)
        now = time.perf_counter()
        stats[name + "_ms"] = round(1e3 * (now - clock[0]), 3)
        clock[0] = now

    # ---- global ids
    sizes = comm.all_gather_np(np.array([n], np.int64))[:, 0]
    gid_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    gid_base = int(gid_off[rank])
    n_total = int(gid_off[-1])
    if n_total >= 0xFFFFFFFF:
        raise ValueError("the sharded train addresses points with 32-bit global ids")

    # ---- bbox (R:dbscan/partition.py:135-137), fused into the first
    # level's moments pass for min_var
    kdlab = ops.zeros(n, torch.int32)
    levels = _split_schedule(P)
    fused = split_method == 'min_var'
    first = None
    if n and fused and levels:
        first, lo, hi, bad = ops.level_pass(X, kdlab, None, [0], True, True)
    elif n:
        lo, hi, bad = ops.bbox(X)
    else:
        lo, hi, bad = np.full(d, np.inf), np.full(d, -np.inf), 0
    # one all-reduce (max) of (-lo, hi, non-finite count): any count > 0 fails
    ext = comm.all_reduce(np.concatenate([-np.asarray(lo, np.float64),
                                          np.asarray(hi, np.float64), [float(bad)]]), "max")
    nbad = ext[2 * d]
    if nbad:
        raise ValueError("Input contains NaN or infinity.")
    if n_total == 0:
        raise ValueError("no points on any rank")
    data_box = np.concatenate([-ext[:d], ext[d:2 * d]])
    box = BoundingBox(k=d).union(BoundingBox(data_box[:d], data_box[d:]))

    # ---- KD partition (R:dbscan/partition.py:139-183): per level one fused
    # pass (the previous level's split + this level's moments) and one counts
    # pass; the last split runs alone
    boxes = {0: box}
    splits = []
    fp32 = X.dtype == torch.float32
    pending = None
    for depth, level in enumerate(levels):
        sel = [c for c, _ in level]
        new = [nl for _, nl in level]
        if split_method == 'rotation':
            # median per split from all-reduced digit histograms: the same
            # sorted_values[len/2] as one device (R:dbscan/partition.py:23-26)
            axes = [depth % d] * len(sel)

            def hist(prefix, shift):
                h = ops.radix_hist(X, kdlab, sel, axes, prefix, shift) if n else \
                    np.zeros((len(sel), 256), np.int64)
                return comm.all_reduce(np.asarray(h, np.int64), "sum")

            med, less, tot = level_medians(hist, len(sel), fp32)
            if n:
                ops.split(X, kdlab, sel, axes, med, new)
            apply_rotation_level(boxes, splits, level, axes, med, less, tot)
            continue
        if not n:
            part = np.zeros((len(sel), 1 + 4 * d))
        elif depth == 0 and first is not None:
            part = first
        else:
            part = ops.level_pass(X, kdlab, pending, sel)
        mom = dd_combine(comm.all_gather_np(part))
        axes, means, vars_, bounds = level_axes(mom)
        cnt = ops.counts(X, kdlab, sel, axes, bounds) if n else np.zeros((len(sel), 8), np.int64)
        cnt = comm.all_reduce(cnt.astype(np.int64), "sum")
        boundary, cand = level_boundaries(cnt, bounds)
        pending = (sel, axes, boundary, new)
        apply_level(boxes, splits, level, axes, means, vars_, cnt, cand, boundary)
    dense = d > 4
    if pending is not None and n and not dense:
        ops.split(X, kdlab, *pending)
    ebox = np.stack([boxes[L].expand(2 * eps).as_array() for L in sorted(boxes)])
    lap("kd")
    if dense:
        return _train_dense(X, eps, min_samples, metric, comm, ops, gid_off, data_box,
                            dict(splits=splits, bounding_boxes=boxes, boxes=ebox), stats, lap)

    # ---- route + exchange (R:dbscan/dbscan.py:114-118,136-151)
    part_rank, local_index = partition_ranks(P, W)
    if n:
        mask, send_counts = ops.route(X, ebox, part_rank, W)
    else:
        mask, send_counts = None, np.zeros(W, np.int64)
    tot = int(send_counts.sum())
    s_coords = ops.empty(tot, X.dtype, d)
    s_gid = ops.empty(tot, torch.int32)
    s_owner = ops.empty(tot, torch.int32)
    s_xr = ops.empty(tot, torch.uint8)
    off = 0
    for dest in range(W):
        c = int(send_counts[dest])
        if c and n:
            m = ops.pack(X, mask, dest, kdlab, part_rank, local_index, gid_base,
                         (s_coords[off:off + c], s_gid[off:off + c], s_owner[off:off + c],
                          s_xr[off:off + c]))
            if m != c:
                raise RuntimeError(f"pack: {m} points for rank {dest}, route said {c}")
        off += c
    recv_counts = comm.all_gather_np(send_counts.astype(np.int64))[:, rank].astype(np.int64)
    dev = getattr(ops, "device", X.device)
    Xr = comm.all_to_all_v(s_coords, send_counts, recv_counts).to(dev).reshape(-1, d)
    gid = comm.all_to_all_v(s_gid, send_counts, recv_counts).to(dev)
    owner = comm.all_to_all_v(s_owner, send_counts, recv_counts).to(dev)
    xr = comm.all_to_all_v(s_xr, send_counts, recv_counts).to(dev)
    del s_coords, s_gid, s_owner, s_xr, mask
    nr = int(recv_counts.sum())
    stats["sent"], stats["received"] = tot, nr
    lap("exchange")

    # ---- phase A on this rank's neighbourhoods
    mine = [L for L in range(P) if part_rank[L] == rank]
    if mine:
        n_exp = ops.train_begin(Xr.contiguous(), eps, min_samples, metric, ebox[mine], owner,
                                gid, xr, data_box)
        e_gid, e_key = ops.exports(n_exp)
    else:
        e_gid = ops.empty(0, torch.int32)
        e_key = ops.empty(0, torch.int32)
    stats["exports"] = int(e_gid.shape[0])
    lap("phase_a")

    # ---- global key merge (R:dbscan/dbscan.py:153-165): one gather of the
    # (id, key) pairs, then the same O(exports) union on every rank
    ex = comm.all_gather_var(torch.stack([e_gid, e_key], 1)).to(dev)
    keymap = ops.merge(ex[:, 0].contiguous(), ex[:, 1].contiguous()) if ex.shape[0] else None
    stats["exports_total"] = int(ex.shape[0])
    lap("merge")

    # ---- phase B, labels
    if mine:
        keys, core = ops.train_end(nr, keymap)
    else:
        keys, core = ops.empty(0, torch.int32), ops.empty(0, torch.uint8)
    roots = ops.select_roots(keys, gid) if nr else ops.empty(0, torch.int32)
    all_roots = comm.all_gather_var(roots).to(dev).contiguous()
    ops.sort(all_roots)
    # one root per cluster over all ranks: only owned records carry keys
    # (shard.hip IsRoot); a duplicate would double-count a cluster
    if all_roots.shape[0] > 1 and bool((all_roots[1:] == all_roots[:-1]).any()):
        raise RuntimeError("sharded train: a cluster root was selected on two ranks")
    labels = ops.rank_labels(keys, all_roots) if nr else ops.empty(0, torch.int32)
    own = owner >= 0
    lap("phase_b")

    # ---- results back to the ranks that hold the points, in input order
    # (the reference's result RDD, R:dbscan/dbscan.py:162-164)
    loc_labels = loc_core = None
    if return_local:
        pairs, back = ops.owned_results(owner, gid, labels, core, gid_off)
        got = comm.all_gather_np(back.astype(np.int64))[:, rank].astype(np.int64)
        pairs_in = comm.all_to_all_v(pairs, back, got).to(dev)
        loc_labels, loc_core = ops.scatter_results(pairs_in, gid_base, n)
        lap("results")
    return ShardedResult(gid=gid[own], labels=labels[own], core=core[own],
                         local_labels=loc_labels, local_core=loc_core, gid_base=gid_base,
                         n_total=n_total, n_clusters=int(all_roots.shape[0]), splits=splits,
                         bounding_boxes=boxes, boxes=ebox, stats=stats)


def _train_dense(X, eps, min_samples, metric, comm, ops, gid_off, data_box, kd, stats, lap):
    """d > 4 (the dense MFMA tile path, dense.hip): the tiles need every point,
    so the slices are all-gathered (1M x 64-D fp32 is 256 MB per GPU) and each
    rank computes its share of the tile rows (row chunks dealt round-robin,
    pd_dense_*).  Four stages, one collective between each: counts (sum),
    core forests (gather), border keys (min).  Every rank ends with the labels
    of all points — sklearn's over the union — and returns its slice's."""
    W, rank = comm.world, comm.rank
    n = X.shape[0]
    n_total = int(gid_off[-1])
    dev = getattr(ops, "device", X.device)
    Xf = comm.all_gather_var(X.contiguous()).to(dev).contiguous()
    stats["received"] = int(Xf.shape[0])
    lap("exchange")
    cnt = ops.dense_count(Xf, eps, min_samples, metric, data_box, rank, W)
    cnt = comm.all_reduce_t(cnt, "sum").to(dev)
    lap("count")
    forest = ops.dense_link(cnt)
    forests = comm.all_gather_var(forest).to(dev)
    stats["exports"] = int(forest.shape[0])
    lap("link")
    best = ops.dense_border(forests, W, n_total)
    best = comm.all_reduce_t(best, "min").to(dev)
    labels, core, ncl = ops.dense_finish(best, n_total)
    lap("border")
    lo = int(gid_off[rank])
    loc_labels, loc_core = labels[lo:lo + n], core[lo:lo + n]
    gid = torch.arange(lo, lo + n, dtype=torch.int32, device=dev)
    return ShardedResult(gid=gid, labels=loc_labels, core=loc_core, local_labels=loc_labels,
                         local_core=loc_core, gid_base=lo, n_total=n_total, n_clusters=ncl,
                         stats=stats, **kd)


def train_threads(slices, eps, min_samples, comms, ops, metric=_native.PD_EUCLIDEAN,
                  max_partitions=None, split_method='min_var'):
    """One process driving several devices: rank r = thread r runs
    ``train_sharded`` on slices[r] with comms[r] (e.g. RcclComm over
    pd_comm_init_all) and ops[r].  Returns the per-rank results in rank order;
    the first rank error is raised (after every thread has finished)."""
    import threading

    W = len(slices)
    out, errs = [None] * W, [None] * W

    def body(r):
        try:
            dev = getattr(ops[r], "device", None)
            if dev is not None and torch.device(dev).type == "cuda":
                torch.cuda.set_device(torch.device(dev))
            out[r] = train_sharded(slices[r], eps, min_samples, metric=metric,
                                   max_partitions=max_partitions, ops=ops[r], comm=comms[r],
                                   split_method=split_method)
        except BaseException as e:   # noqa: B902 - re-raised below
            errs[r] = e

    ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(W)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in errs:
        if e is not None:
            raise e
    return out


_device_comms = {}


def device_comms(devices):
    """RCCL communicators of one process over `devices` (cached)."""
    key = tuple(int(d) for d in devices)
    if key not in _device_comms:
        _device_comms[key] = [RcclComm(c) for c in _native.Comm.init_all(list(key))]
    return _device_comms[key]
