"""Sharded train: one process per GPU, torch.distributed for the exchanges.

The reference spreads its work over Spark executors: the KD partitioner's
aggregates run over every RDD slice (R:dbscan/partition.py:60-63,86-89), the
halo records are shuffled with ``partitionBy(max_partitions)``
(R:dbscan/dbscan.py:114-118), every partition is clustered where it lands
(R:dbscan/dbscan.py:12-34) and the driver merges the cluster ids
(R:dbscan/dbscan.py:153-165, R:dbscan/aggregator.py:9-73).  Here each rank
holds a slice of the points in its GPU's HBM and the same steps are:

  1. bbox (min / max / non-finite count): part of the first KD level's
     gather (min_var), else one all-reduce;
  2. KD levels (pd_kdx_*): per level one all-gather of the double-double
     moment partials (added exactly, so the split axes and bounds equal the
     single-device ones bit for bit) and one all-reduce of the seven-bound
     counts, both as device tensors, the decisions on the device — no host
     round trip until the KD trace is read at the end;
  3. routing: neighbourhood L goes to rank ``L * world // P``; every point
     travels once to each rank whose neighbourhoods' 2·eps boxes hold it
     (pd_route2 / pd_pack2: one ordered pass, the self block packed in place),
     one grouped exchange of all fields (pd_comm_exchange);
  4. phase A on each rank (pd_train_begin): grid, counts, union-find, local
     component keys; export (global id, key) of core points that also live on
     another rank;
  5. one all-gather of the exports; every rank builds the same global key map
     (pd_merge_exports) — the RCCL label merge;
  6. phase B (pd_train_end): border attach with global keys;
  7. labels: all-gather of the cluster roots (one id per cluster), sorted, and
     each key's rank is its label — sklearn's numbering, as the single-device
     pd_train; the owned records of this rank's own block are labelled in
     place, the others go back to their source rank as (gid, label) pairs in
     one exchange (pd_results / pd_results_scatter).

Result: each rank returns the labels of its input slice, in input order
(every point is owned by exactly one rank: the one holding its KD partition).

d > 4 (the dense tile path) shares steps 1-2 (the KD boxes of the API) and
then all-gathers the slices: the distance tiles need every point on every
GPU, and each rank computes its share of the tile rows (``_train_dense``).

The device work goes through an ``ops`` object (``NativeOps``: libpardis on
this rank's GPU).  Collectives run on ``comm_device``: the GPU under RCCL
("nccl"), the host under gloo.
"""
from __future__ import annotations

import heapq
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

    # -- per-neighbourhood records (DBSCAN.data after a sharded train)
    def halo_members(self, X, ebox):
        counts, members = _native.halo_members(X, ebox, ctx=self.ctx)
        return counts, members.cpu().numpy()

    def cluster(self, X, eps, min_samples, metric):
        lab, core, _, _ = _native.cluster(X, eps, min_samples, metric, ctx=self.ctx)
        return lab.cpu().numpy(), core.cpu().numpy()

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

    def train_end(self, n, keymap, n_total=None):
        # global ids below 2^31: the core flags ride the keys' top bit
        self.ctx.set_option(_native.PD_OPT_SHARD_CORE_BIT,
                            1 if n_total is not None and n_total < (1 << 31) else 0)
        return _native.train_end(n, keymap, self.device, ctx=self.ctx)

    def select_roots(self, keys, gid):
        return _native.select_roots(keys, gid, ctx=self.ctx)

    # -- device-decided KD, one-pass exchange, results (pd_kdx_*, pd_route2,
    # pd_pack2, pd_results*)
    def kdx_begin(self, d, levels):
        _native.kdx_begin(d, levels, self.device.index, ctx=self.ctx)

    def kdx_moments(self, X, labels, level, S):
        return _native.kdx_moments(X, labels, level, S, ctx=self.ctx)

    def kdx_axes(self, gathered, n_ranks, level):
        _native.kdx_axes(gathered, n_ranks, level, ctx=self.ctx)

    def kdx_counts(self, X, labels, level, S):
        return _native.kdx_counts(X, labels, level, S, ctx=self.ctx)

    def kdx_boundary(self, counts, level):
        _native.kdx_boundary(counts, level, ctx=self.ctx)

    def kdx_end(self, X, labels, n_splits, final_split):
        return _native.kdx_end(X, labels, n_splits, final_split, ctx=self.ctx)

    def route2(self, X, ebox, part_rank, kdlab, world):
        return _native.route2(X, ebox, part_rank, kdlab, world, ctx=self.ctx)

    def pack2(self, X, kdlab, part_rank, local_index, gid_base, outs):
        _native.pack2(X, kdlab, part_rank, local_index, gid_base, outs, ctx=self.ctx)

    def results(self, keys, core, owner, gid, roots, n_total, gid_base, n_local, world, rank,
                src_off, expect_remote):
        return _native.results(keys, core, owner, gid, roots, n_total, gid_base, n_local, world,
                               rank, src_off, expect_remote, self.device.index, ctx=self.ctx)

    def results_scatter(self, pairs, gid_base, labels, core):
        _native.results_scatter(pairs, gid_base, labels, core, ctx=self.ctx)

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


def partition_ranks(P, world, weights=None, order=None, method=None, chosen=None):
    """Neighbourhood -> rank, and each neighbourhood's index among its rank's
    neighbourhoods (ascending label, so a rank's records keep the KD order).

    Without weights, or with P <= world: contiguous blocks of KD labels.  With
    weights (points per KD leaf) and P > world — the static analogue of Spark
    scheduling the reference's P partition tasks over its executors as they
    free up (R:dbscan/dbscan.py:116-124):
      'ordered' — the leaves in the KD tree's spatial (depth-first) order
          (``order``, kd_leaf_order) cut into world contiguous runs with the
          smallest possible largest load: each rank holds a spatially compact
          group of leaves, so few points are routed to two ranks;
      'lpt' — longest-processing-time-first: leaves by decreasing weight
          (ties: smaller label), each to the least-loaded rank (ties: smaller
          rank); the better balance on skewed leaves, at no locality;
      None — 'ordered' unless its largest load exceeds LPT's by more than 5 %.
    ``chosen``: an optional dict that receives {'placement': the method used}.
    Labels do not depend on the placement (any assignment is exact).
    Cost: O(P log P) for both methods (P up to 65536 leaves)."""
    used = "blocks"
    if weights is None or P <= world:
        part_rank = np.array([L * world // P for L in range(P)], np.int32)
    else:
        w = np.asarray(weights, np.float64)
        if w.shape != (P,):
            raise ValueError("one weight per partition expected")
        lpt = np.zeros(P, np.int32)
        # heaviest first onto the least-loaded rank (a heap of (load, rank):
        # ties go to the smaller rank, as argmin's first minimum did)
        heap = [(0.0, r) for r in range(world)]
        for L in np.lexsort((np.arange(P), -w)):
            load, r = heapq.heappop(heap)
            lpt[L] = r
            heapq.heappush(heap, (load + w[L], r))
        part_rank, used = lpt, "lpt"
        if method in (None, "ordered") and order is not None:
            ordd = _ordered_cut(w, order, world)
            lo = np.bincount(ordd, weights=w, minlength=world).max()
            ll = np.bincount(lpt, weights=w, minlength=world).max()
            if method == "ordered" or lo <= 1.05 * ll:
                part_rank, used = ordd, "ordered"
    if chosen is not None:
        chosen["placement"] = used
    local_index = np.zeros(P, np.int32)
    for r in range(world):
        idx = np.nonzero(part_rank == r)[0]
        local_index[idx] = np.arange(len(idx), dtype=np.int32)
    return part_rank, local_index


def _greedy_runs(S, V):
    """Run starts of the greedy cut of prefix sums S into runs of weight <= V
    (each run as long as it may be)."""
    P = len(S) - 1
    starts, i = [], 0
    while i < P:
        starts.append(i)
        j = int(np.searchsorted(S, S[i] + V, side="right")) - 1
        i = max(j, i + 1)   # a run holds at least one leaf
    return starts


def _ordered_cut(w, order, world):
    """Leaves in `order` cut into min(world, P) non-empty contiguous runs with
    the smallest possible largest run weight; run k -> rank k.

    The smallest feasible bound V is found by bisection over the real line
    with the greedy cut as the feasibility test (a cut into <= K runs of
    weight <= V exists iff the greedy one uses <= K runs; monotone in V), so
    the cost is O(K log P) per step and O(P) memory — no (P+1)^2 tables.
    Runs are then split (never raising the largest) until there are K."""
    order = np.asarray(order, np.int64)
    ws = np.asarray(w, np.float64)[order]
    P = len(ws)
    K = min(world, P)
    S = np.concatenate([[0.0], np.cumsum(ws)])
    lo, hi = float(ws.max()), float(S[-1])
    if len(_greedy_runs(S, lo)) > K:
        for _ in range(200):
            mid = 0.5 * (lo + hi)
            if not lo < mid < hi:
                break
            if len(_greedy_runs(S, mid)) <= K:
                hi = mid
            else:
                lo = mid
        V = hi
    else:
        V = lo
    starts = _greedy_runs(S, V)
    # fewer than K runs: split the last multi-leaf runs until there are K
    bounds = starts + [P]
    while len(bounds) - 1 < K:
        for k in range(len(bounds) - 2, -1, -1):
            if bounds[k + 1] - bounds[k] > 1:
                bounds.insert(k + 1, bounds[k + 1] - 1)
                break
    part_rank = np.zeros(len(ws), np.int32)
    for k in range(K):
        part_rank[order[bounds[k]:bounds[k + 1]]] = k
    return part_rank


def kd_leaf_order(splits):
    """KD leaves in depth-first (spatial) order: a split (cur -> cur, new)
    replaces cur by [cur (v < boundary), new] (R:dbscan/partition.py:66-68).
    Built from the tree in O(P): a label's later splits nest inside it, so
    label L expands to L, then the subtrees of its new labels, latest first."""
    kids = {}
    for sp in splits:
        kids.setdefault(int(sp[0]), []).append(int(sp[1]))
    seq, stack = [], [0]
    while stack:
        L = stack.pop()
        seq.append(L)
        stack.extend(kids.get(L, ()))   # popped latest-first
    return seq


def leaf_sizes(splits, n_total, P):
    """Points per KD leaf from the split trace (R:dbscan/partition.py:151-152:
    each split leaves n_left points with the label and moves n_right to the
    new one) — equal on every rank (the trace's counts are global)."""
    size = np.zeros(P, np.int64)
    size[0] = n_total
    for sp in splits:
        cur, nl, n_left, n_right = sp[0], sp[1], sp[4], sp[5]
        size[cur] = n_left
        size[nl] = n_right
    return size


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
        if op not in _TORCH_OPS:
            raise ValueError(f"unknown reduction {op!r}")
        t = torch.as_tensor(np.ascontiguousarray(arr)).to(self.device)
        dist.all_reduce(t, op=_TORCH_OPS[op], group=self.group)
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

    def all_gather_t(self, t):
        """(world, *t.shape): every rank's tensor of one shape, rank order."""
        x = self.to(t).contiguous()
        outs = [torch.empty_like(x) for _ in range(self.world)]
        dist.all_gather(outs, x, group=self.group)
        return torch.stack(outs)

    def exchange(self, sends, recvs, send_counts, recv_counts, skip_self=True):
        """Field-wise all-to-all into `recvs` (rows grouped by source); with
        skip_self the self blocks are already in place (pd_pack2) and the send
        buffers hold the other ranks' blocks only."""
        me = self.rank
        sc = np.array(send_counts, np.int64)
        rc = np.array(recv_counts, np.int64)
        if skip_self:
            sc[me] = rc[me] = 0
        ro = np.concatenate([[0], np.cumsum(np.asarray(recv_counts, np.int64))])
        for snd, rcv in zip(sends, recvs):
            row = tuple(rcv.shape[1:])
            w = int(np.prod(row)) if row else 1
            got = torch.empty(int(rc.sum()) * w, dtype=rcv.dtype, device=self.device)
            dist.all_to_all_single(got, self.to(snd.reshape(-1)).contiguous(),
                                   output_split_sizes=[int(c) * w for c in rc],
                                   input_split_sizes=[int(c) * w for c in sc], group=self.group)
            got = got.reshape((-1,) + row)
            k = 0
            for r in range(self.world):
                c = int(rc[r])
                if c:
                    rcv[int(ro[r]):int(ro[r]) + c] = got[k:k + c].to(rcv.device)
                k += c

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

    _OPS = {"sum": _native.PD_R_SUM, "min": _native.PD_R_MIN, "max": _native.PD_R_MAX}

    def _op(self, op):
        if op not in self._OPS:
            raise ValueError(f"unknown reduction {op!r}")
        return self._OPS[op]

    def all_reduce(self, arr, op):
        t = torch.as_tensor(np.ascontiguousarray(arr)).to(self.device)
        self.comm.all_reduce(t, self._op(op))
        return t.cpu().numpy()

    def all_reduce_t(self, t, op):
        r = self.to(t).contiguous().clone()
        self.comm.all_reduce(r, self._op(op))
        return r

    def all_gather_t(self, t):
        x = self.to(t).contiguous()
        return self.comm.all_gather_v(x.reshape((1,) + tuple(x.shape)), [1] * self.world)

    def exchange(self, sends, recvs, send_counts, recv_counts, skip_self=True):
        self.comm.exchange([self.to(t) for t in sends], recvs, send_counts, recv_counts,
                           skip_self=skip_self)

    def abort(self):
        self.comm.abort()

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

    :local_labels, local_core: labels / core flags of this rank's INPUT
        points in input order (returned by the owners)
    :gid_base: global id of this rank's first input point
    :n_total: points over all ranks
    :n_clusters: number of clusters over all points
    :splits: the KD trace (identical on every rank)
    :bounding_boxes: label -> BoundingBox of each KD partition
    :boxes: (P, 2, d) expanded boxes
    :gid, labels, core: the records this rank owns (the points of its KD
        partitions): global ids, labels, core flags — computed on first use
        (diagnostics; the train itself never needs them)
    """

    def __init__(self, **kw):
        self._owned = kw.pop("owned", None)
        self._cache = None
        if "gid" in kw:   # given directly (the dense path holds every label)
            self._cache = (kw.pop("gid"), kw.pop("labels"), kw.pop("core"))
        self.__dict__.update(kw)

    def _owned_view(self):
        if self._cache is None:
            if self._owned is None:
                raise AttributeError("owned records were not kept "
                                     "(train_sharded(..., keep_owned=True))")
            ops, keys, core, owner, gid, roots, n = self._owned
            own = owner >= 0
            g = gid if gid is not None else \
                torch.arange(n, dtype=torch.int32, device=owner.device)
            labels = ops.rank_labels(keys, roots) if n else ops.empty(0, torch.int32)
            self._cache = (g[own], labels[own], core[own])
        return self._cache

    @property
    def gid(self):
        return self._owned_view()[0]

    @property
    def labels(self):
        return self._owned_view()[1]

    @property
    def core(self):
        return self._owned_view()[2]


def _kd_host(X, kdlab, levels, ops, comm, split_method, dense, lap):
    """KD partition with the level decisions on the host (rotation; d > 4):
    per level one all-gather of the moment partials and one all-reduce of the
    counts through host memory.  -> (data_box, boxes, splits)."""
    n, d = X.shape
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
    if ext[2 * d]:
        raise ValueError("Input contains NaN or infinity.")
    data_box = np.concatenate([-ext[:d], ext[d:2 * d]])
    boxes = {0: BoundingBox(k=d).union(BoundingBox(data_box[:d], data_box[d:]))}
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
    if pending is not None and n and not dense:
        ops.split(X, kdlab, *pending)
    return data_box, boxes, splits


def _kd_device(X, kdlab, levels, ops, comm, dev):
    """KD partition (min_var, exact sums) with the level decisions on the
    device (pd_kdx_*): per level the moment partials are all-gathered and the
    counts all-reduced as device tensors — no host round trip until the end
    (R:dbscan/partition.py:139-183; the splits equal one device's bit for bit).
    The slice sizes ride level 0's gather as one more fp64 column (exact below
    2^53) and are read back with the KD trace: no collective or host sync of
    their own.  -> (data_box, boxes, splits, sizes); kdlab ends as the
    partition labels."""
    n, d = X.shape
    W = comm.world
    ops.kdx_begin(d, levels)
    sizes_dev = None
    for lv, level in enumerate(levels):
        S = len(level)
        part = ops.kdx_moments(X, kdlab, lv, S)
        if lv == 0:
            L = part.shape[0]
            ext = torch.empty(L + 1, dtype=part.dtype, device=part.device)
            ext[:L] = part
            ext[L] = float(n)
            g = comm.all_gather_t(ext).to(dev)
            sizes_dev = g[:, L].clone()
            ops.kdx_axes(g[:, :L].contiguous(), W, lv)
        else:
            ops.kdx_axes(comm.all_gather_t(part).to(dev), W, lv)
        cnt = ops.kdx_counts(X, kdlab, lv, S)
        ops.kdx_boundary(comm.all_reduce_t(cnt, "sum").to(dev), lv)
    try:
        trace, lo, hi, bad = ops.kdx_end(X, kdlab, sum(len(lv) for lv in levels), True)
    except Exception:
        # every slice empty: the level decisions ran over zero moments; name
        # that (all ranks hold the same sizes, so all raise the same) rather
        # than whatever the empty KD failed on
        if int(sizes_dev.sum().item()) == 0:
            raise ValueError("no points on any rank") from None
        raise
    # the KD trace read above synchronised the stream: this copy waits on nothing
    sizes = sizes_dev.cpu().numpy().astype(np.int64)
    if int(sizes.sum()) == 0:
        raise ValueError("no points on any rank")
    if bad:
        raise ValueError("Input contains NaN or infinity.")
    data_box = np.concatenate([lo, hi])
    boxes = {0: BoundingBox(k=d).union(BoundingBox(lo, hi))}
    splits = []
    k = 0
    for level in levels:
        t = trace[k:k + len(level)]
        k += len(level)
        apply_level(boxes, splits, level, t[:, 0].astype(np.int64).tolist(), t[:, 1], t[:, 2],
                    t[:, 3:11].astype(np.int64), t[:, 11].astype(np.int64).tolist(), t[:, 12])
    return data_box, boxes, splits, sizes


_KD_TAB = 256   # kd.hip kTabLds: labels / splits per level of the device KD tables


def device_kd_ok(levels, split_method, dense):
    """The device-decided KD (pd_kdx_*) applies: min_var, d <= 4, and a
    schedule whose levels fit its LDS tables (every level <= 256 splits,
    every split label < 256, i.e. max_partitions <= 512).  Decided from the
    schedule alone, so every rank decides the same (inputs are made 16-byte
    aligned before the KD)."""
    if split_method != 'min_var' or dense or not levels:
        return False
    return all(len(lv) <= _KD_TAB and all(c < _KD_TAB for c, _ in lv) for lv in levels)


class _PhaseClock(object):
    """Per-phase times of the sharded train (``stats['<phase>_ms']``) without
    host syncs of its own: on a GPU, events recorded on the current stream at
    each phase boundary and read once, when the train has already synchronised
    at its end; on the host (gloo / CPU stand-ins), wall time."""

    def __init__(self, device, stats):
        self.stats = stats
        self.cuda = torch.device(device).type == "cuda"
        self.marks = []
        self.t0 = self._mark()

    def _mark(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def __call__(self, name):
        self.marks.append((name, self._mark()))

    def finish(self):
        prev = self.t0
        if self.cuda and self.marks:
            self.marks[-1][1].synchronize()
        total = 0.0
        for name, m in self.marks:
            ms = prev.elapsed_time(m) if self.cuda else 1e3 * (m - prev)
            self.stats[name + "_ms"] = round(ms, 3)
            total += ms
            prev = m
        self.stats["total_ms"] = round(total, 3)
        if "phase_b_roots_ms" in self.stats:
            self.stats["phase_b_ms"] = round(self.stats["phase_b_border_ms"] +
                                             self.stats["phase_b_roots_ms"], 3)
        self.marks = []


def _exclusive(c):
    c = np.asarray(c, np.int64)
    return np.concatenate([[0], np.cumsum(c)]).astype(np.int64)


def train_sharded(X, eps, min_samples, metric=_native.PD_EUCLIDEAN, max_partitions=None,
                  group=None, ops=None, split_method='min_var', comm=None, return_local=True,
                  keep_owned=False, placement=None):
    """Sharded DBSCAN train over the ranks of ``group`` (default: world).

    X: this rank's (n_i, d) slice (float32/float64, on this rank's GPU for
    NativeOps); the global id of row j is sum(n_0 .. n_{i-1}) + j.
    ``max_partitions`` defaults to the world size (one KD partition per GPU).
    ``split_method``: 'min_var' (default) or 'rotation' (KDPartitioner's).
    ``comm``: a collective layer (make_comm(group, device) by default: RCCL
    through libpardis for an "nccl" group, torch.distributed otherwise).
    ``return_local``: return the labels of this rank's input points (the
    results exchange); False skips it (``local_labels`` is None) and keeps
    the owned records instead.  ``keep_owned``: keep the records this rank
    owns (``gid`` / ``labels`` / ``core`` of the result, ~13 B of HBM per
    received record while the result lives); off by default.
    ``placement``: KD leaves -> ranks when max_partitions > world size.
    None (default): spatially ordered runs balanced by the leaves' point
    counts, or LPT when that balances clearly better; 'ordered' / 'lpt' /
    'blocks' force one (partition_ranks).  Labels do not depend on it.
    """
    if placement not in (None, "ordered", "lpt", "blocks"):
        raise ValueError("placement must be None, 'ordered', 'lpt' or 'blocks'")
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
    dev = getattr(ops, "device", X.device)
    keep_owned = keep_owned or not return_local
    if n and X.is_cuda and X.data_ptr() % 16:
        # a view at an odd offset (e.g. X_full[a:b] of fp32 3-D): the fused
        # KD and record kernels read 16-B vectors; one copy realigns it
        X = X.clone()
    stats = {}
    lap = _PhaseClock(dev, stats)

    # ---- KD partition (R:dbscan/partition.py:135-183); the global ids (rank
    # offset + row) from the slice sizes gathered with it
    kdlab = ops.zeros(n, torch.int32)
    levels = _split_schedule(P)
    dense = d > 4
    if device_kd_ok(levels, split_method, dense):
        data_box, boxes, splits, sizes = _kd_device(X, kdlab, levels, ops, comm, dev)
    else:
        sizes = comm.all_gather_np(np.array([n], np.int64))[:, 0]
        data_box, boxes, splits = _kd_host(X, kdlab, levels, ops, comm, split_method, dense, lap)
    gid_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    gid_base = int(gid_off[rank])
    n_total = int(gid_off[-1])
    if n_total >= 0xFFFFFFFF:
        raise ValueError("the sharded train addresses points with 32-bit global ids")
    if n_total == 0:
        raise ValueError("no points on any rank")
    ebox = np.stack([boxes[L].expand(2 * eps).as_array() for L in sorted(boxes)])
    lap("kd")
    if dense:
        return _train_dense(X, eps, min_samples, metric, comm, ops, gid_off, data_box,
                            dict(splits=splits, bounding_boxes=boxes, boxes=ebox), stats, lap)

    # ---- route + exchange (R:dbscan/dbscan.py:114-118,136-151): one ordered
    # pass packs every destination (the self block straight into the receive
    # buffers), one grouped exchange moves all fields
    # KD leaves -> ranks (partition_ranks): with more leaves than ranks,
    # balanced by the leaves' point counts — spatially ordered runs, or LPT
    # when that balances clearly better; else contiguous label blocks
    weights, order = None, None
    if placement != "blocks" and P > W:
        weights = leaf_sizes(splits, n_total, P)
        order = kd_leaf_order(splits)
    chosen = {}
    part_rank, local_index = partition_ranks(P, W, weights, order, placement, chosen)
    stats["placement"] = chosen["placement"]
    if W == 1:
        # every neighbourhood is here: the slice is the record set as it is
        Xr, gid, owner, xr = X, None, kdlab, None
        nr = n
        recv_counts = np.array([n], np.int64)
        own_counts = np.array([[n]], np.int64)   # [src, dest] owned records
        stats["sent"] = 0
    else:
        cnt = ops.route2(X, ebox, part_rank, kdlab, W)            # (W, 2): routed, owned
        allc = comm.all_gather_np(cnt.astype(np.int64))           # (src, dest, 2)
        send_counts = cnt[:, 0].astype(np.int64)
        recv_counts = allc[:, rank, 0].astype(np.int64)
        own_counts = allc[:, :, 1].astype(np.int64)
        nr = int(recv_counts.sum())
        ro = _exclusive(recv_counts)
        Xr = ops.empty(nr, X.dtype, d)
        gid = ops.empty(nr, torch.int32)
        owner = ops.empty(nr, torch.int32)
        xr = ops.empty(nr, torch.uint8)
        ns = int(send_counts.sum() - send_counts[rank])
        s_coords, s_gid = ops.empty(ns, X.dtype, d), ops.empty(ns, torch.int32)
        s_owner, s_xr = ops.empty(ns, torch.int32), ops.empty(ns, torch.uint8)
        outs, so = [], 0
        for r in range(W):
            c = int(send_counts[r])
            if r == rank:
                a = int(ro[rank])
                outs.append((Xr[a:a + c], gid[a:a + c], owner[a:a + c], xr[a:a + c]))
            else:
                outs.append((s_coords[so:so + c], s_gid[so:so + c], s_owner[so:so + c],
                             s_xr[so:so + c]))
                so += c
        if n:
            ops.pack2(X, kdlab, part_rank, local_index, gid_base, outs)
        comm.exchange([s_coords, s_gid, s_owner, s_xr], [Xr, gid, owner, xr], send_counts,
                      recv_counts, skip_self=True)
        del s_coords, s_gid, s_owner, s_xr, outs
        stats["sent"] = ns
    stats["received"] = nr
    lap("exchange")

    # ---- phase A on this rank's neighbourhoods
    mine = [L for L in range(P) if part_rank[L] == rank]
    if mine and nr:
        n_exp = ops.train_begin(Xr.contiguous(), eps, min_samples, metric, ebox[mine], owner,
                                gid, xr, data_box)
        e_gid, e_key = ops.exports(n_exp)
    else:
        n_exp = 0
        e_gid = ops.empty(0, torch.int32)
        e_key = ops.empty(0, torch.int32)
    stats["exports"] = int(e_gid.shape[0])
    lap("phase_a")

    # ---- global key merge (R:dbscan/dbscan.py:153-165): one gather of the
    # (id, key) pairs, then the same O(exports) union on every rank
    keymap = None
    if W > 1:
        ex = comm.all_gather_var(torch.stack([e_gid, e_key], 1)).to(dev)
        keymap = ops.merge(ex[:, 0].contiguous(), ex[:, 1].contiguous()) if ex.shape[0] else None
        stats["exports_total"] = int(ex.shape[0])
    else:
        stats["exports_total"] = 0
    lap("merge")

    # ---- phase B: border attach with the global keys, the cluster roots of
    # every rank (sklearn's numbering: a key's rank among them)
    if mine and nr:
        keys, core = ops.train_end(nr, keymap, n_total)
    else:
        keys, core = ops.empty(0, torch.int32), ops.empty(0, torch.uint8)
    lap("phase_b_border")
    roots = ops.select_roots(keys, gid) if nr else ops.empty(0, torch.int32)
    all_roots = (comm.all_gather_var(roots) if W > 1 else roots).to(dev).contiguous()
    ops.sort(all_roots)
    # one root per cluster over all ranks: only owned records carry keys
    # (shard.hip IsRoot); a duplicate would double-count a cluster
    if W > 1 and all_roots.shape[0] > 1 and bool((all_roots[1:] == all_roots[:-1]).any()):
        raise RuntimeError("sharded train: a cluster root was selected on two ranks")
    lap("phase_b_roots")

    owned = (ops, keys, core, owner, gid, all_roots, nr) if keep_owned else None
    common = dict(gid_base=gid_base, n_total=n_total, n_clusters=int(all_roots.shape[0]),
                  splits=splits, bounding_boxes=boxes, boxes=ebox, stats=stats, owned=owned)
    if not return_local:
        lap("results")
        lap.finish()
        return ShardedResult(local_labels=None, local_core=None, **common)

    # ---- labels back to the ranks that hold the points, in input order (the
    # reference's result RDD, R:dbscan/dbscan.py:162-164): the self block
    # directly, the rest as (gid, label | core) pairs in one exchange
    src_off = _exclusive(recv_counts)
    back_send = own_counts[:, rank].copy()    # owned records of block r go back to r
    back_recv = own_counts[rank, :].copy()    # my points each rank owns
    back_send[rank] = back_recv[rank] = 0
    loc_labels, loc_core, pairs = ops.results(keys, core, owner, gid, all_roots, n_total,
                                              gid_base, n, W, rank, src_off,
                                              int(back_send.sum()))
    pairs_in = ops.empty(int(back_recv.sum()), torch.int32, 2)
    if W > 1:
        comm.exchange([pairs], [pairs_in], back_send, back_recv, skip_self=False)
    ops.results_scatter(pairs_in, gid_base, loc_labels, loc_core)
    lap("results")
    lap.finish()
    return ShardedResult(local_labels=loc_labels, local_core=loc_core, **common)


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
    lap.finish()
    lo = int(gid_off[rank])
    loc_labels, loc_core = labels[lo:lo + n], core[lo:lo + n]
    gid = torch.arange(lo, lo + n, dtype=torch.int32, device=dev)
    return ShardedResult(gid=gid, labels=loc_labels, core=loc_core, local_labels=loc_labels,
                         local_core=loc_core, gid_base=lo, n_total=n_total, n_clusters=ncl,
                         stats=stats, **kd)


def train_threads(slices, eps, min_samples, comms, ops, metric=_native.PD_EUCLIDEAN,
                  max_partitions=None, split_method='min_var', abort_timeout=60.0,
                  keep_owned=False, placement=None):
    """One process driving several devices: rank r = thread r runs
    ``train_sharded`` on slices[r] with comms[r] (e.g. RcclComm over
    pd_comm_init_all) and ops[r].  Returns the per-rank results in rank order;
    the first rank error is raised.  A rank that fails alone aborts every
    communicator (pd_comm_abort) so the others return instead of waiting for
    it; the aborted communicators are dropped from the caches."""
    import threading

    W = len(slices)
    out, errs = [None] * W, [None] * W
    order = []   # ranks in the order their errors happened: the first is the cause

    def body(r):
        try:
            dev = getattr(ops[r], "device", None)
            if dev is not None and torch.device(dev).type == "cuda":
                torch.cuda.set_device(torch.device(dev))
            out[r] = train_sharded(slices[r], eps, min_samples, metric=metric,
                                   max_partitions=max_partitions, ops=ops[r], comm=comms[r],
                                   split_method=split_method, keep_owned=keep_owned,
                                   placement=placement)
        except BaseException as e:   # noqa: B902 - re-raised below
            errs[r] = e
            order.append(r)

    ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(W)]
    for t in ts:
        t.start()
    # a rank that fails alone would leave the others blocked on it for ever:
    # on the first error abort every communicator (pd_comm_abort releases the
    # ranks waiting in RCCL), then collect the threads
    aborted = False
    while any(t.is_alive() for t in ts):
        for t in ts:
            t.join(timeout=0.05)
        if not aborted and any(e is not None for e in errs):
            aborted = True
            for c in comms:
                if hasattr(c, "abort"):
                    c.abort()
            _forget_comms(comms)
            for t in ts:
                t.join(timeout=abort_timeout)
            break
    if order:
        raise errs[order[0]]
    if any(t.is_alive() for t in ts):
        raise RuntimeError("train_threads: ranks still running after the communicators were "
                           "aborted")
    return out


_device_comms = {}


def _forget_comms(comms):
    """Drop aborted communicators from the caches (a new call re-creates them)."""
    ids = {id(c) for c in comms}
    for cache in (_device_comms, _rccl_cache):
        for k in [k for k, v in cache.items()
                  if (id(v) in ids) or (isinstance(v, list) and any(id(x) in ids for x in v))]:
            del cache[k]


def device_comms(devices):
    """RCCL communicators of one process over `devices` (cached)."""
    key = tuple(int(d) for d in devices)
    if key not in _device_comms:
        _device_comms[key] = [RcclComm(c) for c in _native.Comm.init_all(list(key))]
    return _device_comms[key]
