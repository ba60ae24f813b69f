"""CPU stand-in for ``pypardis_amd.distributed.NativeOps``: the same stage
interface computed by the oracle (numpy / oracle.sharded), so the sharded
orchestration and its collectives run under gloo on a machine without a GPU.
Test infrastructure only."""
from __future__ import annotations

import math

import numpy as np
import torch

import oracle
from oracle import sharded as osh


class OracleOps(object):
    device = torch.device("cpu")

    def __init__(self, metric="euclidean"):
        self.metric = metric
        self.state = None
        self.exp = None

    def empty(self, n, dtype, d=None):
        return torch.empty((n, d) if d is not None else (n,), dtype=dtype)

    def zeros(self, n, dtype):
        return torch.zeros(n, dtype=dtype)

    def bbox(self, X):
        a = X.numpy().astype(np.float64)
        bad = int((~np.isfinite(a)).sum())
        return a.min(0), a.max(0), bad

    def moments_dd(self, X, labels, sel):
        """Exact per-label sums split into (hi, lo); squares rounded in the
        input precision first (as numpy's ``v ** 2`` of the reference)."""
        x = X.numpy()
        lab = labels.numpy()
        d = x.shape[1]
        out = np.zeros((len(sel), 1 + 4 * d))
        for s, L in enumerate(sel):
            v = x[lab == L]
            out[s, 0] = len(v)
            sq = (v * v).astype(np.float64)
            v = v.astype(np.float64)
            for j in range(d):
                for base, col in ((1, v[:, j]), (1 + 2 * d, sq[:, j])):
                    hi = math.fsum(col)
                    lo = math.fsum(list(col) + [-hi])
                    out[s, base + 2 * j] = hi
                    out[s, base + 2 * j + 1] = lo
        return out

    def level_pass(self, X, labels, split, sel, labels_zero=False, bbox=False):
        """pd_kd_pass restated: the previous level's split, then moments_dd
        (and the bbox on the first level)."""
        if split is not None:
            self.split(X, labels, *split)
        dd = self.moments_dd(X, labels, sel)
        if bbox:
            return (dd,) + tuple(self.bbox(X))
        return dd

    def counts(self, X, labels, sel, axes, bounds):
        x = X.numpy().astype(np.float64)
        lab = labels.numpy()
        out = np.zeros((len(sel), 8), np.int64)
        for s, L in enumerate(sel):
            v = x[lab == L, axes[s]]
            out[s, :7] = [(v < b).sum() for b in bounds[s]]
            out[s, 7] = len(v)
        return out

    def radix_hist(self, X, labels, sel, axes, prefix, shift):
        """pd_kd_radix_hist restated: digit histograms of the fp64 order keys."""
        x = X.numpy().astype(np.float64)
        lab = labels.numpy()
        out = np.zeros((len(sel), 256), np.int64)
        for s, L in enumerate(sel):
            b = np.ascontiguousarray(x[lab == L, axes[s]]).view(np.uint64).copy()
            b[b == np.uint64(1 << 63)] = 0
            k = np.where((b >> np.uint64(63)) == 1, ~b, b | np.uint64(1 << 63))
            if shift + 8 < 64:
                k = k[(k >> np.uint64(shift + 8)) == np.uint64(prefix[s])]
            np.add.at(out[s], ((k >> np.uint64(shift)) & np.uint64(255)).astype(np.int64), 1)
        return out

    def split(self, X, labels, sel, axes, boundary, new):
        x = X.numpy().astype(np.float64)
        lab = labels.numpy()
        for s, L in enumerate(sel):
            m = (lab == L) & (x[:, axes[s]] >= boundary[s])
            lab[m] = new[s]

    def route(self, X, ebox, part_rank, world):
        x = X.numpy().astype(np.float64)
        mask = np.zeros(len(x), np.int64)
        for L in range(len(ebox)):
            m = np.all(ebox[L, 0] <= x, axis=1) & np.all(ebox[L, 1] >= x, axis=1)
            mask[m] |= np.int64(1) << int(part_rank[L])
        counts = np.array([((mask >> r) & 1).sum() for r in range(world)], np.int64)
        return torch.from_numpy(mask), counts

    def pack(self, X, mask, dest, kdlab, part_rank, local_index, gid_base, out):
        coords, gid, owner, xr = out
        mk = mask.numpy()
        idx = np.nonzero((mk >> dest) & 1)[0]
        lab = kdlab.numpy()[idx]
        coords.copy_(X[torch.from_numpy(idx)])
        gid.copy_(torch.from_numpy((gid_base + idx).astype(np.int32)))
        own = np.where(part_rank[lab] == dest, local_index[lab], -1).astype(np.int32)
        owner.copy_(torch.from_numpy(own))
        many = np.array([bin(int(v) & ((1 << 64) - 1)).count("1") > 1 for v in mk[idx]], bool)
        xr.copy_(torch.from_numpy(many.astype(np.uint8)))
        return len(idx)

    def train_begin(self, X, eps, min_samples, metric, ebox, owner, gid, xr, data_box):
        m = "euclidean" if metric == 0 else "cityblock"
        self.state, self.exp = osh.phase_a(X.numpy(), eps, min_samples, ebox, owner.numpy(),
                                           gid.numpy(), xr.numpy(), m)
        return len(self.exp[0])

    def exports(self, m):
        g, k = self.exp
        return (torch.from_numpy(g.astype(np.int32)), torch.from_numpy(k.astype(np.int32)))

    def merge(self, gid, key):
        ids, keys = osh.merge(gid.numpy().view(np.uint32), key.numpy().view(np.uint32))
        return (torch.from_numpy(ids.astype(np.uint32).view(np.int32)),
                torch.from_numpy(keys.astype(np.uint32).view(np.int32)))

    def train_end(self, n, keymap):
        km = None if keymap is None else tuple(t.numpy().view(np.uint32) for t in keymap)
        keys, core = osh.phase_b(self.state, km)
        return torch.from_numpy(keys.astype(np.int32)), torch.from_numpy(core)

    def select_roots(self, keys, gid):
        k = keys.numpy()
        return torch.from_numpy(gid.numpy()[(k >= 0) & (k == gid.numpy())].copy())

    def sort(self, data):
        data.copy_(torch.sort(data).values)
        return data

    def rank_labels(self, keys, roots):
        k = keys.numpy().view(np.uint32).astype(np.int64)
        r = roots.numpy().view(np.uint32).astype(np.int64)
        m = k != 0xFFFFFFFF
        pos = np.searchsorted(r, k[m])
        if m.any() and (len(r) == 0 or (r[np.minimum(pos, len(r) - 1)] != k[m]).any()):
            raise RuntimeError("rank_labels: a cluster key has no root")   # pd_rank_labels
        lab = np.full(len(k), -1, np.int32)
        lab[m] = pos
        return torch.from_numpy(lab)

    def owned_results(self, owner, gid, labels, core, gid_offsets):
        """pd_owned_results restated: (gid, (label + 1) | core << 31) of the
        owned records, ascending gid, and the count per holding rank."""
        own = owner.numpy() >= 0
        g = gid.numpy().view(np.uint32)[own].astype(np.int64)
        assert (np.diff(g) > 0).all()
        v = (labels.numpy()[own].astype(np.int64) + 1) | (core.numpy()[own].astype(np.int64) << 31)
        pairs = np.stack([g, v], 1).astype(np.uint32).view(np.int32)
        counts = np.diff(np.searchsorted(g, np.asarray(gid_offsets, np.int64)))
        return torch.from_numpy(np.ascontiguousarray(pairs)), counts.astype(np.int64)

    # -- dense (d > 4) stages: pd_dense_* restated.  This rank's rows are the
    # 2048-row chunks c with c % world == rank (the stand-in deals input rows;
    # the device deals its pruned row order — any split sums to the same).
    def dense_count(self, X, eps, min_samples, metric, data_box, rank, world):
        m = "euclidean" if metric == 0 else "cityblock"
        off, nbr = oracle.neighbors(X.numpy(), eps, m)
        n = len(off) - 1
        mine = (np.arange(n) // 2048) % world == rank
        self.dn = dict(off=off, nbr=nbr, ms=min_samples, n=n, rank=rank, world=world)
        return torch.from_numpy((np.diff(off) * mine).astype(np.int32))

    def dense_link(self, counts):
        dn = self.dn
        core = counts.numpy() >= dn["ms"]
        clist = np.nonzero(core)[0]
        row = np.full(dn["n"], -1, np.int64)
        row[clist] = np.arange(len(clist))
        cmine = self._core_share(len(clist))
        uf = oracle._UF(len(clist))
        off, nbr = dn["off"], dn["nbr"]
        for a in np.nonzero(cmine)[0]:
            p = clist[a]
            for q in nbr[off[p]:off[p + 1]]:
                b = row[q]
                if b > a:
                    uf.union(a, b)
        dn.update(clist=clist, row=row, counts=counts.numpy().copy())
        return torch.from_numpy(np.array([uf.find(a) for a in range(len(clist))], np.int32))

    def _core_share(self, m):
        r, w = self.dn["rank"], self.dn["world"]
        return (np.arange(m) // 2048) % w == r

    def dense_border(self, forests, n_forests, n):
        dn = self.dn
        clist, row = dn["clist"], dn["row"]
        m = len(clist)
        uf = oracle._UF(m)
        f = forests.numpy().reshape(n_forests, m) if m else np.zeros((n_forests, 0), np.int32)
        for r in range(n_forests):
            for a in range(m):
                uf.union(a, int(f[r, a]))
        keyc = np.array([clist[uf.find(a)] for a in range(m)], np.int64)
        cnt = dn["counts"]
        blist = np.nonzero((cnt >= 2) & (cnt < dn["ms"]))[0]
        bmine = (np.arange(len(blist)) // 2048) % dn["world"] == dn["rank"]
        best = np.full(len(blist), 0x7FFFFFFF, np.int64)
        off, nbr = dn["off"], dn["nbr"]
        for k in np.nonzero(bmine)[0]:
            p = blist[k]
            ks = [keyc[row[q]] for q in nbr[off[p]:off[p + 1]] if row[q] >= 0]
            if ks:
                best[k] = min(ks)
        dn.update(keyc=keyc, blist=blist)
        return torch.from_numpy(best.astype(np.int32))

    def dense_finish(self, best, n):
        dn = self.dn
        key = np.full(n, 0xFFFFFFFF, np.int64)
        key[dn["clist"]] = dn["keyc"]
        b = best.numpy().astype(np.int64)
        key[dn["blist"]] = np.where(b == 0x7FFFFFFF, 0xFFFFFFFF, b)
        roots = np.unique(key[key != 0xFFFFFFFF])
        labels = np.full(n, -1, np.int32)
        m = key != 0xFFFFFFFF
        labels[m] = np.searchsorted(roots, key[m])
        core = (dn["counts"] >= dn["ms"]).astype(np.uint8)
        return torch.from_numpy(labels), torch.from_numpy(core), len(roots)

    def scatter_results(self, pairs, gid_base, n):
        p = pairs.numpy().view(np.uint32).astype(np.int64).reshape(-1, 2)
        idx = p[:, 0] - gid_base
        assert len(p) == n and (np.sort(idx) == np.arange(n)).all()
        labels = np.empty(n, np.int32)
        core = np.empty(n, np.uint8)
        labels[idx] = (p[:, 1] & 0x7FFFFFFF) - 1
        core[idx] = p[:, 1] >> 31
        return torch.from_numpy(labels), torch.from_numpy(core)
