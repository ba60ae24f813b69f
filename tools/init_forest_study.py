"""Offline study (CPU): quality of the union-find forest that the link stage
starts from, on a density-preserving C2 slice, for candidate parent rules.

Record order as engine.hip (eps-cell key, axis 0 in eps/2 sub-cells).  Rules:
  A  count pass's smallest seen neighbour (centre batch first, early exit at
     min_samples after a group of four), kept if it is core and smaller
  B  smallest core neighbour overall (a sweep of the rows in ascending key
     order stopping at the first core hit)
Prints, per rule: trees (core roots), tree depth (mean / p99 / max), and for B
the candidates a sweep would test before its first core hit.

  python tools/init_forest_study.py [n]
"""
import sys

import numpy as np

sys.path.insert(0, ".")
import oracle  # noqa: E402
from pypardis_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
X, cfg = synth.make_config("C2", n=n)
eps, ms = cfg["eps"], cfg["min_samples"]
X64 = X.astype(np.float64)
lo = X64.min(0)
cw = eps * (1 + 2.0 ** -20)
c = np.floor((X64 - lo) / np.array([cw / 2, cw, cw])).astype(np.int64)
nc = c.max(0) + 1
key = c[:, 0] + nc[0] * (c[:, 1] + nc[1] * c[:, 2])
order = np.argsort(key, kind="stable")
rec = np.empty(n, np.int64)
rec[order] = np.arange(n)
off, nbr = oracle.neighbors(X, eps)
cnt = np.diff(off)
core_r = (cnt >= ms)[order]
src = np.repeat(np.arange(n), cnt)
i_r, j_r = rec[src], rec[nbr]                       # edges in record space (incl. self)
dy = c[nbr, 1] - c[src, 1]
dz = c[nbr, 2] - c[src, 2]
need = np.minimum(cnt[order], ms)                    # hits needed (or all)


def smallest_seen(bt_order, row_order):
    # count pass scan rank: batches by oz, rows in a batch by oy, then index;
    # candidates are hits only here (non-neighbours are skipped by the
    # predicate and do not move the count); the scan stops after the group of
    # four in which the count reaches ms
    bt_rank = np.select([dz == v for v in bt_order], [0, 1, 2])
    row_rank = np.select([dy == v for v in row_order], [0, 1, 2])
    o = np.lexsort((j_r, row_rank, bt_rank, i_r))
    i_s, j_s = i_r[o], j_r[o]
    start = np.searchsorted(i_s, np.arange(n))
    pos = np.arange(len(i_s)) - start[i_s]
    seen = pos < ((need[i_s] + 3) // 4) * 4
    mn = np.full(n, np.iinfo(np.int64).max)
    np.minimum.at(mn, i_s[seen], j_s[seen])
    return mn


def smallest_core_of_k_seen(k, bt_order=(0, 1, -1), row_order=(0, -1, 1)):
    # the count pass keeps the k smallest neighbours it saw; init takes the
    # smallest of them that is core
    bt_rank = np.select([dz == v for v in bt_order], [0, 1, 2])
    row_rank = np.select([dy == v for v in row_order], [0, 1, 2])
    o = np.lexsort((j_r, row_rank, bt_rank, i_r))
    i_s, j_s = i_r[o], j_r[o]
    start = np.searchsorted(i_s, np.arange(n))
    pos = np.arange(len(i_s)) - start[i_s]
    seen = pos < ((need[i_s] + 3) // 4) * 4
    i2, j2 = i_s[seen], j_s[seen]
    o2 = np.lexsort((j2, i2))
    i2, j2 = i2[o2], j2[o2]
    st2 = np.searchsorted(i2, np.arange(n))
    rank = np.arange(len(i2)) - st2[i2]
    keep = (rank < k) & core_r[j2]
    mn = np.full(n, np.iinfo(np.int64).max)
    np.minimum.at(mn, i2[keep], j2[keep])
    return mn


mnA = smallest_seen((0, 1, -1), (0, -1, 1))     # engine.hip today
mnA2 = smallest_seen((0, 1, -1), (-1, 0, 1))    # centre batch first, rows ascending
mnA3 = smallest_seen((-1, 0, 1), (-1, 0, 1))    # ascending key order


def forest(parent):
    par = parent.copy()
    depth = np.zeros(n, np.int64)
    cur = par.copy()
    act = core_r & (cur != np.arange(n))
    while act.any():
        depth[act] += 1
        cur[act] = par[cur[act]]
        act = act & (cur != par[cur])
    roots = core_r & (par == np.arange(n))
    d = depth[core_r]
    return int(roots.sum()), d.mean(), np.percentile(d, 99), d.max()


ar = np.arange(n)
def par_of(mn):
    return np.where(core_r & core_r[np.minimum(mn, n - 1)] & (mn < ar), mn, ar)


pA, pA2, pA3 = par_of(mnA), par_of(mnA2), par_of(mnA3)
pK2, pK4 = par_of(smallest_core_of_k_seen(2)), par_of(smallest_core_of_k_seen(4))
# B: smallest core neighbour
cc = core_r[i_r] & core_r[j_r]
mnB = np.full(n, np.iinfo(np.int64).max)
np.minimum.at(mnB, i_r[cc], j_r[cc])
pB = np.where(core_r & (mnB < ar), mnB, ar)
print(f"n={n} records={n} core={core_r.sum()} clusters~{oracle.dbscan(X, eps, ms)[3]}")
for name, p in (("A count smallest seen", pA), ("A2 rows ascending", pA2),
                ("A3 key order", pA3), ("K2 core of 2 seen", pK2), ("K4 core of 4 seen", pK4),
                ("B smallest core nbr", pB)):
    t, dm, d99, dmax = forest(p)
    print(f"{name:24s} trees={t:9d}  depth mean={dm:.2f} p99={d99:.0f} max={dmax}")
