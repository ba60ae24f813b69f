"""Offline study (CPU, oracle neighbour lists) of the link stage on a C2-density
slice: how converged is the union-find forest when the full link pass starts,
and how many candidates / cells a parent-based skip could avoid?

Emulates engine.hip's record order (neighbourhood + eps-cell key, axis 0 cut
in eps/2 sub-cells), the count pass's smallest-neighbour choice (centre row
first, early exit at min_samples), init_kernel + 4 pointer jumps, and an
optional centre-row pre-link.  Prints tree counts and skip rates.
"""
import sys

import numpy as np

sys.path.insert(0, ".")
import oracle  # noqa: E402
from pypardis_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000
X, cfg = synth.make_config("C2", n=n)
eps, ms = cfg["eps"], cfg["min_samples"]
X64 = X.astype(np.float64)
lo = X64.min(0)
cw = eps * (1 + 2.0 ** -20)
c = np.floor((X64 - lo) / np.array([cw / 2, cw, cw])).astype(np.int64)
nc = c.max(0) + 1
key = c[:, 0] + nc[0] * (c[:, 1] + nc[1] * c[:, 2])
order = np.argsort(key, kind="stable")          # record -> point
rec_of = np.empty(n, np.int64)
rec_of[order] = np.arange(n)                     # point -> record
ckey = key[order]
cell_id = np.concatenate([[0], np.cumsum(ckey[1:] != ckey[:-1])])   # record -> cell

off, nbr = oracle.neighbors(X, eps)
cnt = np.diff(off)
core_pt = cnt >= ms
core = core_pt[order]                           # per record
print(f"n={n} core={core.mean():.3f} cells={cell_id[-1] + 1}")

# neighbour lists in record space
rows_r = [None] * n
row_of = (c[:, 1] + nc[1] * c[:, 2])            # y-z row of a point
for p in range(n):
    r = rec_of[p]
    nb = rec_of[nbr[off[p]:off[p + 1]]]
    rows_r[r] = (nb, row_of[nbr[off[p]:off[p + 1]]] - row_of[p])

# smallest neighbour seen by the count pass (centre row first, early exit)
mn = np.arange(n)
for r in range(n):
    nb, drow = rows_r[r]
    cen = np.sort(nb[drow == 0])
    rest = np.sort(nb[drow != 0])
    seq = np.concatenate([cen, rest])
    seen = seq[:max(ms, 0)] if len(seq) >= ms else seq
    mn[r] = seen.min() if len(seen) else r

par = np.where(core, np.arange(n), -1)
ok = core & (mn < np.arange(n)) & core[mn]
par[ok] = mn[ok]


def roots(par):
    p = par.copy()
    idx = np.nonzero(p >= 0)[0]
    while True:
        q = p[p[idx]]
        if np.array_equal(q, p[idx]):
            break
        p[idx] = q
    return p


def report(tag, par):
    rt = roots(par)
    cr = np.nonzero(core)[0]
    trees = len(np.unique(rt[cr]))
    same = tot = 0
    for r in cr:
        nb, _ = rows_r[r]
        nb = nb[(nb > r) & core[nb]]
        tot += len(nb)
        same += int((rt[nb] == rt[r]).sum())
    # cells whose core records share one root
    cc = cell_id[cr]
    rr = rt[cr]
    uni = 0
    cells = np.unique(cc)
    first = np.searchsorted(cc, cells)
    last = np.searchsorted(cc, cells, side="right")
    for a, b in zip(first, last):
        uni += int(np.all(rr[a:b] == rr[a]))
    print(f"{tag}: trees={trees} core-core edges j>r={tot} same-root={same / max(tot, 1):.3f} "
          f"uniform core cells={uni / len(cells):.3f}")
    return rt


report("init (mn) + full compression", par)
# centre-row pre-link: union every core record with its core centre-row neighbours
p2 = roots(par)


def find(x):
    while p2[x] != x:
        p2[x] = p2[p2[x]]
        x = p2[x]
    return x


for r in np.nonzero(core)[0]:
    nb, drow = rows_r[r]
    for j in nb[(drow == 0) & (nb > r)]:
        if core[j]:
            a, b = find(r), find(j)
            if a != b:
                p2[max(a, b)] = min(a, b)
report("+ centre-row pre-link", p2)

# k neighbours sampled by the count pass (its scan order: centre row first,
# early exit at min_samples), united with r when core — no extra sweep
for k in (1, 2, 4, 8):
    p3 = np.where(core, np.arange(n), -1)

    def find3(x):
        while p3[x] != x:
            p3[x] = p3[p3[x]]
            x = p3[x]
        return x

    for r in np.nonzero(core)[0]:
        nb, drow = rows_r[r]
        seq = np.concatenate([np.sort(nb[drow == 0]), np.sort(nb[drow != 0])])
        seq = seq[:ms]
        seq = seq[seq != r][:k]
        for j in seq:
            if core[j]:
                a, b = find3(r), find3(j)
                if a != b:
                    p3[max(a, b)] = min(a, b)
    report(f"{k} count-pass samples", p3)
