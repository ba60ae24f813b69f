"""Windowed oracle spot checks for full-size GPU runs (test infrastructure).

A full-size result (100M C2 points, 1B C4 points) is far beyond what the CPU
oracle can recompute, but DBSCAN is local: every fact about a point depends
only on the points within 2·eps of it.  For a window W (Chebyshev radius h
around a centre c) the test pulls every point within h + 2·eps out of the
device tensor with plain torch masking and runs the oracle on that extract:

* inner points (|x - c|_inf <= h): all neighbours lie inside the extract, so
  their neighbour counts are exact;
* mid points (<= h + eps): all neighbours of theirs too, so their core flags
  are exact (a neighbour count of an outer point can only be too low: the
  oracle never marks a point core that is not);
* core-core edges of inner points: both ends must carry the same GPU label;
* inner border points: the smallest GPU label among their core neighbours
  (sklearn's first-discovered cluster, SK:cluster/_dbscan_inner.pyx:19-41,
  because labels are numbered by smallest core index); noise: -1;
* local clusters of the extract (oracle.dbscan): every core point of one
  local cluster is truly core and truly connected, so they must share one
  GPU label; a local cluster whose core points all lie inside W is a whole
  true cluster, so no point anywhere else may carry its GPU label (a
  bincount over all n labels checks that).

Per-partition semantics: R:dbscan/dbscan.py:12-34 (sklearn inside each
2·eps-expanded KD box); the merge intent: R:dbscan/dbscan.py:153-165.
"""
from __future__ import annotations

import numpy as np
import torch

import oracle


def dense_centres(X, eps, k, sample=1_000_000, seed=0):
    """Centres of the k most populated eps-cells of a random sample."""
    g = torch.Generator(device=X.device)
    g.manual_seed(seed)
    n = X.shape[0]
    idx = torch.randint(0, n, (min(sample, n),), generator=g, device=X.device)
    S = X[idx].double()
    q = torch.floor(S / eps).long()
    q = q - q.min(0).values
    span = q.max(0).values + 1
    lin = torch.zeros(len(q), dtype=torch.long, device=X.device)
    for j in range(q.shape[1] - 1, -1, -1):
        lin = lin * span[j] + q[:, j]
    u, inv, cnt = torch.unique(lin, return_inverse=True, return_counts=True)
    top = torch.topk(cnt, min(k, len(cnt))).indices
    out = []
    for t in top.tolist():
        rows = torch.nonzero(inv == t).flatten()
        out.append(S[rows[0]].cpu().numpy())
    return out


def random_centres(X, k, seed=1):
    """k centres at random points (density-weighted) and k uniform in the bbox."""
    rng = np.random.default_rng(seed)
    n = X.shape[0]
    pts = X[torch.from_numpy(rng.integers(0, n, k)).to(X.device)].double().cpu().numpy()
    lo = X.min(0).values.double().cpu().numpy()
    hi = X.max(0).values.double().cpu().numpy()
    uni = lo + (hi - lo) * rng.uniform(size=(k, X.shape[1]))
    return list(pts), list(uni)


def _extract_mask(X, c, r):
    m = None
    for j in range(X.shape[1]):
        mj = (X[:, j].double() - float(c[j])).abs() <= r
        m = mj if m is None else (m & mj)
    return m


def extract(X, c, h, eps, max_pts):
    """Smallest h' in {h, h/2, ...} >= eps/8 whose extract (radius h' + 2 eps,
    plus a small slack) holds <= max_pts points; returns (h', ids) or None."""
    while True:
        m = _extract_mask(X, c, h + 2 * eps * (1 + 1e-6) + 1e-12)
        cnt = int(m.sum().item())
        if cnt <= max_pts:
            return h, torch.nonzero(m).flatten()
        if h <= eps / 8:
            return None
        h = h / 2


def check_window(X, labels, core, counts, label_hist, eps, ms, c, h, ids, full_counts):
    """All checks of the module docstring for one window.  labels/core/counts
    are device tensors over all n points (counts may be None), label_hist =
    bincount(labels + 1) over all n.  Returns a dict of tallies."""
    ids_np = ids.cpu().numpy()
    Xe = X[ids].double().cpu().numpy()
    lab = labels[ids].cpu().numpy().astype(np.int64)
    cor = core[ids].cpu().numpy().astype(bool)
    dist = np.abs(Xe - np.asarray(c, np.float64)[None, :]).max(axis=1)
    inner = dist <= h
    mid = dist <= h + eps
    off, nbr = oracle.neighbors(Xe, eps)
    cnt = np.diff(off)
    core_x = cnt >= ms
    bad = []
    # counts (inner) and core flags (mid)
    if counts is not None:
        got = counts[ids].cpu().numpy().astype(np.int64)
        want = cnt if full_counts else np.minimum(cnt, ms)
        if not np.array_equal(got[inner], want[inner]):
            bad.append(f"counts differ at {int((got[inner] != want[inner]).sum())} inner points")
    if not np.array_equal(cor[mid], core_x[mid]):
        bad.append(f"core flags differ at {int((cor[mid] != core_x[mid]).sum())} points")
    # edges and borders of inner points
    rows = np.repeat(np.arange(len(Xe)), cnt)
    sel = inner[rows]
    i_, j_ = rows[sel], nbr[sel]
    cc = core_x[i_] & core_x[j_]
    if not np.array_equal(lab[i_[cc]], lab[j_[cc]]):
        bad.append(f"{int((lab[i_[cc]] != lab[j_[cc]]).sum())} core-core edges split")
    if np.any(lab[inner & core_x] < 0):
        bad.append("core point labelled noise")
    border = inner & ~core_x
    want_b = np.full(len(Xe), -1, np.int64)
    bsel = border[i_] & core_x[j_]
    if bsel.any():
        big = np.iinfo(np.int64).max
        tmp = np.full(len(Xe), big, np.int64)
        np.minimum.at(tmp, i_[bsel], lab[j_[bsel]])
        want_b = np.where(tmp == big, -1, tmp)
    if not np.array_equal(lab[border], want_b[border]):
        bad.append(f"{int((lab[border] != want_b[border]).sum())} border/noise labels differ")
    # local clusters: refinement and closed clusters
    lab_l, core_l, _, ncl_l = oracle.dbscan(Xe, eps, ms)
    core_l = core_l.astype(bool)
    closed = 0
    for k in range(ncl_l):
        mem_core = np.nonzero((lab_l == k) & core_l)[0]
        g = np.unique(lab[mem_core])
        if len(g) != 1:
            bad.append(f"local cluster {k} spans GPU labels {g[:4]}")
            continue
        if not np.all(inner[mem_core]):
            continue
        closed += 1
        gl = int(g[0])
        # every point carrying gl: a core of k, or a non-core point within eps of one
        carry = np.nonzero(lab == gl)[0]
        mk = np.zeros(len(Xe), bool)
        mk[mem_core] = True
        adj = np.zeros(len(Xe), bool)
        ks = mk[rows]
        adj[nbr[ks]] = True
        ok = mk[carry] | (adj[carry] & ~core_x[carry])
        if not ok.all():
            bad.append(f"closed cluster {k}: {int((~ok).sum())} foreign points carry its label")
        if int(label_hist[gl + 1]) != len(carry):
            bad.append(f"closed cluster {k}: label {gl} also used outside the window "
                       f"({int(label_hist[gl + 1])} points vs {len(carry)})")
    if bad:
        raise AssertionError(f"window at {np.asarray(c).tolist()} h={h}: " + "; ".join(bad))
    return dict(points=len(Xe), inner=int(inner.sum()), core=int((inner & core_x).sum()),
                border=int((border & (want_b >= 0)).sum()), noise=int((border & (want_b < 0)).sum()),
                edges=int(cc.sum()), local_clusters=int(ncl_l), closed=closed)


def check_clique_window(X, labels, core, counts, eps, ms, c, max_pts=3_000_000):
    """A window too dense for the sweep oracle (a C4 city centre holds ~6e4
    points per eps-cell): inner half-width h = eps / (2 sqrt(d)) (minus a
    1e-6 margin), so every two inner points are neighbours.  Checked exactly:
    neighbour counts capped at min_samples and core flags of every inner
    point (brute force against every point within h + eps, which holds all
    their neighbours), and — the inner core points forming a clique — one
    GPU label for all of them; an inner non-core point next to that clique
    carries a label no larger than it (its smallest adjacent cluster)."""
    d = X.shape[1]
    h = eps / (2.0 * np.sqrt(d)) * (1 - 1e-6)
    m = _extract_mask(X, c, h + eps * (1 + 1e-6) + 1e-12)
    ids = torch.nonzero(m).flatten()
    if ids.numel() > max_pts:
        raise AssertionError(f"clique window at {np.asarray(c).tolist()}: {ids.numel()} points")
    Xm = X[ids].double().cpu().numpy()
    dist = np.abs(Xm - np.asarray(c, np.float64)[None, :]).max(axis=1)
    inner = dist <= h
    lab = labels[ids].cpu().numpy().astype(np.int64)[inner]
    cor = core[ids].cpu().numpy().astype(bool)[inner]
    cnt = oracle.counts_capped(Xm[inner], Xm, eps, ms)
    core_x = cnt >= ms
    bad = []
    if counts is not None:
        got = np.minimum(counts[ids].cpu().numpy().astype(np.int64)[inner], ms)
        if not np.array_equal(got, cnt):
            bad.append(f"capped counts differ at {int((got != cnt).sum())} inner points")
    if not np.array_equal(cor, core_x):
        bad.append(f"core flags differ at {int((cor != core_x).sum())} inner points")
    g = np.unique(lab[core_x])
    if len(g) > 1 or (len(g) == 1 and g[0] < 0):
        bad.append(f"inner clique spans GPU labels {g[:4]}")
    if len(g) == 1 and np.any((lab[~core_x] < 0) | (lab[~core_x] > g[0])):
        bad.append("border point next to the clique with a larger label or noise")
    if bad:
        raise AssertionError(f"clique window at {np.asarray(c).tolist()}: " + "; ".join(bad))
    return dict(points=len(Xm), inner=int(inner.sum()), core=int(core_x.sum()),
                border=int((~core_x).sum()), noise=0,
                edges=int(core_x.sum()) * (int(core_x.sum()) - 1) // 2, local_clusters=len(g),
                closed=0)


def check_numbering(labels, core):
    """Global, size-independent: clusters are numbered 0..C-1 in order of
    their smallest core point index and each holds a core point (sklearn's
    order).  Returns C."""
    lab = labels.long()
    c = core.bool() & (lab >= 0)
    C = int(lab.max().item()) + 1 if lab.numel() else 0
    if C == 0:
        return 0
    n = lab.numel()
    first = torch.full((C,), n, dtype=torch.long, device=lab.device)
    idx = torch.arange(n, device=lab.device)
    first.scatter_reduce_(0, lab[c], idx[c], reduce="amin")
    assert int(first.max().item()) < n, "a cluster without a core point"
    assert bool((first[1:] > first[:-1]).all().item()), "clusters not in smallest-core order"
    assert not bool((core.bool() & (lab < 0)).any().item()), "core point labelled noise"
    return C


def run_windows(X, labels, core, counts, eps, ms, full_counts, n_random=30, n_dense=10,
                n_uniform=10, max_pts=20_000, seed=0):
    """The window sweep; returns the list of per-window tallies and the
    windows that took the clique check (even h = eps/8 held too many points
    for the sweep oracle)."""
    hist = torch.bincount(labels.long() + 1).cpu().numpy()
    pts, uni = random_centres(X, max(n_random, n_uniform), seed=seed + 1)
    centres = [("dense", c) for c in dense_centres(X, eps, n_dense, seed=seed)]
    centres += [("random", c) for c in pts[:n_random]] + [("uniform", c) for c in uni[:n_uniform]]
    out, clique = [], []
    for kind, c in centres:
        e = extract(X, c, 10 * eps, eps, max_pts)
        if e is None:
            t = check_clique_window(X, labels, core, counts, eps, ms, c)
            t.update(kind=kind, h=None, clique=True)
            clique.append(kind)
        else:
            h, ids = e
            t = check_window(X, labels, core, counts, hist, eps, ms, c, h, ids, full_counts)
            t.update(kind=kind, h=h, clique=False)
        out.append(t)
    return out, clique
