"""Full-size parity at the configs the bench reports:
C2 (100M 3-D points, max_partitions=8 — the headline), C1 (10M 2-D points,
64 centres) and C4 (1B 2-D GPS-like points, max_partitions=8).

The full answers are out of the CPU oracle's reach, so each run is checked
by windowed oracle spot checks (tests/window_check.py: exact neighbour
counts, exact core flags, core-core edges, border rule, closed local
clusters) at ~50 windows — density-weighted random points, the most
populated eps-cells, and uniform positions — plus global size-independent
properties: sklearn's cluster numbering, and labels independent of
max_partitions and of PD_OPT_FULL_COUNTS.

Reference semantics: R:dbscan/dbscan.py:12-34 (sklearn per 2·eps-expanded
box) and the merge intent of R:dbscan/dbscan.py:153-165.
"""
import numpy as np
import pytest
import torch

import window_check as wc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from pypardis_amd import _native
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    _native.load()
    return _native


def _train_counts(native, Xd, eps, ms, P, full):
    """DBSCAN.train's stages with the neighbour counts requested
    (PD_OPT_FULL_COUNTS: exact counts; otherwise capped at min_samples)."""
    from pypardis_amd import KDPartitioner
    kd = KDPartitioner(Xd, P)
    ebox = np.stack([kd.bounding_boxes[L].expand(2 * eps).as_array()
                     for L in sorted(kd.bounding_boxes)])
    ctx = native.context()
    ctx.set_option(native.PD_OPT_FULL_COUNTS, 1 if full else 0)
    try:
        lo, hi = kd.data_box
        lab, core, cnt, ncl = native.train(Xd, eps, ms, native.PD_EUCLIDEAN, ebox,
                                           owner=kd.labels if len(ebox) > 1 else None,
                                           data_box=np.stack([lo, hi]), want_counts=True)
    finally:
        ctx.set_option(native.PD_OPT_FULL_COUNTS, 0)
    return lab, core, cnt, ncl


def _full_run(native, name, Xd, P, full_counts, windows_min):
    from pypardis_amd import DBSCAN, synth
    cfg = synth.CONFIGS[name]
    eps, ms = cfg["eps"], cfg["min_samples"]
    m = DBSCAN(eps=eps, min_samples=ms, max_partitions=P).train(Xd)
    lab, core, cnt, ncl = _train_counts(native, Xd, eps, ms, P, full_counts)
    # the counting mode changes only what is counted, never the answer
    assert ncl == m.n_clusters_
    assert torch.equal(lab, m.labels_)
    assert torch.equal(core, m.core_sample_mask_)
    assert wc.check_numbering(m.labels_, m.core_sample_mask_) == m.n_clusters_
    tallies, clique = wc.run_windows(Xd, m.labels_, m.core_sample_mask_, cnt, eps, ms,
                                      full_counts)
    kinds = {k: sum(1 for t in tallies if t["kind"] == k) for k in ("dense", "random", "uniform")}
    tot = {k: sum(t[k] for t in tallies) for k in ("inner", "core", "border", "noise", "edges",
                                                   "closed")}
    print(f"\n{name}: n={Xd.shape[0]} clusters={m.n_clusters_} windows={kinds} "
          f"clique-checked={len(clique)} {tot}")
    assert len(tallies) >= windows_min, len(tallies)
    assert tot["core"] > 0 and tot["edges"] > 0
    return m


def test_c2_full_100m(native):
    """The headline workload, exactly as bench.py runs it."""
    from pypardis_amd import synth
    X, cfg = synth.make_config("C2")
    Xd = torch.from_numpy(X).cuda()
    del X
    _full_run(native, "C2", Xd, 8, True, 50)


def test_c1_full_10m(native):
    """C1 at full size (64 centres), one neighbourhood (its config) and 8."""
    from pypardis_amd import DBSCAN, synth
    X, cfg = synth.make_config("C1")
    Xd = torch.from_numpy(X).cuda()
    m = _full_run(native, "C1", Xd, 1, True, 50)
    m8 = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=8).train(Xd)
    assert torch.equal(m8.labels_, m.labels_)


def test_c4_full_1b(native):
    """C4 at full size (1B points generated on the device, as the bench does).
    Neighbour counts are checked capped at min_samples (an uncapped count of
    a city centre is ~1e5 candidates per point); the densest windows that the
    oracle can take hold 40k points; P=1 must give the same labels."""
    from pypardis_amd import DBSCAN, synth
    cfg = synth.CONFIGS["C4"]
    Xd = synth.gps_skew(cfg["n"], seed=cfg["seed"], device="cuda")
    m = _full_run(native, "C4", Xd, 8, False, 50)
    lab8 = m.labels_.clone()
    del m
    m1 = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=1).train(Xd)
    assert torch.equal(m1.labels_, lab8)


def test_c4_device_sample_vs_oracle(native):
    """The bench's C4 points come from the device RNG stream: a 1M-point sample
    of that stream, labels / core flags / cluster count against the oracle."""
    import oracle
    from pypardis_amd import DBSCAN, synth
    cfg = synth.CONFIGS["C4"]
    Xd = synth.gps_skew(1_000_000, seed=cfg["seed"], device="cuda")
    X = Xd.cpu().numpy()
    want, core_w, _, nc = oracle.dbscan(X, cfg["eps"], cfg["min_samples"])
    m = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=8).train(Xd)
    assert m.n_clusters_ == nc
    assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), want)
    assert np.array_equal(m.core_sample_mask_.cpu().numpy(), core_w)


# ------------------------------------------------------------ C3 (d = 64) at full size
def _exact_neighbours(X64, Q, eps, chunk=16384):
    """Every point within eps of each query (self included), by sklearn's exact
    predicate: candidates from an fp64 Gram bound with a wide margin, then the
    per-axis sum in axis order, every operation rounded (numpy elementwise),
    `<= eps*eps` (SK:neighbors/_binary_tree.pxi.tp:1949-1958; at d > 15 the
    reference's brute query differs only inside a 1-ulp band)."""
    qn = (X64[Q] ** 2).sum(1)
    cand = [[] for _ in Q]
    for s in range(0, len(X64), chunk):
        C = X64[s:s + chunk]
        cn = (C ** 2).sum(1)
        d2 = qn[:, None] + cn[None, :] - 2.0 * (X64[Q] @ C.T)
        ok = d2 <= eps * eps * 1.001 + 1e-9 * (qn[:, None] + cn[None, :])
        qi, ci = np.nonzero(ok)
        for a, b in zip(qi.tolist(), (ci + s).tolist()):
            cand[a].append(b)
    out = []
    eps2 = eps * eps
    for a, q in enumerate(Q):
        c = np.asarray(cand[a], np.int64)
        acc = np.zeros(len(c))
        for j in range(X64.shape[1]):
            t = X64[c, j] - X64[q, j]
            acc = acc + t * t
        out.append(c[acc <= eps2])
    return out


def test_c3_full_1m_vs_oracle(native):
    """The bench's C3 answer (1M x 64-D embeddings, eps 0.114028,
    min_samples 10) against the exact predicate on a sample:
    2,000 random points plus every core point of a random 20 % of the
    clusters — exact neighbour counts over all 1M points (the oracle's
    counts_capped on each candidate set, and the numpy restatement), exact
    core flags, equal labels on every core-core edge, each sampled cluster
    one connected component of its core points, and the border rule (the
    smallest label among the core neighbours, -1 without one)."""
    import oracle
    from pypardis_amd import synth
    X, cfg = synth.make_config("C3")
    eps, ms = cfg["eps"], cfg["min_samples"]
    ctx = native.context()
    ctx.set_option(native.PD_OPT_FULL_COUNTS, 1)
    try:
        lab_t, core_t, cnt_t, ncl = native.cluster(torch.from_numpy(X).cuda(), eps, ms,
                                                   want_counts=True)
    finally:
        ctx.set_option(native.PD_OPT_FULL_COUNTS, 0)
    lab = lab_t.cpu().numpy().astype(np.int64)
    core = core_t.cpu().numpy().astype(bool)
    cnt = cnt_t.cpu().numpy().astype(np.int64)
    assert ncl > 100 and core.sum() > 1000
    rng = np.random.default_rng(11)
    sample = rng.choice(len(X), 2000, replace=False)
    chosen = rng.choice(ncl, max(1, ncl // 5), replace=False)
    core_pts = np.nonzero(core & np.isin(lab, chosen))[0]
    Q = np.unique(np.concatenate([sample, core_pts]))
    X64 = X.astype(np.float64)
    nb = _exact_neighbours(X64, Q, eps)
    pos = {int(q): i for i, q in enumerate(Q)}
    edges = 0
    for i, q in enumerate(Q):
        c = nb[i]
        # pinned oracle on the candidate superset == the restatement == GPU
        assert oracle.counts_capped(X64[q:q + 1], X64[c], eps, 0)[0] == len(c)
        assert len(c) == cnt[q], (q, len(c), cnt[q])
        assert (len(c) >= ms) == core[q], q
        cn = c[core[c]]
        if core[q]:
            assert (lab[cn] == lab[q]).all(), q
            edges += len(cn)
        elif len(cn):
            assert lab[q] == lab[cn].min(), q
        else:
            assert lab[q] == -1, q
    # every chosen cluster's core points form one component of exact edges
    parent = {int(p): int(p) for p in core_pts}

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for p in core_pts:
        for r in nb[pos[int(p)]]:
            r = int(r)
            if r in parent:
                a, b = find(int(p)), find(r)
                if a != b:
                    parent[max(a, b)] = min(a, b)
    roots = {}
    for p in core_pts:
        roots.setdefault(int(lab[p]), set()).add(find(int(p)))
    assert set(roots) == set(int(c) for c in chosen if (lab[core] == c).any())
    assert all(len(r) == 1 for r in roots.values())
    print(f"\nC3 1M: clusters={ncl} queries={len(Q)} core-queries={len(core_pts)} "
          f"core-core edges={edges}")
