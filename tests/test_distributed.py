"""Sharded train (pypardis_amd/distributed.py) over gloo, world size 2 and 3,
on CPU: the orchestration and every collective are the product code; the
per-rank device stages are the oracle stand-in (tests/sharded_ops.py).  The
assembled labels must equal sklearn's on the golden data sets, and the KD
trace must equal the single-process exact-sum partition."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from conftest import load_golden
from dist_worker import run_world
from pypardis_amd.distributed import dd_combine, partition_ranks

CASES = [("c0", 2, 2), ("c0", 3, 4), ("b2d_20k", 2, 8), ("b3d_20k", 2, 4), ("ident_40", 2, 4),
         ("c0_p5_cityblock", 2, 5), ("dup_1d", 3, 3), ("lattice_900", 2, 8)]


@pytest.mark.parametrize("name,world,P", CASES)
def test_sharded_labels_equal_sklearn(tmp_path, name, world, P):
    g = load_golden(name)
    metric = str(g["metric"]) if "metric" in g else "euclidean"
    X = g["X"]
    if X.ndim == 1:
        X = X[:, None]
    mcode = 1 if metric in ("cityblock", "manhattan") else 0
    # contiguous label blocks (interleaved halves of the KD tree: many points
    # on two ranks, the cross-rank merge exercised); the other placements:
    # test_sharded_lpt_equals_blocks
    out = run_world(world, X, float(g["eps"]), int(g["min_samples"]), mcode, P, str(tmp_path),
                    placement="blocks")
    assert (out["seen"] == 1).all(), "every point owned by exactly one rank"
    np.testing.assert_array_equal(out["labels"], g["sk_labels"])
    np.testing.assert_array_equal(out["core"], g["sk_core"].astype(np.uint8))
    assert out["ncl"] == {int(g["sk_labels"].max()) + 1}
    assert out["received"] >= len(X)   # halo copies travel to both sides
    # labels returned to the ranks holding the points, in input order
    np.testing.assert_array_equal(out["loc_labels"], g["sk_labels"])
    np.testing.assert_array_equal(out["loc_core"], g["sk_core"].astype(np.uint8))
    if name in ("b2d_20k", "b3d_20k", "lattice_900"):
        assert out["exports"] > 0      # the cross-rank merge is exercised
    kd = oracle.kd_partition(X, P, sums="exact")
    for sp in out["splits"]:
        np.testing.assert_array_equal(sp, np.array(kd["splits"], np.float64))


def test_partition_ranks_lpt():
    """LPT placement of KD leaves: heaviest leaf first onto the
    least-loaded rank — non-contiguous label sets, loads within one leaf of
    each other; contiguous blocks without weights or when P <= world."""
    from pypardis_amd.distributed import partition_ranks, leaf_sizes
    pr, li = partition_ranks(6, 2, [10, 1, 1, 10, 5, 5])
    assert pr.tolist() == [0, 0, 1, 1, 0, 1]
    assert li.tolist() == [0, 1, 0, 1, 2, 2]
    pr, _ = partition_ranks(6, 2)
    assert pr.tolist() == [0, 0, 0, 1, 1, 1]
    pr, _ = partition_ranks(2, 4, [5, 7])
    assert pr.tolist() == [0, 2]
    rng = np.random.default_rng(0)
    w = rng.zipf(1.5, 64).astype(np.float64)
    pr, _ = partition_ranks(64, 8, w)
    load = np.bincount(pr, weights=w, minlength=8)
    assert load.max() - load.min() <= w.max() + 1e-9
    # leaf sizes from a split trace (cur, new, axis, cand, n_left, n_right, ...)
    sp = [(0, 1, 0, 3, 60, 40, 0., 0., 0.), (0, 2, 1, 3, 25, 35, 0., 0., 0.),
          (1, 3, 1, 3, 30, 10, 0., 0., 0.)]
    assert leaf_sizes(sp, 100, 4).tolist() == [25, 30, 35, 10]


def test_partition_ranks_ordered():
    """Spatially ordered placement: the KD leaves' depth-first order (a BFS
    schedule of 8 leaves: 0 4 2 6 1 5 3 7) cut into balanced contiguous runs
    — for equal leaves exactly the subtrees (2 ranks: the two halves of the
    first split; 4 ranks: the four quarters); the default picks LPT only when
    it balances more than 5 % better."""
    from pypardis_amd.distributed import kd_leaf_order, partition_ranks
    order = kd_leaf_order([(a, b, 0, 0, 0, 0) for a, b in
                           [(0, 1), (0, 2), (1, 3), (0, 4), (1, 5), (2, 6), (3, 7)]])
    assert order == [0, 4, 2, 6, 1, 5, 3, 7]
    pr, _ = partition_ranks(8, 2, np.ones(8), order)
    assert pr.tolist() == [0, 1, 0, 1, 0, 1, 0, 1]
    pr, _ = partition_ranks(8, 4, np.ones(8), order)
    assert [sorted(np.nonzero(pr == r)[0].tolist()) for r in range(4)] == \
        [[0, 4], [2, 6], [1, 5], [3, 7]]
    # skew that contiguous runs cannot balance: LPT is taken
    w = np.array([1, 1, 1, 1, 1, 1, 9, 9.])   # leaves 6 and 7 in runs 1 and 3
    pr_o, _ = partition_ranks(8, 2, w, order, "ordered")
    pr_l, _ = partition_ranks(8, 2, w, order, "lpt")
    pr_d, _ = partition_ranks(8, 2, w, order)
    lo = np.bincount(pr_o, weights=w).max()
    ll = np.bincount(pr_l, weights=w).max()
    assert ll <= lo
    assert pr_d.tolist() == (pr_o if lo <= 1.05 * ll else pr_l).tolist()
    # every rank gets a non-empty run when there are enough leaves
    rng = np.random.default_rng(3)
    pr, _ = partition_ranks(64, 8, rng.random(64) + 0.1, list(rng.permutation(64)), "ordered")
    assert set(pr.tolist()) == set(range(8))


def _dp_cut_max(w, order, world):
    """The smallest largest run load of a cut of `order` into min(world, P)
    contiguous runs, by the O(world P^2) dynamic programme (the round-5 form)."""
    ws = np.asarray(w, np.float64)[list(order)]
    P = len(ws)
    S = np.concatenate([[0.0], np.cumsum(ws)])
    dp = S.copy()
    dp[0] = np.inf
    for _ in range(2, min(world, P) + 1):
        nd = np.full(P + 1, np.inf)
        for i in range(1, P + 1):
            nd[i] = min((max(dp[j], S[i] - S[j]) for j in range(1, i)), default=np.inf)
        dp = nd
    return dp[P]


def test_ordered_cut_is_optimal_and_scales():
    """the ordered cut by bisection + greedy feasibility is as good
    as the exact dynamic programme (random small cases), every rank gets a
    non-empty contiguous run, and P = 65536 leaves over 8 ranks costs
    O(P log P) — no (P+1)^2 tables; kd_leaf_order is built from the tree."""
    import collections
    import time
    from pypardis_amd.distributed import _ordered_cut, kd_leaf_order
    rng = np.random.default_rng(5)
    for t in range(120):
        P, W = int(rng.integers(1, 24)), int(rng.integers(1, 9))
        w = rng.zipf(1.5, P).astype(np.float64) if t % 2 else rng.random(P) + 0.1
        order = list(rng.permutation(P))
        pr = _ordered_cut(w, order, W)
        assert len(set(pr.tolist())) == min(W, P)
        runs = [int(pr[L]) for L in order]
        assert runs == sorted(runs)
        best = _dp_cut_max(w, order, W)
        assert np.bincount(pr, weights=w).max() <= best * (1 + 1e-12)
    # a BFS schedule of 65536 leaves (labels as _create_partitions assigns them)
    P, splits, nxt, q = 65536, [], 1, collections.deque([0])
    while nxt < P:
        level, q = list(q), collections.deque()
        for c in level:
            if nxt < P:
                splits.append((c, nxt, 0, 0, 0, 0))
                q.extend([c, nxt])
                nxt += 1
            else:
                q.append(c)
    t0 = time.perf_counter()
    order = kd_leaf_order(splits)
    assert sorted(order) == list(range(P))
    w = rng.zipf(1.3, P).astype(np.float64)
    pr, li = partition_ranks(P, 8, w, order, "ordered")
    assert time.perf_counter() - t0 < 10.0
    assert set(pr.tolist()) == set(range(8))
    assert [int(pr[L]) for L in order] == sorted(int(pr[L]) for L in order)
    # the depth-first order equals the splice-based definition on a small tree
    seq = [0]
    for cur, nl, *_ in splits[:300]:
        i = seq.index(cur)
        seq[i:i + 1] = [cur, nl]
    assert kd_leaf_order(splits[:300]) == seq


@pytest.mark.parametrize("name,world,P", [("b3d_20k", 3, 8), ("lattice_900", 2, 8)])
def test_sharded_lpt_equals_blocks(tmp_path, name, world, P):
    """The sharded train with LPT leaf placement (non-contiguous label sets
    per rank), spatially ordered runs (the default's usual choice) and
    contiguous label blocks: all give sklearn's labels and core flags on
    every point."""
    from pypardis_amd.distributed import partition_ranks, leaf_sizes
    g = load_golden(name)
    X = g["X"]
    kd = oracle.kd_partition(X, P, sums="exact")
    pr, _ = partition_ranks(P, world, leaf_sizes(kd["splits"], len(X), P))
    for placement in ("lpt", "ordered", "blocks"):
        (tmp_path / placement).mkdir()
        out = run_world(world, X, float(g["eps"]), int(g["min_samples"]), 0, P,
                        str(tmp_path / placement), placement=placement)
        assert (out["seen"] == 1).all()
        np.testing.assert_array_equal(out["labels"], g["sk_labels"])
        np.testing.assert_array_equal(out["core"], g["sk_core"].astype(np.uint8))
        np.testing.assert_array_equal(out["loc_labels"], g["sk_labels"])
        assert {str(r["placement"]) for r in out["ranks"]} == {placement}
    if name == "b3d_20k":   # the case really is non-contiguous
        assert any(pr[i] > pr[i + 1] for i in range(P - 1)), pr


@pytest.mark.parametrize("name,world,P", [("b3d_20k", 2, 8), ("c0", 3, 5)])
def test_sharded_rotation_split(tmp_path, name, world, P):
    """split_method='rotation' over ranks: the all-reduced digit histograms
    give the same medians as one process (oracle sort), labels stay sklearn's."""
    g = load_golden(name)
    X = g["X"]
    out = run_world(world, X, float(g["eps"]), int(g["min_samples"]), 0, P, str(tmp_path),
                    split_method="rotation")
    np.testing.assert_array_equal(out["labels"], g["sk_labels"])
    kd = oracle.kd_partition(X, P, split_method="rotation")
    want = np.array(kd["splits"], np.float64)
    for sp in out["splits"]:
        np.testing.assert_array_equal(sp, want)


def test_dd_combine_matches_exact_sum():
    rng = np.random.default_rng(3)
    v = rng.normal(size=(3, 1000)) * 10.0 ** rng.integers(-8, 8, size=(3, 1000))
    import math
    parts = []
    for chunk in np.array_split(np.arange(1000), 4):
        p = np.zeros((1, 5))
        p[0, 0] = len(chunk)
        hi = math.fsum(v[0, chunk])
        p[0, 1], p[0, 2] = hi, math.fsum(list(v[0, chunk]) + [-hi])
        hi = math.fsum(v[1, chunk])
        p[0, 3], p[0, 4] = hi, math.fsum(list(v[1, chunk]) + [-hi])
        parts.append(p)
    mom = dd_combine(np.stack(parts))
    assert mom[0, 0, 0] == 1000
    assert mom[0, 1, 0] == math.fsum(v[0])
    assert mom[0, 2, 0] == math.fsum(v[1])


def test_partition_ranks():
    pr, li = partition_ranks(8, 8)
    assert pr.tolist() == list(range(8)) and li.tolist() == [0] * 8
    pr, li = partition_ranks(5, 2)
    assert pr.tolist() == [0, 0, 0, 1, 1] and li.tolist() == [0, 1, 2, 0, 1]
    pr, li = partition_ranks(2, 4)
    assert pr.tolist() == [0, 2] and li.tolist() == [0, 0]


def test_sharded_c4_skew(tmp_path):
    """C4-like skewed 2-D density (40 Zipf cities in a 2°x1° tile, sigma0 =
    0.002°, eps = 0.001°, min_samples = 20) over 2 ranks with P = 8: the KD
    boxes are unbalanced and halo copies are dense, the labels still equal
    the oracle's global DBSCAN."""
    from pypardis_amd import synth
    X = synth.gps_skew(20_000, seed=8, n_cities=40, sigma0=0.002, lon=(-1.0, 1.0),
                       lat=(-0.5, 0.5)).numpy()
    want, core, _, nc = oracle.dbscan(X, 0.001, 20)
    out = run_world(2, X, 0.001, 20, 0, 8, str(tmp_path))
    assert (out["seen"] == 1).all()
    np.testing.assert_array_equal(out["labels"], want)
    np.testing.assert_array_equal(out["core"], core.astype(np.uint8))
    assert out["ncl"] == {nc}
    assert out["received"] >= len(X)


@pytest.mark.parametrize("name,world,P,keyed", [("b2d_20k", 2, 8, False), ("c0", 3, 4, True),
                                                 ("c0_p5_cityblock", 2, 5, False)])
def test_reference_api_in_process_group(tmp_path, name, world, P, keyed):
    """dbscan.DBSCAN(...).train(slice) inside a gloo process group runs the
    sharded train: every rank gets its slice's labels in input order, the
    global n_clusters_, identical bounding boxes (those of one process), and
    assignments() returns every (key, label) sorted by key."""
    g = load_golden(name)
    metric = str(g["metric"]) if "metric" in g else "euclidean"
    X = g["X"]
    mcode = 1 if metric in ("cityblock", "manhattan") else 0
    out = run_world(world, X, float(g["eps"]), int(g["min_samples"]), mcode, P, str(tmp_path),
                    api=True, keyed=keyed)
    np.testing.assert_array_equal(out["loc_labels"], g["sk_labels"])
    np.testing.assert_array_equal(out["loc_core"], g["sk_core"].astype(np.uint8))
    kd = oracle.kd_partition(X, P, sums="exact")
    want_keys = np.array([("k%06d" % i) if keyed else str(i) for i in range(len(X))])
    order = np.arange(len(X))   # key order = input order (numeric / zero-padded keys)
    for z in out["ranks"]:
        assert int(z["n_clusters_"]) == int(g["sk_labels"].max()) + 1
        np.testing.assert_array_equal(z["boxes_api"][:, 0], kd["box_lo"])
        np.testing.assert_array_equal(z["boxes_api"][:, 1], kd["box_hi"])
        np.testing.assert_array_equal(z["assign_keys"], want_keys[order])
        np.testing.assert_array_equal(z["assign_labels"], g["sk_labels"][order])
        assert int(z["count"]) == len(X)


@pytest.mark.parametrize("name,world,P,keyed", [("c0_p3", 2, 3, False), ("b2d_20k", 3, 8, True)])
def test_sharded_model_data_is_partition_records(tmp_path, name, world, P, keyed):
    """DBSCAN.data after a sharded train (a gloo group) is the
    reference's per-partition records (R:dbscan/dbscan.py:116-125): for each
    neighbourhood, in partition order, its members in input order as (key,
    'L:c[*]') with the neighbourhood's own sklearn labels — the records one
    device gives for the union of the slices (same KD boxes: exact sums), on
    every rank; count() equals the number of records."""
    g = load_golden(name)
    X = g["X"]
    eps, ms = float(g["eps"]), int(g["min_samples"])
    out = run_world(world, X, eps, ms, 0, P, str(tmp_path), api=True, keyed=keyed)
    kd = oracle.kd_partition(X, P, sums="exact")
    _, _, members = oracle.halo(X, kd["box_lo"], kd["box_hi"], eps)
    want_k, want_s = [], []
    for L, idx in enumerate(members):
        if not len(idx):
            continue
        lab, core, _, _ = oracle.dbscan(X[idx], eps, ms)
        want_k += [("k%06d" % i) if keyed else str(i) for i in idx.tolist()]
        want_s += ["%i:%i%s" % (L, c, "" if f else "*") for c, f in zip(lab.tolist(), core.tolist())]
    for z in out["ranks"]:
        assert z["data_keys"].tolist() == want_k
        assert z["data_recs"].tolist() == want_s
        assert int(z["data_count"]) == len(want_k)
    if name == "c0_p3" and np.array_equal(kd["box_lo"], g["box_lo"]):
        # the exact-sum boxes are the reference's here: its own records
        po = g["part_out"]
        ref = ["%i:%i%s" % (L, c, "" if f else "*") for L, _, c, f in po.tolist()]
        assert want_k == [str(int(k)) for k in po[:, 1]] and want_s == ref


def test_train_threads_local_comm():
    """One process, several ranks as threads (the n_gpus > 1 path without a
    process group): distributed.train_threads with an in-process collective
    layer and the oracle stand-in gives sklearn's labels on every slice."""
    from local_comm import local_comms
    from pypardis_amd.distributed import train_threads
    from sharded_ops import OracleOps
    import torch
    g = load_golden("b3d_20k")
    X = g["X"]
    W = 3
    cuts = [r * len(X) // W for r in range(W + 1)]
    slices = [torch.from_numpy(np.ascontiguousarray(X[cuts[r]:cuts[r + 1]])) for r in range(W)]
    res = train_threads(slices, float(g["eps"]), int(g["min_samples"]), local_comms(W),
                        [OracleOps() for _ in range(W)], max_partitions=4)
    labels = np.concatenate([r.local_labels.numpy() for r in res])
    np.testing.assert_array_equal(labels, g["sk_labels"])
    assert {r.n_clusters for r in res} == {int(g["sk_labels"].max()) + 1}


def test_all_slices_empty_raises_clearly():
    """Every rank's slice empty: the sharded train names that ("no points on
    any rank") on every rank, not an error of the empty KD."""
    from local_comm import local_comms
    from pypardis_amd.distributed import train_threads
    from sharded_ops import OracleOps
    import torch
    W = 2
    slices = [torch.zeros((0, 3), dtype=torch.float32) for _ in range(W)]
    with pytest.raises(ValueError, match="no points on any rank"):
        train_threads(slices, 0.1, 5, local_comms(W), [OracleOps() for _ in range(W)],
                      max_partitions=4, abort_timeout=30.0)


def test_train_threads_rank_failure_aborts():
    """A rank that fails alone (here: its ops raise in phase A) must not leave
    the other ranks waiting for it for ever: train_threads aborts the
    communicators and raises that rank's error."""
    import time

    from local_comm import local_comms
    from pypardis_amd.distributed import train_threads
    from sharded_ops import OracleOps
    import torch

    class Failing(OracleOps):
        def train_begin(self, *a, **k):
            raise RuntimeError("injected failure on one rank")

    g = load_golden("b3d_20k")
    X = g["X"]
    W = 3
    cuts = [r * len(X) // W for r in range(W + 1)]
    slices = [torch.from_numpy(np.ascontiguousarray(X[cuts[r]:cuts[r + 1]])) for r in range(W)]
    ops = [OracleOps(), Failing(), OracleOps()]
    t0 = time.time()
    with pytest.raises(RuntimeError, match="injected failure"):
        train_threads(slices, float(g["eps"]), int(g["min_samples"]), local_comms(W), ops,
                      max_partitions=4, abort_timeout=30.0)
    assert time.time() - t0 < 60


def _dense_blobs(n=6000, d=8, seed=5):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-4, 4, size=(6, d))
    X = c[rng.integers(0, 6, n)] + rng.normal(scale=0.35, size=(n, d))
    X[: n // 20] = rng.uniform(-5, 5, size=(n // 20, d))   # noise
    return X.astype(np.float32)


@pytest.mark.parametrize("case,world,api", [("c3_5k", 2, False), ("c3_5k", 3, True),
                                            ("blobs8", 2, False), ("blobs8", 3, True)])
def test_sharded_dense_equals_sklearn(tmp_path, case, world, api):
    """d > 4 over ranks (distributed._train_dense): slices all-gathered, the
    count / link / border stages split by row chunks with a sum, a forest
    gather and a min between them.  Labels equal sklearn's (the golden C3
    slice) or the oracle's (8-D blobs with > 2048 core points, so every
    rank's link share is non-empty); KD boxes equal one process's."""
    if case == "c3_5k":
        g = load_golden("c3_5k")
        X, eps, ms, P = g["X"], float(g["eps"]), int(g["min_samples"]), int(g["P"])
        want, core = g["sk_labels"], g["sk_core"].astype(np.uint8)
    else:
        X, eps, ms, P = _dense_blobs(), 0.9, 8, 4
        want, core, _, _ = oracle.dbscan(X, eps, ms)
        assert core.sum() > 2048
    out = run_world(world, X, eps, ms, 0, P, str(tmp_path), api=api)
    assert (out["seen"] == 1).all()
    np.testing.assert_array_equal(out["labels"], want)
    np.testing.assert_array_equal(out["core"], core)
    np.testing.assert_array_equal(out["loc_labels"], want)
    assert out["ncl"] == {int(want.max()) + 1}
    kd = oracle.kd_partition(X, P, sums="exact")
    for sp in out["splits"]:
        np.testing.assert_array_equal(sp, np.array(kd["splits"], np.float64))


def test_device_kd_applicability_from_schedule():
    """The device-decided KD needs levels that fit its 256-entry tables; the
    decision comes from the schedule alone, so every rank takes the same path
    (P = 1000 used to raise PD_EUNSUPPORTED on the sharded path)."""
    from pypardis_amd.distributed import device_kd_ok
    from pypardis_amd.partition import _split_schedule
    assert device_kd_ok(_split_schedule(8), 'min_var', False)
    assert device_kd_ok(_split_schedule(512), 'min_var', False)
    assert not device_kd_ok(_split_schedule(1000), 'min_var', False)
    assert not device_kd_ok(_split_schedule(8), 'rotation', False)
    assert not device_kd_ok(_split_schedule(8), 'min_var', True)
    assert not device_kd_ok(_split_schedule(1), 'min_var', False)


def test_sharded_result_keeps_owned_records_only_on_request():
    """train_sharded frees the per-record arrays unless keep_owned (ADVICE
    r03); return_local=False returns no local labels and keeps them."""
    from local_comm import local_comms
    from pypardis_amd.distributed import train_threads
    from sharded_ops import OracleOps
    import torch
    g = load_golden("b3d_20k")
    X = g["X"]
    W = 2
    cuts = [r * len(X) // W for r in range(W + 1)]
    slices = [torch.from_numpy(np.ascontiguousarray(X[cuts[r]:cuts[r + 1]])) for r in range(W)]
    res = train_threads(slices, float(g["eps"]), int(g["min_samples"]), local_comms(W),
                        [OracleOps() for _ in range(W)], max_partitions=4)
    with pytest.raises(AttributeError, match="keep_owned"):
        res[0].gid
    res = train_threads(slices, float(g["eps"]), int(g["min_samples"]), local_comms(W),
                        [OracleOps() for _ in range(W)], max_partitions=4, keep_owned=True)
    gid = np.concatenate([r.gid.numpy() for r in res])
    lab = np.concatenate([r.labels.numpy() for r in res])
    order = np.argsort(gid)
    np.testing.assert_array_equal(gid[order], np.arange(len(X)))
    np.testing.assert_array_equal(lab[order], g["sk_labels"])
