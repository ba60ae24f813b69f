"""GPU parity: the HIP path (through the C ABI) against the pinned oracle and
the reference goldens.  Bit-exact for everything integer-valued (labels, core
flags, neighbour counts, halo membership, split sizes, split boundaries —
the latter in 'sequential' sums mode against the reference, in the default
correctly-rounded mode against the oracle's exact sums)."""
import numpy as np
import pytest
import torch

import oracle
from conftest import GOLDEN, golden_names, load_golden, rotation_names

pytestmark = pytest.mark.gpu

NAMES = golden_names()


def _metric(g):
    m = str(g["metric"])
    return "euclidean" if m == "callable" else m


def _P(g):
    P = int(g["max_partitions"])
    return None if P < 0 else P


def _dev(X):
    return torch.from_numpy(np.ascontiguousarray(X)).cuda()


@pytest.fixture(scope="module")
def native():
    from pypardis_amd import _native
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    _native.load()
    return _native


def _cluster(native, X, eps, ms, metric="euclidean", full=False):
    ctx = native.context()
    ctx.set_option(native.PD_OPT_FULL_COUNTS, 1 if full else 0)
    try:
        lab, core, cnt, ncl = native.cluster(_dev(X), eps, ms, native.metric_code(metric),
                                             want_counts=full)
    finally:
        ctx.set_option(native.PD_OPT_FULL_COUNTS, 0)
    out = (lab.cpu().numpy().astype(np.int64), core.cpu().numpy(), ncl)
    if full:
        out = out + (cnt.cpu().numpy().astype(np.int64),)
    return out


# ------------------------------------------------------------ pd_cluster
def test_sklearn_kats(native):
    z = np.load(f"{GOLDEN}/sklearn_kat.npz")
    for ms in (1, 2, 3, 4):
        lab, core, _ = _cluster(native, z["toy_X"], 1.0, ms)
        assert np.array_equal(lab, z[f"toy_ms{ms}_labels"])
        assert np.array_equal(np.nonzero(core)[0], z[f"toy_ms{ms}_core"])
    assert np.array_equal(np.nonzero(_cluster(native, z["bnd_a_X"], 2, 2)[1])[0], z["bnd_a_core"])
    assert np.array_equal(np.nonzero(_cluster(native, z["bnd_b_X"], 1, 2)[1])[0],
                          z["bnd_b_core_eps1"])
    assert np.array_equal(np.nonzero(_cluster(native, z["bnd_b_X"], 0.99, 2)[1])[0],
                          z["bnd_b_core_eps099"])
    lab, core, _ = _cluster(native, z["clustered_X"], 0.8, 10)
    assert np.array_equal(lab, z["clustered_labels"])


@pytest.mark.parametrize("name", NAMES)
def test_cluster_equals_sklearn(native, name):
    g = load_golden(name)
    lab, core, ncl, cnt = _cluster(native, g["X"], float(g["eps"]), int(g["min_samples"]),
                                   _metric(g), full=True)
    assert np.array_equal(cnt, g["sk_counts"])
    assert np.array_equal(core, g["sk_core"])
    assert np.array_equal(lab, g["sk_labels"])
    assert ncl == int(g["sk_labels"].max()) + 1


# ------------------------------------------------------------ KD + halo
def _kd_arrays(splits):
    sp = np.array([s[:6] for s in splits], np.int64).reshape(-1, 6)
    sf = np.array([s[6:] for s in splits], np.float64).reshape(-1, 3)
    return sp, sf


@pytest.mark.parametrize("name", NAMES)
def test_kd_partitioner_sequential_is_bit_exact_with_reference(native, name):
    """sums='sequential': every split, boundary, box and owner label is
    bit-identical to the reference run (same fold order)."""
    from pypardis_amd import KDPartitioner
    g = load_golden(name)
    kd = KDPartitioner(_dev(g["X"]), _P(g), sums="sequential")
    sp, sf = _kd_arrays(kd.splits)
    assert np.array_equal(sp, g["splits"])
    assert np.array_equal(sf, g["split_f"])
    assert np.array_equal(kd.box_array()[:, 0], g["box_lo"])
    assert np.array_equal(kd.box_array()[:, 1], g["box_hi"])
    assert np.array_equal(kd.labels.cpu().numpy(), g["owner"])


@pytest.mark.parametrize("name", NAMES)
def test_kd_partitioner_exact_sums_match_oracle(native, name):
    """Default sums='exact': bit-identical to the oracle's correctly rounded
    restatement (and to the reference wherever its decision is not a tie —
    tests/test_oracle.py::test_exact_sums_agree_with_reference_except_ties)."""
    from pypardis_amd import KDPartitioner
    g = load_golden(name)
    kd = KDPartitioner(_dev(g["X"]), _P(g))
    ref = oracle.kd_partition(g["X"], _P(g), sums="exact")
    sp, sf = _kd_arrays(kd.splits)
    rp, rf = _kd_arrays(ref["splits"])
    assert np.array_equal(sp, rp)
    assert np.array_equal(sf, rf)
    assert np.array_equal(kd.box_array()[:, 0], ref["box_lo"])
    assert np.array_equal(kd.box_array()[:, 1], ref["box_hi"])
    assert np.array_equal(kd.labels.cpu().numpy(), ref["owner"])


@pytest.mark.parametrize("name", rotation_names())
def test_kd_partitioner_rotation_matches_reference(native, name):
    """split_method='rotation': the GPU radix-select medians, split sizes,
    boxes and owner labels are bit-identical to the reference's
    median_search_split (R:dbscan/partition.py:8-30) run on the same points."""
    from pypardis_amd import KDPartitioner
    g = load_golden(name, "rot")
    kd = KDPartitioner(_dev(g["X"]), int(g["max_partitions"]), split_method="rotation")
    sp = np.array([[s[0], s[1], s[2], s[4], s[5]] for s in kd.splits], np.int64)
    assert np.array_equal(sp, g["splits"])
    assert np.array_equal(np.array([s[8] for s in kd.splits]), g["medians"])
    assert np.array_equal(kd.box_array()[:, 0], g["box_lo"])
    assert np.array_equal(kd.box_array()[:, 1], g["box_hi"])
    assert np.array_equal(kd.labels.cpu().numpy(), g["owner"])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_kd_rotation_large_matches_oracle(native, dtype):
    """2M points with heavy ties and negative values, P=13: GPU medians vs the
    oracle's sort (fp32 and fp64 inputs)."""
    from pypardis_amd import KDPartitioner
    rng = np.random.default_rng(31)
    X = np.round(rng.normal(size=(2_000_000, 3)) * 50.0, 1).astype(dtype)
    kd = KDPartitioner(_dev(X), 13, split_method="rotation")
    ref = oracle.kd_partition(X, 13, split_method="rotation")
    assert np.array_equal(np.array([s[8] for s in kd.splits]),
                          np.array([s[8] for s in ref["splits"]]))
    assert np.array_equal(kd.labels.cpu().numpy(), ref["owner"])


@pytest.mark.parametrize("name", NAMES)
def test_halo_members_match_reference(native, name):
    g = load_golden(name)
    ebox = np.stack([g["ebox_lo"], g["ebox_hi"]], axis=1)
    counts, members = native.halo_members(_dev(g["X"]), ebox)
    m = members.cpu().numpy()
    off = np.concatenate([[0], np.cumsum(counts)])
    pairs = np.array(sorted((L, int(i)) for L in range(len(counts)) for i in m[off[L]:off[L + 1]]),
                     np.int64).reshape(-1, 2)
    assert np.array_equal(pairs, g["halo"])


# ------------------------------------------------------------ end to end
@pytest.mark.parametrize("name", NAMES)
def test_train_equals_global_dbscan(native, name):
    import dbscan   # the drop-in import name
    g = load_golden(name)
    X = g["X"]
    model = dbscan.DBSCAN(eps=float(g["eps"]), min_samples=int(g["min_samples"]),
                          metric=_metric(g), max_partitions=_P(g), kd_sums="sequential")
    model.train([(i, X[i]) for i in range(len(X))])
    a = model.assignments()
    assert [k for k, _ in a] == list(range(len(X)))
    assert np.array_equal(np.array([v for _, v in a]), g["sk_labels"])
    assert np.array_equal(model.core_sample_mask_.cpu().numpy(), g["sk_core"])
    P = int(g["P"])
    assert sorted(model.bounding_boxes) == list(range(P))
    for L in range(P):
        assert np.array_equal(model.expanded_boxes[L].lower, g["ebox_lo"][L])
        assert np.array_equal(model.expanded_boxes[L].upper, g["ebox_hi"][L])
        ref = g["halo"][g["halo"][:, 0] == L, 1]
        assert np.array_equal(np.sort(model.neighbors[L].keys()), ref)


def test_dbscan_partition_string_records(native):
    from pypardis_amd import dbscan_partition
    g = load_golden("c0_p3")
    po = g["part_out"]
    X = g["X"]
    params = {"eps": float(g["eps"]), "min_samples": int(g["min_samples"]), "metric": "euclidean"}
    for L in range(int(g["P"])):
        rows = po[po[:, 0] == L]
        recs = [((int(k), L), X[k]) for k in rows[:, 1]]
        out = list(dbscan_partition(iter(recs), params))
        want = [(int(k), "%i:%i%s" % (L, c, "" if core else "*")) for _, k, c, core in rows]
        assert [(int(k), s) for k, s in out] == want


def test_model_data_is_reference_partition_records(native):
    """DBSCAN.data after train is what the reference leaves there
    (R:dbscan/dbscan.py:116-125): per KD partition, in partition order, its
    halo members in input order as (key, 'L:c[*]') with the partition's own
    sklearn label — equal to the reference's dbscan_partition records
    (kd_sums='sequential': the reference's boxes)."""
    from pypardis_amd import DBSCAN
    g = load_golden("c0_p3")
    po = g["part_out"]
    m = DBSCAN(eps=float(g["eps"]), min_samples=int(g["min_samples"]),
               max_partitions=int(g["P"]), kd_sums="sequential").train(_dev(g["X"]))
    want = []
    for L in range(int(g["P"])):
        for _, k, c, core in po[po[:, 0] == L]:
            want.append((int(k), "%i:%i%s" % (L, c, "" if core else "*")))
    got = [(int(k), s) for k, s in m.data.collect()]
    assert got == want
    assert m.data.count() == len(want)


# ------------------------------------------------------------ larger vs oracle
CASES = [
    ("2d_c1slice", dict(n=150_000, d=2, side=100 * (0.015 ** 0.5), n_centers=1, sigma=1.0,
                        noise_frac=0.1, seed=21), 0.05, 10, "euclidean", 4),
    ("3d_c2slice", dict(n=200_000, d=3, side=100 * (0.002 ** (1 / 3)), n_centers=1, sigma=1.0,
                        noise_frac=0.1, seed=22), 0.1, 10, "euclidean", 8),
    ("3d_dense", dict(n=120_000, d=3, side=8.0, n_centers=6, sigma=0.5, noise_frac=0.05,
                      seed=23), 0.08, 20, "euclidean", 8),
    ("2d_cityblock", dict(n=100_000, d=2, side=30.0, n_centers=10, sigma=0.7, noise_frac=0.2,
                          seed=24), 0.06, 8, "cityblock", 5),
    ("4d", dict(n=60_000, d=4, side=6.0, n_centers=8, sigma=0.4, noise_frac=0.1, seed=25),
     0.25, 10, "euclidean", 4),
    ("1d", dict(n=50_000, d=1, side=50.0, n_centers=20, sigma=0.3, noise_frac=0.3, seed=26),
     0.002, 5, "euclidean", 4),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_train_matches_oracle(native, case):
    from pypardis_amd import DBSCAN, synth
    _, kw, eps, ms, metric, P = case
    X = synth.blobs_noise(**kw)
    lab_o, core_o, cnt_o, _ = oracle.dbscan(X, eps, ms, metric)
    lab, core, ncl, cnt = _cluster(native, X, eps, ms, metric, full=True)
    assert np.array_equal(cnt, cnt_o)
    assert np.array_equal(core, core_o)
    assert np.array_equal(lab, lab_o)
    m = DBSCAN(eps=eps, min_samples=ms, metric=metric, max_partitions=P).train(_dev(X))
    assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), lab_o)
    assert m.n_clusters_ == ncl


@pytest.mark.parametrize("stats", [0, 1])
def test_sweeps_exact(native, stats):
    """The shipped sweeps — the count sweep at 8 waves per SIMD, its
    instrumented form (PD_OPT_SWEEP_STATS), the window union + cell verify
    link and the border sweep — give the oracle's counts, core flags and
    labels on every case: 1-D..4-D, cityblock, fp64, exact ties,
    min_samples 1..34, several neighbourhoods (waves straddling two), the
    sharded phases (1-rank RCCL) and the goldens."""
    from pypardis_amd import DBSCAN, distributed, synth
    ctx = native.context()
    ctx.set_option(native.PD_OPT_SWEEP_STATS, stats)
    try:
        for _, kw, eps, ms, metric, P in CASES:
            X = synth.blobs_noise(**kw)
            lab_o, core_o, cnt_o, _ = oracle.dbscan(X, eps, ms, metric)
            lab, core, ncl, cnt = _cluster(native, X, eps, ms, metric, full=True)
            assert np.array_equal(cnt, cnt_o), kw
            assert np.array_equal(lab, lab_o), kw
            m = DBSCAN(eps=eps, min_samples=ms, metric=metric, max_partitions=P).train(_dev(X))
            assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), lab_o), kw
            assert np.array_equal(m.core_sample_mask_.cpu().numpy(), core_o), kw
        g = np.arange(60, dtype=np.float32) * np.float32(0.05)
        lattice = np.stack(np.meshgrid(g, g, indexing="ij"), -1).reshape(-1, 2)
        lab_o, _, cnt_o, _ = oracle.dbscan(lattice, float(np.float32(0.05)), 5)
        lab, _, _, cnt = _cluster(native, lattice, float(np.float32(0.05)), 5, full=True)
        assert np.array_equal(cnt, cnt_o) and np.array_equal(lab, lab_o)
        X = synth.blobs_noise(30_000, 3, side=5.0, n_centers=4, sigma=0.3, seed=61)
        X64 = X.astype(np.float64) + np.random.default_rng(2).uniform(-1e-9, 1e-9, X.shape)
        for Y, ms in ((X, 1), (X, 30), (X64, 6)):
            lab_o, core_o, _, _ = oracle.dbscan(Y, 0.06, ms)
            m = DBSCAN(eps=0.06, min_samples=ms, max_partitions=6).train(_dev(Y))
            assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), lab_o), ms
        X = synth.blobs_noise(40_000, 3, side=5.0, n_centers=4, sigma=0.3, noise_frac=0.3,
                              seed=71)
        for ms in (2, 20, 33, 34):
            lab_o, core_o, _, _ = oracle.dbscan(X, 0.06, ms)
            m = DBSCAN(eps=0.06, min_samples=ms, max_partitions=6).train(_dev(X))
            assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), lab_o), ms
            assert np.array_equal(m.core_sample_mask_.cpu().numpy(), core_o), ms
        if stats:
            comm = distributed.device_comms([0])[0]
            res = distributed.train_threads([_dev(X)], 0.06, 10, [comm],
                                            [distributed.NativeOps(torch.device("cuda", 0))],
                                            max_partitions=8)
            lab_o, core_o, _, _ = oracle.dbscan(X, 0.06, 10)
            np.testing.assert_array_equal(res[0].local_labels.cpu().numpy().astype(np.int64),
                                          lab_o)
            np.testing.assert_array_equal(res[0].local_core.cpu().numpy(), core_o)
        for name in ("b3d_20k", "b2d_20k", "c0_p5_cityblock", "dup_1d"):
            gd = load_golden(name)
            lab, core, _ = _cluster(native, gd["X"], float(gd["eps"]), int(gd["min_samples"]),
                                    _metric(gd))
            assert np.array_equal(lab, gd["sk_labels"]) and np.array_equal(core, gd["sk_core"])
    finally:
        ctx.set_option(native.PD_OPT_SWEEP_STATS, 0)


def test_retired_options_raise(native):
    """The tuning knobs retired in round 5 (their losing kernels are gone)
    are refused, not silently ignored."""
    ctx = native.context()
    for opt in native.PD_OPT_RETIRED:
        with pytest.raises(native.PardisError):
            ctx.set_option(opt, 1)


@pytest.mark.parametrize("key_bytes,bits,n", [
    (4, 32, 0), (4, 32, 1), (4, 8, 5), (4, 1, 8191), (4, 9, 8192), (4, 32, 8193),
    (4, 7, 1_000_003), (4, 32, 3_000_001), (8, 37, 1), (8, 37, 6145), (8, 64, 200_003),
    (8, 37, 2_000_000)])
def test_record_sort_is_stable_and_exact(native, key_bytes, bits, n):
    """The train's record sort (rsort.hpp, pd_sort_pairs) against numpy's
    stable argsort: tiles of 8192 / 6144 items, partial last tiles, one-pass
    and multi-pass key widths, heavy duplicate keys (stability), 64-bit keys."""
    rng = np.random.default_rng(n + bits)
    if key_bytes == 4:
        hi = (1 << bits) - 1
        if n % 2:   # 1024 distinct keys spread over the key range: long equal runs
            k = (rng.integers(0, 1024, n, dtype=np.uint64) * np.uint64(max(1, hi // 1023))) & np.uint64(hi)
        else:
            k = rng.integers(0, hi + 1, n, dtype=np.uint64)
        k = k.astype(np.uint32)
        kt = torch.from_numpy(k.view(np.int32)).cuda()
    else:
        k = rng.integers(0, 1 << min(bits, 63), n, dtype=np.uint64)
        if bits == 64:
            k |= (rng.integers(0, 2, n, dtype=np.uint64) << np.uint64(63))
        k[: n // 3] = k[0] if n else k[: n // 3]   # a run of equal keys
        kt = torch.from_numpy(k.view(np.int64)).cuda()
    v = np.arange(n, dtype=np.uint32)[::-1].copy()
    vt = torch.from_numpy(v.view(np.int32)).cuda()
    native.sort_pairs(kt, vt, bits)
    order = np.argsort(k, kind="stable")
    got_k = kt.cpu().numpy().view(np.uint32 if key_bytes == 4 else np.uint64)
    got_v = vt.cpu().numpy().view(np.uint32)
    assert np.array_equal(got_k, k[order])
    assert np.array_equal(got_v, v[order])


@pytest.mark.parametrize("key_bytes,bits", [(4, 20), (4, 13), (8, 37), (8, 3)])
def test_record_sort_ignores_bits_above_key_bits(native, key_bytes, bits):
    """pd_sort_pairs sorts by key bits [0, key_bits) only — keys
    with bits set above key_bits order as numpy's stable sort of the masked
    keys (equal masked keys keep their input order), not by the 8-bit digit's
    upper bits."""
    rng = np.random.default_rng(bits)
    n = 300_007
    dt = np.uint32 if key_bytes == 4 else np.uint64
    k = rng.integers(0, np.iinfo(np.int64).max, n, dtype=np.uint64).astype(dt)
    v = np.arange(n, dtype=np.uint32)
    kt = torch.from_numpy(k.view(np.int32 if key_bytes == 4 else np.int64)).cuda()
    vt = torch.from_numpy(v.view(np.int32)).cuda()
    native.sort_pairs(kt, vt, bits)
    order = np.argsort(k & dt((1 << bits) - 1), kind="stable")
    assert np.array_equal(kt.cpu().numpy().view(dt), k[order])
    assert np.array_equal(vt.cpu().numpy().view(np.uint32), v[order])


def test_record_sort_unaligned_keys(native):
    """pd_sort_pairs on a key view that is not 16-byte aligned (the digit
    histogram then reads key by key)."""
    rng = np.random.default_rng(5)
    n = 100_003
    k = rng.integers(0, 1 << 20, n + 1, dtype=np.uint64).astype(np.uint32)
    kt = torch.from_numpy(k.view(np.int32)).cuda()[1:]
    v = np.arange(n, dtype=np.uint32)
    vt = torch.from_numpy(v.view(np.int32)).cuda()
    assert kt.data_ptr() % 16 != 0
    native.sort_pairs(kt, vt, 20)
    order = np.argsort(k[1:], kind="stable")
    assert np.array_equal(kt.cpu().numpy().view(np.uint32), k[1:][order])
    assert np.array_equal(vt.cpu().numpy().view(np.uint32), v[order])


def test_fp64_input_exact(native):
    from pypardis_amd import synth
    X = synth.blobs_noise(40_000, 2, side=10.0, n_centers=5, sigma=0.3, seed=31).astype(np.float64)
    X += np.random.default_rng(0).uniform(-1e-9, 1e-9, X.shape)   # not fp32-representable
    lab_o, core_o, _, _ = oracle.dbscan(X, 0.05, 7)
    lab, core, _ = _cluster(native, X, 0.05, 7)
    assert np.array_equal(lab, lab_o) and np.array_equal(core, core_o)


def test_exact_ties_lattice(native):
    g = np.arange(60, dtype=np.float32) * np.float32(0.05)
    X = np.stack(np.meshgrid(g, g, indexing="ij"), -1).reshape(-1, 2)
    for eps in (float(np.float32(0.05)), 0.05, float(np.float32(0.05) * np.sqrt(2))):
        lab_o, core_o, cnt_o, _ = oracle.dbscan(X, eps, 5)
        lab, core, _, cnt = _cluster(native, X, eps, 5, full=True)
        assert np.array_equal(cnt, cnt_o), eps
        assert np.array_equal(lab, lab_o), eps


def test_edge_cases(native):
    from pypardis_amd import DBSCAN
    # all identical points, several partitions (A5)
    X = np.full((500, 3), 0.7, np.float32)
    m = DBSCAN(eps=0.1, min_samples=5, max_partitions=4).train(_dev(X))
    assert np.all(m.labels_.cpu().numpy() == 0)
    # min_samples = 1: every point is core
    X = np.random.default_rng(1).uniform(0, 100, (2000, 2)).astype(np.float32)
    lab_o, _, _, _ = oracle.dbscan(X, 0.5, 1)
    lab, core, _ = _cluster(native, X, 0.5, 1)
    assert np.array_equal(lab, lab_o) and core.all()
    # eps larger than the whole extent: one cell
    lab, core, ncl = _cluster(native, X, 1000.0, 3)
    assert ncl == 1 and np.all(lab == 0)
    # single point; all noise
    lab, core, ncl = _cluster(native, X[:1], 0.1, 2)
    assert ncl == 0 and lab[0] == -1
    # empty input
    lab, core, ncl = _cluster(native, np.zeros((0, 2), np.float32), 0.1, 2)
    assert ncl == 0 and len(lab) == 0
    # negative / huge offsets (grid clipped to the data, not the sentinel box)
    Y = (X - np.float32(1e6)).astype(np.float32)
    lab_o, _, _, _ = oracle.dbscan(Y, 0.5, 3)
    m = DBSCAN(eps=0.5, min_samples=3, max_partitions=4).train(_dev(Y))
    assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), lab_o)


def test_nan_rejected(native):
    from pypardis_amd import _native
    X = np.zeros((10, 2), np.float32)
    X[3, 1] = np.nan
    with pytest.raises(_native.PardisError):
        _native.cluster(_dev(X), 0.1, 2)
    from pypardis_amd import DBSCAN
    with pytest.raises(ValueError):
        DBSCAN(eps=0.1, min_samples=2).train(_dev(X))


def test_partition_count_invariance_large(native):
    """Size-independent property at 4M 3-D points: labels do not depend on
    max_partitions (the halo + merge reproduce the one-partition answer)."""
    from pypardis_amd import DBSCAN, synth
    X, cfg = synth.make_config("C2", n=4_000_000)
    Xd = _dev(X)
    ref, core1, _, nc1 = native.cluster(Xd, cfg["eps"], cfg["min_samples"])
    for P in (2, 8, 13):
        m = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=P).train(Xd)
        assert m.n_clusters_ == nc1
        assert torch.equal(m.labels_, ref), P
        assert torch.equal(m.core_sample_mask_, core1), P
    # sklearn numbering: cluster ids appear in order of their smallest core index
    lab = ref.cpu().numpy()
    c = core1.cpu().numpy().astype(bool)
    idx = np.nonzero(c)[0]
    first = np.full(nc1, -1)
    seen = np.zeros(nc1, bool)
    u, fi = np.unique(lab[idx], return_index=True)
    first[u] = idx[fi]
    assert np.all(np.diff(first) > 0)


def test_fp32_screen_is_exact(native):
    """The fp32 screen only decides pairs outside a 2^-18 band around eps; the
    result must be identical with the screen disabled (exact fp64 for every
    pair), including on exact ties."""
    from pypardis_amd import synth
    g = np.arange(80, dtype=np.float32) * np.float32(0.05)
    lattice = np.stack(np.meshgrid(g, g, indexing="ij"), -1).reshape(-1, 2)
    blobs = synth.blobs_noise(60_000, 3, side=6.0, n_centers=5, sigma=0.4, seed=41)
    ctx = native.context()
    for X, eps, ms in ((lattice, float(np.float32(0.05)), 5), (lattice, 0.05, 5),
                       (blobs, 0.07, 8)):
        out = []
        for screen in (1, 0):
            ctx.set_option(native.PD_OPT_FP32_SCREEN, screen)
            try:
                out.append(_cluster(native, X, eps, ms, full=True))
            finally:
                ctx.set_option(native.PD_OPT_FP32_SCREEN, 1)
        (l1, c1, n1, k1), (l0, c0, n0, k0) = out
        assert np.array_equal(k1, k0) and np.array_equal(l1, l0) and n1 == n0


# ------------------------------------------------------------ sharded train
def test_sharded_stage_primitives(native):
    """pd_kd_moments_dd / pd_route / pd_pack / pd_merge_exports /
    pd_select_roots / pd_sort_u32 / pd_rank_labels against numpy and the
    oracle restatement (oracle/sharded.py)."""
    from oracle import sharded as osh
    from pypardis_amd import synth
    from pypardis_amd.distributed import dd_combine, partition_ranks
    rng = np.random.default_rng(5)
    X = synth.blobs_noise(50_000, 3, side=5.0, n_centers=4, sigma=0.5, seed=51)
    Xd = _dev(X)
    lab = torch.from_numpy(rng.integers(0, 5, len(X)).astype(np.int32)).cuda()
    dd = native.kd_moments_dd(Xd, lab, [0, 2, 4])
    mom = native.kd_moments(Xd, lab, [0, 2, 4])
    np.testing.assert_array_equal(dd_combine(dd[None]), mom)
    # route: 5 boxes over 3 ranks
    lo, hi = X.min(0).astype(np.float64), X.max(0).astype(np.float64)
    cuts = np.linspace(lo[0], hi[0], 6)
    ebox = np.stack([np.stack([np.r_[cuts[i] - 0.1, lo[1:]], np.r_[cuts[i + 1] + 0.1, hi[1:]]])
                     for i in range(5)])
    pr, li = partition_ranks(5, 3)
    mask, counts = native.route(Xd, ebox, pr, 3)
    x64 = X.astype(np.float64)
    want = np.zeros(len(X), np.int64)
    for L in range(5):
        m = np.all(ebox[L, 0] <= x64, 1) & np.all(ebox[L, 1] >= x64, 1)
        want[m] |= 1 << int(pr[L])
    np.testing.assert_array_equal(mask.cpu().numpy(), want)
    assert counts.tolist() == [int(((want >> r) & 1).sum()) for r in range(3)]
    kdlab = torch.from_numpy(rng.integers(0, 5, len(X)).astype(np.int32)).cuda()
    for dest in range(3):
        c = int(counts[dest])
        out = (torch.empty((c, 3), dtype=Xd.dtype, device="cuda"),
               torch.empty(c, dtype=torch.int32, device="cuda"),
               torch.empty(c, dtype=torch.int32, device="cuda"),
               torch.empty(c, dtype=torch.uint8, device="cuda"))
        m = native.pack(Xd, mask, dest, kdlab, pr, li, 1000, out)
        assert m == c
        idx = np.nonzero((want >> dest) & 1)[0]
        kl = kdlab.cpu().numpy()[idx]
        np.testing.assert_array_equal(out[0].cpu().numpy(), X[idx])
        np.testing.assert_array_equal(out[1].cpu().numpy(), idx + 1000)
        np.testing.assert_array_equal(out[2].cpu().numpy(), np.where(pr[kl] == dest, li[kl], -1))
        many = np.array([bin(v).count("1") > 1 for v in want[idx]])
        np.testing.assert_array_equal(out[3].cpu().numpy().astype(bool), many)
    # merge: random pairs over a sparse id space (ids up to 2^32 - 2)
    pool = rng.choice(0xFFFFFFFE, 8000, replace=False)
    ga = pool[rng.integers(0, len(pool), 5000)]
    gb = pool[rng.integers(0, len(pool), 5000)]
    as_i32 = (lambda a: torch.from_numpy(a.astype(np.uint32).view(np.int32)).cuda())
    ids, mk = native.merge_exports(as_i32(ga), as_i32(gb))
    wids, wkeys = osh.merge(ga, gb)
    np.testing.assert_array_equal(ids.cpu().numpy().view(np.uint32), wids)
    np.testing.assert_array_equal(mk.cpu().numpy().view(np.uint32), wkeys)
    e = native.merge_exports(as_i32(ga[:0]), as_i32(gb[:0]))
    assert e[0].shape[0] == 0
    # roots / sort / ranks
    gid = np.sort(rng.choice(1 << 30, 30_000, replace=False)).astype(np.int64)
    keys = np.where(rng.random(len(gid)) < 0.3, -1, gid[rng.integers(0, len(gid), len(gid))])
    keys[::7] = gid[::7]
    kd_, gd_ = (torch.from_numpy(keys.astype(np.int32)).cuda(),
                torch.from_numpy(gid.astype(np.int32)).cuda())
    roots = native.select_roots(kd_, gd_).cpu().numpy().astype(np.int64)
    np.testing.assert_array_equal(roots, gid[(keys >= 0) & (keys == gid)])
    shuf = torch.from_numpy(rng.permutation(roots).astype(np.int32)).cuda()
    native.sort_u32(shuf)
    np.testing.assert_array_equal(shuf.cpu().numpy(), np.sort(roots))
    ok = (keys < 0) | np.isin(keys, roots)
    kd_ok = torch.from_numpy(np.where(ok, keys, -1).astype(np.int32)).cuda()
    labs = native.rank_labels(kd_ok, shuf).cpu().numpy()
    m = (keys >= 0) & ok
    np.testing.assert_array_equal(labs[m], np.searchsorted(roots, keys[m]))
    assert (labs[~m] == -1).all()
    # a key with no root (roots not gathered from every device) is an error
    with pytest.raises(native.PardisError, match="no root"):
        native.rank_labels(kd_, shuf)
    # results back to the holders: owned records, grouped by holding rank
    n = 40_000
    owner = torch.from_numpy(np.where(rng.random(n) < 0.6, 0, -1).astype(np.int32)).cuda()
    g2 = np.sort(rng.choice(100_000, n, replace=False)).astype(np.int64)
    lab2 = rng.integers(-1, 1000, n).astype(np.int32)
    core2 = (rng.random(n) < 0.5).astype(np.uint8)
    offs = np.array([0, 30_000, 70_000, 100_000], np.int64)
    pairs, cnt = native.owned_results(owner, torch.from_numpy(g2.astype(np.int32)).cuda(),
                                      torch.from_numpy(lab2).cuda(),
                                      torch.from_numpy(core2).cuda(), offs)
    own = owner.cpu().numpy() >= 0
    p = pairs.cpu().numpy().view(np.uint32).astype(np.int64)
    np.testing.assert_array_equal(p[:, 0], g2[own])
    np.testing.assert_array_equal((p[:, 1] & 0x7FFFFFFF) - 1, lab2[own])
    np.testing.assert_array_equal(p[:, 1] >> 31, core2[own])
    assert cnt.tolist() == np.diff(np.searchsorted(g2[own], offs)).tolist()
    # scatter: a full permutation of one holder's slice
    base, nloc = 1000, 5000
    perm = rng.permutation(nloc)
    lab3 = rng.integers(-1, 50, nloc).astype(np.int64)
    pr3 = np.stack([perm + base, ((lab3[perm] + 1) | (perm % 2) << 31)], 1)
    pt = torch.from_numpy(pr3.astype(np.uint32).view(np.int32)).cuda()
    l3, c3 = native.scatter_results(pt, base, nloc, torch.device("cuda", 0))
    np.testing.assert_array_equal(l3.cpu().numpy(), lab3)
    np.testing.assert_array_equal(c3.cpu().numpy(), np.arange(nloc) % 2)
    with pytest.raises(native.PardisError, match="no result"):
        dup = pt.clone()
        dup[1] = dup[0]
        native.scatter_results(dup, base, nloc, torch.device("cuda", 0))


SHARDED = [("b3d_20k", 2, 8), ("c0", 3, 4), ("c0_p5_cityblock", 2, 5), ("dup_1d", 2, 3)]


@pytest.mark.parametrize("name,world,P", SHARDED)
def test_sharded_native_equals_sklearn(native, tmp_path, name, world, P):
    """Two/three gloo ranks sharing cuda:0, every device stage native."""
    from dist_worker import run_world
    g = load_golden(name)
    X = g["X"] if g["X"].ndim == 2 else g["X"][:, None]
    mcode = native.metric_code(_metric(g))
    out = run_world(world, X, float(g["eps"]), int(g["min_samples"]), mcode, P, str(tmp_path),
                    native=True)
    assert (out["seen"] == 1).all()
    np.testing.assert_array_equal(out["labels"], g["sk_labels"])
    np.testing.assert_array_equal(out["core"], g["sk_core"].astype(np.uint8))
    np.testing.assert_array_equal(out["loc_labels"], g["sk_labels"])
    np.testing.assert_array_equal(out["loc_core"], g["sk_core"].astype(np.uint8))


@pytest.mark.parametrize("name,world,P,keyed", [("b3d_20k", 2, 8, False), ("c0", 3, 4, True)])
def test_reference_api_process_group_native(native, tmp_path, name, world, P, keyed):
    """dbscan.DBSCAN(...).train(slice) in a gloo process group, every device
    stage native on cuda:0: input-order labels on every rank, the global
    cluster count, and assignments() over all ranks."""
    from dist_worker import run_world
    g = load_golden(name)
    X = g["X"]
    out = run_world(world, X, float(g["eps"]), int(g["min_samples"]), 0, P, str(tmp_path),
                    native=True, api=True, keyed=keyed)
    np.testing.assert_array_equal(out["loc_labels"], g["sk_labels"])
    np.testing.assert_array_equal(out["loc_core"], g["sk_core"].astype(np.uint8))
    for z in out["ranks"]:
        assert int(z["n_clusters_"]) == int(g["sk_labels"].max()) + 1
        np.testing.assert_array_equal(z["assign_labels"], g["sk_labels"])
        assert int(z["count"]) == len(X)


def test_rccl_comm_single_rank(native):
    """pd_comm_* through RCCL on one device (a 1-rank communicator: this box
    has one GPU): the collectives' data movement, then the whole sharded
    train on RcclComm (threaded runner, pd_comm_init_all) against pd_cluster."""
    from pypardis_amd import distributed, synth
    comm = distributed.device_comms([0])[0]
    t = torch.arange(10, dtype=torch.float64, device="cuda")
    assert comm.all_reduce(t.cpu().numpy(), "max").tolist() == list(range(10))
    v = torch.arange(7, dtype=torch.int32, device="cuda")
    assert comm.all_gather_var(v).cpu().tolist() == list(range(7))
    w = torch.arange(12, dtype=torch.int64, device="cuda").reshape(6, 2)
    np.testing.assert_array_equal(comm.all_to_all_v(w, [6], [6]).cpu().numpy(),
                                  w.cpu().numpy())
    np.testing.assert_array_equal(comm.all_gather_np(np.array([3, 4])), [[3, 4]])
    # the W > 1 init check's pattern, fill and verify kernels (at W = 1 the
    # self blocks carry it), the grouped field exchange and the device gather
    comm.comm.self_check()
    assert comm.comm.size() == (1, 0)       # as RCCL reports it (bench.py's rccl_ranks)
    a = torch.arange(15, dtype=torch.float32, device="cuda").reshape(5, 3)
    b = torch.arange(5, dtype=torch.int32, device="cuda")
    ra, rb = torch.empty_like(a), torch.empty_like(b)
    comm.exchange([a, b], [ra, rb], [5], [5], skip_self=False)
    assert torch.equal(ra, a) and torch.equal(rb, b)
    assert torch.equal(comm.all_gather_t(b), b[None])
    X, cfg = synth.make_config("C2", n=300_000)
    Xd = _dev(X)
    lab1, core1, _, nc1 = native.cluster(Xd, cfg["eps"], cfg["min_samples"])
    res = distributed.train_threads([Xd], cfg["eps"], cfg["min_samples"], [comm],
                                    [distributed.NativeOps(torch.device("cuda", 0))],
                                    max_partitions=8)
    assert res[0].n_clusters == nc1
    np.testing.assert_array_equal(res[0].local_labels.cpu().numpy(), lab1.cpu().numpy())
    np.testing.assert_array_equal(res[0].local_core.cpu().numpy(), core1.cpu().numpy())


def test_sharded_unaligned_view_and_wide_schedule(native):
    """a slice that is a view at a 12-byte offset (fp32 3-D
    X_full[1:]) and max_partitions = 1000 (KD levels wider than the device
    tables: the host-decided KD) both train on a 1-rank RCCL communicator and
    equal pd_cluster."""
    from pypardis_amd import distributed, synth
    comm = distributed.device_comms([0])[0]
    X, cfg = synth.make_config("C2", n=200_001)
    Xfull = _dev(X)
    view = Xfull[1:]
    assert view.data_ptr() % 16 != 0
    want, core_w, _, nc = native.cluster(view.contiguous(), cfg["eps"], cfg["min_samples"])
    for P in (8, 1000):
        res = distributed.train_threads([view], cfg["eps"], cfg["min_samples"], [comm],
                                        [distributed.NativeOps(torch.device("cuda", 0))],
                                        max_partitions=P)
        assert res[0].n_clusters == nc, P
        np.testing.assert_array_equal(res[0].local_labels.cpu().numpy(), want.cpu().numpy())
        np.testing.assert_array_equal(res[0].local_core.cpu().numpy(), core_w.cpu().numpy())


def test_rccl_process_group_single_rank(native, tmp_path):
    """A 1-rank "nccl" process group: the RCCL id is handed over through
    torch.distributed and DBSCAN(...).train runs the sharded path on
    pd_comm (forced with group=)."""
    from dist_worker import run_rccl_world1
    from pypardis_amd import synth
    X, cfg = synth.make_config("C2", n=200_000)
    lab1, _, _, nc1 = native.cluster(_dev(X), cfg["eps"], cfg["min_samples"])
    got = run_rccl_world1(X, cfg["eps"], cfg["min_samples"], 8, str(tmp_path))
    assert got["n_clusters"] == nc1
    np.testing.assert_array_equal(got["labels"], lab1.cpu().numpy())


def test_sharded_native_large(native, tmp_path):
    """400k 3-D C2-density points, 2 ranks x 4 neighbourhoods each: labels
    equal the single-device pd_cluster answer."""
    from dist_worker import run_world
    from pypardis_amd import synth
    X, cfg = synth.make_config("C2", n=400_000)
    lab1, core1, _, nc1 = native.cluster(_dev(X), cfg["eps"], cfg["min_samples"])
    out = run_world(2, X, cfg["eps"], cfg["min_samples"], 0, 8, str(tmp_path), native=True)
    assert (out["seen"] == 1).all()
    assert out["ncl"] == {nc1}
    assert out["exports"] > 0
    np.testing.assert_array_equal(out["loc_labels"], lab1.cpu().numpy().astype(np.int64))
    np.testing.assert_array_equal(out["labels"], lab1.cpu().numpy().astype(np.int64))
    np.testing.assert_array_equal(out["core"], core1.cpu().numpy())


# ------------------------------------------------------------ dense (d > 4) path
DENSE = [
    # (name, X builder, eps, min_samples, metric, max_partitions)
    ("c3_30k", lambda: __import__("pypardis_amd.synth").synth.make_config("C3", n=30_000)[0],
     0.114028, 10, "euclidean", 1),
    ("c3_wide_eps", lambda: __import__("pypardis_amd.synth").synth.make_config("C3", n=8_000)[0],
     0.9, 25, "euclidean", 3),
    ("d5_blobs", lambda: __import__("pypardis_amd.synth").synth.blobs_noise(
        20_000, 5, side=6.0, n_centers=8, sigma=0.4, seed=71), 0.3, 8, "euclidean", 1),
    ("d100_f64", lambda: __import__("pypardis_amd.synth").synth.blobs_noise(
        6_000, 100, side=4.0, n_centers=6, sigma=0.15, seed=72).astype(np.float64) + 1e3,
     1.6, 5, "euclidean", 1),
    ("d200_brute", lambda: __import__("pypardis_amd.synth").synth.blobs_noise(
        3_000, 200, side=3.0, n_centers=4, sigma=0.1, seed=73), 2.0, 5, "euclidean", 1),
    ("d8_cityblock", lambda: __import__("pypardis_amd.synth").synth.blobs_noise(
        8_000, 8, side=5.0, n_centers=6, sigma=0.3, seed=74), 1.2, 6, "cityblock", 1),
]


@pytest.mark.parametrize("case", DENSE, ids=[c[0] for c in DENSE])
def test_dense_path_matches_oracle(native, case):
    """d > 4: split-bf16 MFMA Gram tiles with the exact fp64 band recheck (or
    the exact VALU tile for cityblock / d > 128): neighbour counts, core flags
    and labels bit-identical to the oracle (sklearn kd_tree semantics)."""
    from pypardis_amd import DBSCAN
    _, build, eps, ms, metric, P = case
    X = np.ascontiguousarray(build())
    lab_o, core_o, cnt_o, nc_o = oracle.dbscan(X, eps, ms, metric)
    lab, core, ncl, cnt = _cluster(native, X, eps, ms, metric, full=True)
    assert np.array_equal(cnt, cnt_o)
    assert np.array_equal(core, core_o)
    assert np.array_equal(lab, lab_o) and ncl == nc_o
    m = DBSCAN(eps=eps, min_samples=ms, metric=metric, max_partitions=P).train(_dev(X))
    assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), lab_o)
    assert 0 < int(core_o.sum()) < len(X)   # the case exercises core, border and noise


def test_dense_exact_ties(native):
    """A 6-D fp32 lattice with eps equal to the spacing: every axis neighbour
    is an exact tie (inside the MFMA error band), decided by the fp64 recheck."""
    g = np.arange(6, dtype=np.float32) * np.float32(0.05)
    X = np.stack(np.meshgrid(*([g] * 6), indexing="ij"), -1).reshape(-1, 6).astype(np.float32)
    for eps in (float(np.float32(0.05)), 0.05):
        lab_o, core_o, cnt_o, _ = oracle.dbscan(X, eps, 7)
        lab, core, _, cnt = _cluster(native, X, eps, 7, full=True)
        assert np.array_equal(cnt, cnt_o), eps
        assert np.array_equal(lab, lab_o), eps


@pytest.mark.parametrize("n,eps", [(1_000_000, 0.114028), (300_000, 0.3), (60_000, 0.02)])
def test_dense_prune_full_size(native, n, eps):
    """Projection pruning of the count pass is exact: at C3's full size (and
    with wide / tiny windows over many bands) the pruned and the all-pairs
    runs give identical counts, core flags and labels — a size-independent
    property where the CPU oracle is too slow to run."""
    from pypardis_amd import synth
    X = synth.make_config("C3", n=n)[0]
    ctx = native.context()
    lab0, core0, ncl0, cnt0 = _cluster(native, X, eps, 10, full=True)
    for mode in (0, 2):   # all pairs; per-band runs (the segment-overflow path)
        ctx.set_option(native.PD_OPT_DENSE_PRUNE, mode)
        try:
            lab1, core1, ncl1, cnt1 = _cluster(native, X, eps, 10, full=True)
        finally:
            ctx.set_option(native.PD_OPT_DENSE_PRUNE, 1)
        assert np.array_equal(cnt0, cnt1), mode
        assert np.array_equal(core0, core1), mode
        assert np.array_equal(lab0, lab1) and ncl0 == ncl1, mode
    if eps > 0.1:   # the tiny window has no core points, only counts
        assert int(core0.sum()) > 0


def _subnormal_heavy():
    """16-D points whose coordinates mostly fall in e4m3's subnormal range
    after scaling (a few far outliers set the scale), with pairs near eps."""
    rng = np.random.default_rng(77)
    X = rng.normal(scale=1e-5, size=(6000, 16)).astype(np.float32)
    X[:3000] += np.float32(3e-5)
    X[-4:] = np.sign(rng.normal(size=(4, 16))).astype(np.float32)   # scale ~ 1
    return X


@pytest.mark.parametrize("case", ["c3_30k", "d5_blobs", "d100_f64", "subnormal", "ties", "c3_1m"])
def test_dense_screens_equal(native, case):
    """The count pass's e4m3 screen (PD_OPT_DENSE_SCREEN = 1, default) and the
    bf16 hi.hi screen decide the same counts: bit-identical counts, core flags
    and labels, and the oracle's where it runs (the e4m3 rounding bound is
    checked here on coordinates in e4m3's subnormal range and on exact ties)."""
    from pypardis_amd import synth
    if case == "subnormal":
        X, eps, ms = _subnormal_heavy(), 3e-5, 6
    elif case == "ties":
        g = np.arange(6, dtype=np.float32) * np.float32(0.05)
        X = np.stack(np.meshgrid(*([g] * 6), indexing="ij"), -1).reshape(-1, 6).astype(np.float32)
        eps, ms = float(np.float32(0.05)), 7
    elif case == "c3_1m":
        X, eps, ms = synth.make_config("C3", n=1_000_000)[0], 0.114028, 10
    else:
        c = next(c for c in DENSE if c[0] == case)
        X, eps, ms = np.ascontiguousarray(c[1]()), c[2], c[3]
    ctx = native.context()
    outs = []
    for screen in (1, 0):
        ctx.set_option(native.PD_OPT_DENSE_SCREEN, screen)
        try:
            outs.append(_cluster(native, X, eps, ms, full=True))
        finally:
            ctx.set_option(native.PD_OPT_DENSE_SCREEN, 1)
    (lab1, core1, ncl1, cnt1), (lab0, core0, ncl0, cnt0) = outs
    assert np.array_equal(cnt1, cnt0)
    assert np.array_equal(core1, core0)
    assert np.array_equal(lab1, lab0) and ncl1 == ncl0
    if len(X) <= 60_000:
        lab_o, core_o, cnt_o, nc_o = oracle.dbscan(X, eps, ms)
        assert np.array_equal(cnt1, cnt_o)
        assert np.array_equal(lab1, lab_o) and ncl1 == nc_o
    if case == "subnormal":
        assert 0 < int(core1.sum()) < len(X)


def test_dense_edge_cases(native):
    from pypardis_amd import DBSCAN
    X = np.full((300, 16), 0.25, np.float32)   # identical points
    m = DBSCAN(eps=0.1, min_samples=5, max_partitions=2).train(_dev(X))
    assert np.all(m.labels_.cpu().numpy() == 0)
    rng = np.random.default_rng(3)
    X = rng.normal(size=(700, 12)).astype(np.float32)
    for ms in (1, 2):
        lab_o, _, _, _ = oracle.dbscan(X, 2.5, ms)
        lab, _, _ = _cluster(native, X, 2.5, ms)
        assert np.array_equal(lab, lab_o), ms
    lab, core, ncl = _cluster(native, X[:1], 0.5, 2)
    assert ncl == 0 and lab[0] == -1
    lab, core, ncl = _cluster(native, np.zeros((0, 12), np.float32), 0.5, 2)
    assert ncl == 0 and len(lab) == 0


# ------------------------------------------------------------ C4: GPS-like skew
@pytest.mark.parametrize("case", ["sample_200k", "dense_tile_100k"])
def test_c4_skew_vs_oracle(native, case):
    """C4 (SURVEY.md §8(d), 2-D GPS-like Zipf skew, eps=0.001°, min_samples=20):
    a 200k sample of the 1B distribution (10k cities over the globe; mostly
    sparse), and a dense tile (40 cities in 2°x1°, sigma0=0.002°: ~1000 points
    per eps-cell at the densest city) — labels and core flags bit-exact
    against the oracle at max_partitions=8 and 1."""
    from pypardis_amd import DBSCAN, synth
    if case == "sample_200k":
        X, cfg = synth.make_config("C4", n=200_000)
    else:
        cfg = dict(synth.CONFIGS["C4"])
        X = synth.gps_skew(100_000, seed=6, n_cities=40, sigma0=0.002, lon=(-1.0, 1.0),
                           lat=(-0.5, 0.5)).numpy()
    eps, ms = cfg["eps"], cfg["min_samples"]
    want, core_w, _, nc = oracle.dbscan(X, eps, ms)
    Xd = _dev(X)
    for P in (8, 1):
        m = DBSCAN(eps=eps, min_samples=ms, max_partitions=P).train(Xd)
        assert m.n_clusters_ == nc, P
        assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), want), P
        assert np.array_equal(m.core_sample_mask_.cpu().numpy(), core_w), P
    # dense-cell tuning knobs change the work order, never the answer:
    # rotated count starts on every long list / never; window union of 2 /
    # 4 / 16 / 64 records
    ctx = native.context()
    CW = -1
    for opts in (((native.PD_OPT_COUNT_ROTATE, 16, 1024),),
                 ((native.PD_OPT_COUNT_ROTATE, 0, 1024),),
                 ((native.PD_OPT_CENTRE_WINDOW, 64, CW),),
                 ((native.PD_OPT_CENTRE_WINDOW, 16, CW),),
                 ((native.PD_OPT_CENTRE_WINDOW, 2, CW),),
                 ((native.PD_OPT_CENTRE_WINDOW, 4, CW),)):
        for opt, val, _ in opts:
            ctx.set_option(opt, val)
        try:
            m = DBSCAN(eps=eps, min_samples=ms, max_partitions=8).train(Xd)
        finally:
            for opt, _, default in opts:
                ctx.set_option(opt, default)
        opt, val = opts[-1][0], opts[-1][1]
        assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), want), (opt, val)
        assert np.array_equal(m.core_sample_mask_.cpu().numpy(), core_w), (opt, val)


def test_c4_partition_invariance_large(native):
    """Size-independent property on a 20M C4 sample (skewed density, up to
    ~1000 points per eps-cell): labels and core flags do not depend on
    max_partitions, and clusters are numbered in sklearn's order."""
    from pypardis_amd import DBSCAN, synth
    cfg = synth.CONFIGS["C4"]
    Xd = synth.gps_skew(20_000_000, seed=cfg["seed"], device="cuda")
    eps, ms = cfg["eps"], cfg["min_samples"]
    ref = DBSCAN(eps=eps, min_samples=ms, max_partitions=1).train(Xd)
    m = DBSCAN(eps=eps, min_samples=ms, max_partitions=8).train(Xd)
    assert m.n_clusters_ == ref.n_clusters_
    assert torch.equal(m.labels_, ref.labels_)
    assert torch.equal(m.core_sample_mask_, ref.core_sample_mask_)
    lab = ref.labels_.cpu().numpy()
    idx = np.nonzero(ref.core_sample_mask_.cpu().numpy())[0]
    u, fi = np.unique(lab[idx], return_index=True)
    assert np.array_equal(u, np.arange(ref.n_clusters_))
    assert np.all(np.diff(idx[fi]) > 0)


# ------------------------------------------------------------ sharded dense (d > 4)
def _dense_stages(native, Xd, eps, ms, metric, W, full=False):
    """W ranks simulated in one process: one context each on cuda:0, the
    collectives done by hand (sum of counts, concatenation of the forests,
    min of the border keys) — pd_dense_* exactly as distributed._train_dense
    drives them."""
    lo = Xd.min(0).values.double().cpu().numpy()
    hi = Xd.max(0).values.double().cpu().numpy()
    dbox = np.stack([lo, hi])
    ctxs = [native.Context(0) for _ in range(W)]
    for c in ctxs:
        c.set_option(native.PD_OPT_FULL_COUNTS, int(full))
    parts = [native.dense_count(Xd, eps, ms, metric, dbox, r, W, ctx=ctxs[r]) for r in range(W)]
    cnt = torch.stack(parts).sum(0).to(torch.int32)
    forests = torch.cat([native.dense_link(cnt, ctx=c) for c in ctxs])
    n = Xd.shape[0]
    best = torch.stack([native.dense_border(forests, W, n, ctx=c) for c in ctxs]).min(0).values \
        if n else torch.empty(0, dtype=torch.int32, device=Xd.device)
    outs = [native.dense_finish(best, n, Xd.device, want_counts=full, ctx=c) for c in ctxs]
    for o in outs[1:]:   # every rank ends with the same answer
        assert torch.equal(o[0], outs[0][0]) and o[3] == outs[0][3]
    return outs[0], parts


DENSE_SHARD = [("c3_60k", 4, "euclidean"), ("c3_60k", 8, "euclidean"), ("d5_blobs", 3, "euclidean"),
               ("d8_cityblock", 2, "cityblock"), ("d100_f64", 3, "euclidean")]


@pytest.mark.parametrize("name,W,metric", DENSE_SHARD, ids=[f"{c[0]}-w{c[1]}" for c in DENSE_SHARD])
def test_dense_sharded_stages_match_oracle(native, name, W, metric):
    """The sharded dense stages over W simulated ranks give the oracle's
    counts, core flags and labels; each rank's count share is non-trivial."""
    from pypardis_amd import synth
    if name == "c3_60k":
        X, eps, ms = synth.make_config("C3", n=60_000)[0], 0.114028, 10
    else:
        case = {c[0]: c for c in DENSE}[name]
        X, eps, ms = np.ascontiguousarray(case[1]()), case[2], case[3]
    (lab, core, cnt, ncl), parts = _dense_stages(native, _dev(X), eps, ms,
                                                 native.metric_code(metric), W, full=True)
    lab_o, core_o, cnt_o, nc_o = oracle.dbscan(X, eps, ms, metric)
    assert np.array_equal(cnt.cpu().numpy().astype(np.int64), cnt_o)
    assert np.array_equal(lab.cpu().numpy().astype(np.int64), lab_o) and ncl == nc_o
    assert np.array_equal(core.cpu().numpy(), core_o)
    if len(X) >= 2048 * W:
        for p in parts:   # every rank computed some rows, and only its own
            assert int((p > 0).sum()) > 0


def test_dense_sharded_single_rank_equals_cluster(native):
    """Rank 0 of 1 through pd_dense_* equals pd_cluster; edge cases: no core
    point, one point, empty input."""
    from pypardis_amd import synth
    X = synth.make_config("C3", n=20_000)[0]
    Xd = _dev(X)
    lab1, core1, _, nc1 = native.cluster(Xd, 0.114028, 10)
    (lab, core, _, ncl), _ = _dense_stages(native, Xd, 0.114028, 10, 0, 1)
    assert torch.equal(lab, lab1) and torch.equal(core, core1) and ncl == nc1
    (lab, _, _, ncl), _ = _dense_stages(native, Xd, 1e-6, 10, 0, 3)    # nothing core
    assert ncl == 0 and int((lab != -1).sum()) == 0
    (lab, _, _, ncl), _ = _dense_stages(native, Xd[:1].contiguous(), 0.5, 1, 0, 2)
    assert ncl == 1 and lab.tolist() == [0]


def test_dense_sharded_process_group_native(native, tmp_path):
    """dbscan.DBSCAN(...).train(slice) with 64-D points in a gloo group of 3
    ranks sharing cuda:0: labels equal the single-device dense path."""
    from dist_worker import run_world
    from pypardis_amd import synth
    X = synth.make_config("C3", n=40_000)[0]
    lab1, core1, _, nc1 = native.cluster(_dev(X), 0.114028, 10)
    out = run_world(3, X, 0.114028, 10, 0, 4, str(tmp_path), native=True, api=True)
    np.testing.assert_array_equal(out["loc_labels"], lab1.cpu().numpy().astype(np.int64))
    np.testing.assert_array_equal(out["loc_core"], core1.cpu().numpy())
    for z in out["ranks"]:
        assert int(z["n_clusters_"]) == nc1


# ------------------------------------------------------------ directory budget
@pytest.mark.parametrize("name,budget", [("b2d_20k", 4096), ("b3d_20k", 4096), ("c0", 32),
                                         ("lattice_900", 32), ("c0_p5_cityblock", 32)])
def test_grid_growth_is_exact(native, name, budget):
    """Cells wider than eps (the directory budget forces them to grow) give
    sklearn's counts, core flags and labels — through pd_cluster and through
    the partitioned train (halo, merge, border).  The flat directory is
    forced: the paged one's budget only bounds its extent-dependent pages,
    which these small grids never fill."""
    from pypardis_amd import DBSCAN
    g = load_golden(name)
    ctx = native.context()
    ctx.set_option(native.PD_OPT_DIR_BUDGET, budget)
    ctx.set_option(native.PD_OPT_DIR_PAGED, 0)
    try:
        lab, core, ncl, cnt = _cluster(native, g["X"], float(g["eps"]), int(g["min_samples"]),
                                       _metric(g), full=True)
        grow = ctx.timings()["grid_grow"]
        P = int(g["max_partitions"])
        m = DBSCAN(eps=float(g["eps"]), min_samples=int(g["min_samples"]), metric=_metric(g),
                   max_partitions=P if P > 0 else None).train(_dev(g["X"]))
    finally:
        ctx.set_option(native.PD_OPT_DIR_BUDGET, 32 << 30)
        ctx.set_option(native.PD_OPT_DIR_PAGED, -1)
    assert grow > 1.5, grow
    assert np.array_equal(cnt, g["sk_counts"])
    assert np.array_equal(core, g["sk_core"])
    assert np.array_equal(lab, g["sk_labels"]) and ncl == int(g["sk_labels"].max()) + 1
    assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), g["sk_labels"])


@pytest.mark.parametrize("name", ["b2d_20k", "b3d_20k", "c0", "lattice_900", "c0_p5_cityblock",
                                  "neg_3k", "dup_1d", "c0_p3"])
def test_dir_layouts_equal(native, name):
    """The paged directory (occupied words only) and the flat one give
    sklearn's counts, core flags and labels on the goldens — pd_cluster and
    the partitioned train — with both layouts forced."""
    from pypardis_amd import DBSCAN
    g = load_golden(name)
    ctx = native.context()
    P = int(g["max_partitions"])
    for layout in (1, 0):
        ctx.set_option(native.PD_OPT_DIR_PAGED, layout)
        try:
            lab, core, ncl, cnt = _cluster(native, g["X"], float(g["eps"]),
                                           int(g["min_samples"]), _metric(g), full=True)
            t = ctx.timings()
            m = DBSCAN(eps=float(g["eps"]), min_samples=int(g["min_samples"]), metric=_metric(g),
                       max_partitions=P if P > 0 else None).train(_dev(g["X"]))
        finally:
            ctx.set_option(native.PD_OPT_DIR_PAGED, -1)
        assert t["dir_paged"] == layout
        assert np.array_equal(cnt, g["sk_counts"])
        assert np.array_equal(core, g["sk_core"])
        assert np.array_equal(lab, g["sk_labels"]) and ncl == int(g["sk_labels"].max()) + 1
        assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), g["sk_labels"])


@pytest.mark.parametrize("cfg,n", [("C4", 4_000_000), ("C2", 1_000_000), ("C1", 300_000)])
def test_dir_paged_equals_flat_synth(native, cfg, n):
    """Paged == flat directory on the bench distributions (C4's globe-wide
    noise and dense cities: words spanning waves, empty pages between
    occupied ones), labels and core flags bit-identical, and the oracle's on
    a 300k C4 sample with the paged layout."""
    from pypardis_amd import DBSCAN, synth
    X, c = synth.make_config(cfg, n=n, device="cuda" if cfg == "C4" else "cpu")
    Xd = X if torch.is_tensor(X) else _dev(X)
    ctx = native.context()
    outs = []
    for layout in (1, 0):
        ctx.set_option(native.PD_OPT_DIR_PAGED, layout)
        try:
            m = DBSCAN(eps=c["eps"], min_samples=c["min_samples"],
                       max_partitions=c.get("max_partitions") or 1).train(Xd)
            words = ctx.timings()["dir_words"]
        finally:
            ctx.set_option(native.PD_OPT_DIR_PAGED, -1)
        outs.append((m.labels_.clone(), m.core_sample_mask_.clone(), m.n_clusters_, words))
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0]) and torch.equal(outs[0][1], o[1])
        assert outs[0][2] == o[2]
    assert outs[0][3] <= outs[1][3]   # occupied words only
    if cfg == "C4":
        Xs = Xd[:300_000].cpu().numpy()
        lab_o, core_o, _, nc_o = oracle.dbscan(Xs, c["eps"], c["min_samples"])
        ctx.set_option(native.PD_OPT_DIR_PAGED, 1)
        try:
            m = DBSCAN(eps=c["eps"], min_samples=c["min_samples"], max_partitions=8).train(
                _dev(Xs))
        finally:
            ctx.set_option(native.PD_OPT_DIR_PAGED, -1)
        assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), lab_o)
        assert np.array_equal(m.core_sample_mask_.cpu().numpy(), core_o)


@pytest.mark.parametrize("d", [2, 3, 4])
def test_globe_sized_extent(native, d):
    """Clusters 1e7 eps apart on every axis (a bbox-sized directory of 1e14 -
    1e28 cells): the cells grow to the default 32 GiB budget and the answer
    still equals the oracle's (dense clusters, noise, a chain across cells)."""
    rng = np.random.default_rng(40 + d)
    eps = 0.01
    parts = [rng.normal(scale=0.02, size=(3000, d)) + c
             for c in (np.zeros(d), np.full(d, 1e5), np.r_[1e5, np.zeros(d - 1)])]
    chain = np.zeros((400, d))
    chain[:, 0] = -1.0 - 0.009 * np.arange(400)   # spacing < eps: one chain cluster
    noise = rng.uniform(-2e5, 2e5, size=(500, d))
    X = np.concatenate(parts + [chain, noise]).astype(np.float64)
    lab_o, core_o, cnt_o, nc_o = oracle.dbscan(X, eps, 5)
    lab, core, ncl, cnt = _cluster(native, X, eps, 5, full=True)
    assert native.context().timings()["grid_grow"] > 1.0
    assert np.array_equal(cnt, cnt_o)
    assert np.array_equal(core, core_o)
    assert np.array_equal(lab, lab_o) and ncl == nc_o
    from pypardis_amd import DBSCAN
    m = DBSCAN(eps=eps, min_samples=5, max_partitions=8).train(_dev(X))
    assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), lab_o)


# ------------------------------------------------------------ device-decided KD
KD_DEV = [("c2_1m", 8), ("c2_1m", 13), ("c2_1m", 64), ("c4_500k", 16), ("f64_300k", 5),
          ("ident_5k", 8), ("tiny_7", 4), ("d1_200k", 32), ("d4_300k", 256)]


def _kd_case(name):
    from pypardis_amd import synth
    rng = np.random.default_rng(11)
    if name == "c2_1m":
        return synth.make_config("C2", n=1_000_000)[0]
    if name == "c4_500k":
        return synth.gps_skew(500_000, seed=8, n_cities=200).numpy()
    if name == "f64_300k":
        return rng.normal(size=(300_000, 3)) * np.array([1.0, 1e-3, 5.0]) + 1e4
    if name == "ident_5k":
        return np.full((5_000, 2), 0.5, np.float32)
    if name == "tiny_7":
        return rng.normal(size=(7, 3)).astype(np.float32)
    if name == "d1_200k":
        return rng.uniform(-1, 1, size=(200_000, 1)).astype(np.float32)
    return rng.normal(size=(300_000, 4)).astype(np.float32)


@pytest.mark.parametrize("name,P", KD_DEV, ids=[f"{c[0]}-P{c[1]}" for c in KD_DEV])
def test_kd_device_decisions_equal_host(native, name, P):
    """pd_kd_build (level decisions on the device, one sync) gives the per-pass
    host-decided path's split trace, boxes and labels bit for bit — levels of
    1..128 splits, fp32 / fp64, zero variance, fewer points than partitions —
    without the fused levels (the default), with them (PD_OPT_KD_FUSE:
    counts + the children's interval moments in one pass) and with the
    labels replayed from the split tree instead of kept in HBM
    (PD_OPT_KD_REPLAY)."""
    from pypardis_amd import KDPartitioner, partition
    X = _kd_case(name)
    Xd = _dev(X)
    a = KDPartitioner(Xd, P)
    ctx = native.context()
    ctx.set_option(native.PD_OPT_KD_FUSE, 1)
    try:
        c = KDPartitioner(Xd, P)
    finally:
        ctx.set_option(native.PD_OPT_KD_FUSE, 0)
    ctx.set_option(native.PD_OPT_KD_REPLAY, 1)
    try:
        r = KDPartitioner(Xd, P)
        r.labels   # (replayed now, under the option)
    finally:
        ctx.set_option(native.PD_OPT_KD_REPLAY, 0)
    partition.DEVICE_DECISIONS = False
    try:
        b = KDPartitioner(Xd, P)
    finally:
        partition.DEVICE_DECISIONS = True
    sb, fb = _kd_arrays(b.splits)
    for m in (a, c, r):
        sa, fa = _kd_arrays(m.splits)
        assert np.array_equal(sa, sb)
        assert np.array_equal(fa, fb, equal_nan=True)
        assert np.array_equal(m.box_array(), b.box_array(), equal_nan=True)
        assert torch.equal(m.labels, b.labels)
        assert m.data_box[0].tolist() == b.data_box[0].tolist()
    sa, fa = _kd_arrays(a.splits)
    if name == "c2_1m" and P == 8:   # and the oracle's exact restatement
        ref = oracle.kd_partition(X, P, sums="exact")
        assert np.array_equal(sa, _kd_arrays(ref["splits"])[0])
        assert np.array_equal(a.labels.cpu().numpy(), ref["owner"])


@pytest.mark.parametrize("P", [300, 1000])
def test_train_many_partitions_fallbacks(native, P):
    """Many partitions: P = 300 keeps the device-decided KD (split labels <
    256) with the split tree replayed from global memory in the unmasked
    halo kernel (P > 64); P = 1000 has split labels beyond the LDS tables, so
    KDPartitioner falls back to the per-pass path and DBSCAN.train to owner
    labels — labels the oracle's either way."""
    from pypardis_amd import DBSCAN, synth
    X, cfg = synth.make_config("C2", n=200_000)
    lab_o, core_o, _, nc_o = oracle.dbscan(X, cfg["eps"], cfg["min_samples"])
    m = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=P).train(_dev(X))
    assert (m.partitioner.split_tree() is None) == (P > 512)
    assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), lab_o)
    assert np.array_equal(m.core_sample_mask_.cpu().numpy(), core_o)
    assert m.n_clusters_ == nc_o and len(m.bounding_boxes) == P


@pytest.mark.parametrize("P,cap", [(8, 0), (8, 1000), (8, -1), (300, 0), (300, 1000),
                                   (300, -1), (1000, 0), (1000, 1000)])
def test_halo_single_pass_equals_two_pass(native, P, cap):
    """PD_OPT_HALO_PASSES: the single-pass halo (look-back offsets into
    buffers of a guessed capacity) writes the same records as the two-pass
    form — identical labels, core flags and record counts — with the key grids
    and the split tree in LDS (P <= 64), the unmasked kernel reading the tree
    from global memory (P = 300) and owner labels (P = 1000); cap 1000 forces
    the overflow fallback (every tile past the capacity drops its stores, the
    host reruns two passes), cap -1 sets the capacity to exactly the total
    (no fallback, every slot written).  The round-5 fault (an illegal access
    on the P = 300 overflow path) is this case.  A second train at the
    default capacity follows one that overflowed: the capacity grows to the
    previous records per point, so it takes a single pass."""
    from pypardis_amd import DBSCAN, synth
    X, cfg = synth.make_config("C2", n=200_000)
    lab_o, core_o, _, nc_o = oracle.dbscan(X, cfg["eps"], cfg["min_samples"])
    ctx = native.context()
    Xd = _dev(X)
    try:
        ctx.set_option(native.PD_OPT_HALO_PASSES, 2)
        m2 = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=P).train(Xd)
        R = int(ctx.timings()["records"])
        ctx.set_option(native.PD_OPT_HALO_PASSES, 1)
        ctx.set_option(native.PD_OPT_HALO_CAP, R if cap < 0 else cap)
        m1 = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=P).train(Xd)
        t = ctx.timings()
        ctx.set_option(native.PD_OPT_HALO_CAP, 0)   # (still the single pass)
        m0 = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=P).train(Xd)
        t0 = ctx.timings()
    finally:
        ctx.set_option(native.PD_OPT_HALO_PASSES, 2)
        ctx.set_option(native.PD_OPT_HALO_CAP, 0)
    assert int(t["records"]) == R
    if cap != 0:   # (the default capacity adapts to the previous train's records)
        assert int(t["halo_fallback"]) == (1 if cap == 1000 else 0)
    assert int(t0["records"]) == R and int(t0["halo_fallback"]) == 0
    for m in (m0, m1, m2):
        assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), lab_o)
        assert np.array_equal(m.core_sample_mask_.cpu().numpy(), core_o)
        assert m.n_clusters_ == nc_o


HALO_TREE = [("c2", 8), ("c2", 64), ("c4", 8), ("c4", 37), ("lattice", 16), ("f64_4d", 13),
             ("dup", 8), ("city", 5)]


@pytest.mark.parametrize("case,P", HALO_TREE, ids=[f"{c}-P{p}" for c, p in HALO_TREE])
def test_halo_tree_equals_full_test(native, case, P):
    """PD_OPT_HALO_TREE (opt-in, measured slower): the halo's near-plane path — a
    point farther than 2 eps from every split plane on its KD path gets its
    owner's record only, the rest the full box test — writes the records of
    the full test (same count) and gives the oracle's labels: 2-D / 3-D / 4-D,
    fp32 / fp64, lattice points exactly on split planes, duplicates, cityblock,
    up to 64 partitions."""
    from pypardis_amd import DBSCAN, synth
    rng = np.random.default_rng(P)
    metric, eps, ms = "euclidean", 0.1, 10
    if case == "c2":
        X, cfg = synth.make_config("C2", n=300_000)
        eps, ms = cfg["eps"], cfg["min_samples"]
    elif case == "c4":
        X = synth.gps_skew(400_000, seed=8, n_cities=300).numpy()
        eps, ms = 0.01, 20
    elif case == "lattice":
        g = np.arange(200, dtype=np.float32) * np.float32(0.05)
        X = np.stack(np.meshgrid(g, g, indexing="ij"), -1).reshape(-1, 2)
        eps, ms = float(np.float32(0.05)), 5
    elif case == "f64_4d":
        X = rng.normal(size=(150_000, 4)) * 3.0
        eps, ms = 0.35, 8
    elif case == "dup":
        X = np.repeat(rng.uniform(0, 5, size=(20_000, 3)).astype(np.float32), 5, axis=0)
        eps, ms = 0.05, 6
    else:
        X = synth.blobs_noise(120_000, 2, side=30.0, n_centers=10, sigma=0.7, noise_frac=0.2,
                              seed=24)
        metric, eps, ms = "cityblock", 0.06, 8
    lab_o, core_o, _, nc_o = oracle.dbscan(X, eps, ms, metric)
    ctx = native.context()
    Xd = _dev(X)
    out = []
    for on in (1, 0):
        ctx.set_option(native.PD_OPT_HALO_TREE, on)
        try:
            m = DBSCAN(eps=eps, min_samples=ms, metric=metric, max_partitions=P).train(Xd)
        finally:
            ctx.set_option(native.PD_OPT_HALO_TREE, 0)
        out.append((m, int(ctx.timings()["records"])))
    assert out[0][1] == out[1][1]
    for m, _ in out:
        assert np.array_equal(m.labels_.cpu().numpy().astype(np.int64), lab_o)
        assert np.array_equal(m.core_sample_mask_.cpu().numpy(), core_o)
        assert m.n_clusters_ == nc_o


@pytest.mark.parametrize("cfg,n", [("C2", 2_000_000), ("C4", 3_000_000), ("C1", 500_000)])
def test_verify_fused_equals_listed(native, cfg, n):
    """PD_OPT_VERIFY_FUSED: the cell verify over every cell with the screen
    inline gives the labels of the screen -> flag list -> verify form."""
    from pypardis_amd import DBSCAN, synth
    X, c = synth.make_config(cfg, n=n, device="cuda" if cfg == "C4" else "cpu")
    Xd = X if torch.is_tensor(X) else _dev(X)
    ctx = native.context()
    outs = []
    for on in (1, 0):
        ctx.set_option(native.PD_OPT_VERIFY_FUSED, on)
        try:
            m = DBSCAN(eps=c["eps"], min_samples=c["min_samples"],
                       max_partitions=c.get("max_partitions") or 1).train(Xd)
        finally:
            ctx.set_option(native.PD_OPT_VERIFY_FUSED, 0)
        outs.append((m.labels_.clone(), m.core_sample_mask_.clone(), m.n_clusters_))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2]


@pytest.mark.parametrize("cfg,n", [("C2", 2_000_000), ("C4", 3_000_000), ("C1", 500_000)])
def test_label_buckets_equal_direct_scatter(native, cfg, n):
    """PD_OPT_LABEL_BUCKETS (default on): the labels reach input order through
    the bucketed (point, key) pair passes instead of one scattered write per
    owner record — identical labels and core flags from the block-local pass
    (1: 2^19-point buckets split into 2^15-point ones placed in LDS), the
    round-4 L2-bucket scatter (2) and the direct scatter (0); several buckets,
    partial last bucket, noise and border points included."""
    from pypardis_amd import DBSCAN, synth
    X, c = synth.make_config(cfg, n=n, device="cuda" if cfg == "C4" else "cpu")
    Xd = X if torch.is_tensor(X) else _dev(X)
    ctx = native.context()
    outs = []
    for on in (1, 2, 0):
        ctx.set_option(native.PD_OPT_LABEL_BUCKETS, on)
        try:
            m = DBSCAN(eps=c["eps"], min_samples=c["min_samples"],
                       max_partitions=c.get("max_partitions") or 1).train(Xd)
        finally:
            ctx.set_option(native.PD_OPT_LABEL_BUCKETS, -1)
        outs.append((m.labels_.clone(), m.core_sample_mask_.clone(), m.n_clusters_))
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0]) and torch.equal(outs[0][1], o[1])
        assert outs[0][2] == o[2]
    lab = outs[0][0]
    assert bool((lab == -1).any()) and bool((lab >= 0).any())
