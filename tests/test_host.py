"""CPU tests of the host-side logic that mirrors the reference (no GPU)."""
import sys

import numpy as np
import pytest
import torch

import oracle
from conftest import golden_names, load_golden
from pypardis_amd import BoundingBox, ClusterAggregator, default_value
from pypardis_amd import partition as part
from pypardis_amd._data import as_points


@pytest.mark.parametrize("P", [1, 2, 3, 5, 8, 16, 17, 64, 100])
def test_split_schedule_matches_reference_bfs(P):
    assert part._split_schedule(P) == oracle.split_schedule(P)


def test_split_schedule_label_order_p8():
    # 0→1 · 0→2, 1→3 · 0→4, 2→5, 1→6, 3→7
    assert part._split_schedule(8) == [[(0, 1)], [(0, 2), (1, 3)], [(0, 4), (2, 5), (1, 6), (3, 7)]]


@pytest.mark.parametrize("name", golden_names())
def test_bounds_expression_bit_exact(name):
    g = load_golden(name)
    for (mean, var, boundary), (_, _, _, cand, _, _) in zip(g["split_f"], g["splits"]):
        assert part._bounds(mean, var)[cand] == boundary


def test_bounding_box_sentinels_and_ops():
    b = BoundingBox(k=2)
    assert b.lower[0] == sys.float_info.max and b.upper[0] == sys.float_info.min
    u = b.union(BoundingBox(np.array([-5.0, 1.0])))
    assert u.upper[0] == sys.float_info.min and u.lower[0] == -5.0 and u.upper[1] == 1.0
    left, right = BoundingBox([0.0, 0.0], [2.0, 2.0]).split(1, 0.5)
    assert left.upper[1] == 0.5 and right.lower[1] == 0.5 and left.lower[1] == 0.0
    e = BoundingBox([0.0], [1.0]).expand(0.25)
    assert e.lower[0] == -0.25 and e.upper[0] == 1.25
    m = BoundingBox([0.0], [2.0]).expand(0.5, how="multiply")
    assert m.lower[0] == -1.0 and m.upper[0] == 3.0
    assert BoundingBox([0.0, 0.0], [1.0, 1.0]).contains(np.array([1.0, 0.0]))
    assert not BoundingBox([0.0, 0.0], [1.0, 1.0]).contains(np.array([1.0, 1.0 + 1e-12]))
    i = BoundingBox([0.0], [2.0]).intersection(BoundingBox([1.0], [3.0]))
    assert i.lower[0] == 1.0 and i.upper[0] == 2.0


@pytest.mark.parametrize("name", ["c0", "neg_3k", "b3d_20k"])
def test_expanded_boxes_from_golden_boxes(name):
    g = load_golden(name)
    eps = float(g["eps"])
    for L in range(int(g["P"])):
        e = BoundingBox(g["box_lo"][L], g["box_hi"][L]).expand(2 * eps)
        assert np.array_equal(e.lower, g["ebox_lo"][L]) and np.array_equal(e.upper, g["ebox_hi"][L])


def _order_keys(v):
    """numpy twin of kd.hip order_key (fp64 bits -> order-preserving u64)."""
    b = np.ascontiguousarray(v, np.float64).view(np.uint64).copy()
    b[b == np.uint64(1 << 63)] = 0
    neg = (b >> np.uint64(63)) == 1
    return np.where(neg, ~b, b | np.uint64(1 << 63))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_level_medians_radix_select(dtype):
    """Host side of split_method='rotation': the digit walk over emulated
    pd_kd_radix_hist histograms returns sorted(v)[len // 2] exactly, with
    ties, negative values and signed zeros, for several splits at once."""
    rng = np.random.default_rng(5)
    groups = [rng.normal(size=1001), np.round(rng.normal(size=64), 1),
              np.array([-0.0, 0.0, -0.0, 1.0, -2.5]), np.full(7, 3.25), np.array([-7.0])]
    groups = [g.astype(dtype) for g in groups]
    keys = [_order_keys(g.astype(np.float64)) for g in groups]

    def hist_fn(prefix, shift):
        h = np.zeros((len(groups), 256), np.int64)
        for s, k in enumerate(keys):
            if shift + 8 < 64:
                k = k[(k >> np.uint64(shift + 8)) == np.uint64(prefix[s])]
            np.add.at(h[s], ((k >> np.uint64(shift)) & np.uint64(255)).astype(np.int64), 1)
        return h

    med, less, tot = part.level_medians(hist_fn, len(groups), dtype == np.float32)
    for s, g in enumerate(groups):
        want = np.sort(g.astype(np.float64))[len(g) // 2]
        assert med[s] == want, s
        assert less[s] == int((g.astype(np.float64) < want).sum()) and tot[s] == len(g)
    with pytest.raises(IndexError):
        part.level_medians(lambda p, s: np.zeros((1, 256), np.int64), 1, False)


def test_cluster_aggregator_links_core_labels_only():
    agg = ClusterAggregator()
    agg + (0, ["0:0", "1:3"])          # core in two neighbourhoods: link
    agg + (1, ["1:3", "2:1"])
    agg + (2, ["0:5*", "1:3"])         # border label must not link 0:5
    agg + (3, ["0:5", "1:-1*"])
    assert agg.fwd["0:0"] == agg.fwd["1:3"] == agg.fwd["2:1"]
    assert agg.fwd["0:5"] != agg.fwd["0:0"]
    assert "1:-1*" not in agg.fwd and "0:5*" not in agg.fwd
    other = ClusterAggregator()
    other + (9, ["0:5", "2:1"])
    agg + other
    assert agg.fwd["0:5"] == agg.fwd["0:0"]
    assert default_value() == sys.maxsize


def test_as_points_forms_cpu():
    X = np.random.default_rng(0).normal(size=(10, 3)).astype(np.float32)
    p = as_points(X, device="cpu")
    assert p.X.dtype == torch.float32 and p.keys is None and p.n == 10
    p = as_points([(i, X[i]) for i in range(10)], device="cpu")
    assert p.keys is None and torch.equal(p.X, torch.from_numpy(X))
    p = as_points([(f"k{i}", X[i].astype(np.float64)) for i in range(10)], device="cpu")
    assert p.X.dtype == torch.float64 and p.keys[3] == "k3"

    class RDD:
        def collect(self):
            return [(10 - i, X[i]) for i in range(10)]
    p = as_points(RDD(), device="cpu")
    assert list(p.keys) == list(range(10, 0, -1))
    p = as_points((np.arange(10) * 2, X), device="cpu")
    assert p.keys[1] == 2


def test_as_points_edge_forms_cpu():
    X = np.arange(6, dtype=np.float32).reshape(3, 2)
    # a tuple of exactly two (key, vector) records is records, not (keys, X)
    p = as_points(((7, X[0]), (9, X[1])), device="cpu")
    assert list(p.keys) == [7, 9] and p.n == 2 and p.d == 2
    # (keys, X) with two points
    p = as_points((np.array([4, 5]), X[:2]), device="cpu")
    assert list(p.keys) == [4, 5] and torch.equal(p.X, torch.from_numpy(X[:2]))
    # (keys, X) with a torch key tensor (its elements are 0-d tensors)
    p = as_points((torch.arange(3) + 10, X), device="cpu")
    assert list(p.keys) == [10, 11, 12] and p.keys.dtype == np.int64 and p.n == 3
    p = as_points((torch.arange(3), torch.from_numpy(X)), device="cpu")
    assert list(p.keys) == [0, 1, 2] and torch.equal(p.X, torch.from_numpy(X))
    # dtype from every vector: one float64 vector after many float32 ones
    recs = [(i, X[i % 3]) for i in range(100)] + [(100, np.array([0.1, 0.2]))]
    p = as_points(recs, device="cpu")
    assert p.X.dtype == torch.float64 and float(p.X[100, 0]) == 0.1
    # integer vectors become float64; 1-D input is one axis
    assert as_points([(0, [1, 2]), (1, [3, 4])], device="cpu").X.dtype == torch.float64
    assert as_points(np.arange(5.0), device="cpu").d == 1
    with pytest.raises(ValueError):
        as_points([], device="cpu")


def test_native_ingest_matches_numpy_unzip(monkeypatch):
    """csrc/ingest.cpp's one-pass unzip gives the same X (values and dtype)
    and keys as the numpy path, for every record form it accepts."""
    from pypardis_amd import _data
    from pypardis_amd.build import build_ingest
    build_ingest()
    from pypardis_amd import _ingest  # noqa: F401  (must import once built)
    rng = np.random.default_rng(3)
    X = rng.normal(size=(50, 3)).astype(np.float32)
    X64 = X.astype(np.float64) + 1e-9
    forms = [
        [(i, X[i]) for i in range(50)],
        [(49 - i, X[i]) for i in range(50)],
        [(i, X64[i]) for i in range(50)],
        [(i, X[i] if i % 3 else X64[i]) for i in range(50)],
        [(f"k{i}", list(map(float, X64[i]))) for i in range(50)],
        [[i, X[i].astype(np.float16)] for i in range(50)],
        [(i, np.asarray(X.T)[:, i]) for i in range(50)],          # strided rows
        [(2 ** 65 + i, X[i]) for i in range(50)],                  # non-int64 keys
        [(i, [1, 2, 3]) for i in range(50)],
    ]
    for recs in forms:
        got = _data._unzip_native(recs)
        assert got is not None
        monkeypatch.setattr(_data, "_unzip_native", lambda r: None)
        want = _data.as_points(recs, device="cpu")
        monkeypatch.undo()
        gx, gk = got
        assert gx.dtype == want.X.numpy().dtype
        assert np.array_equal(gx, want.X.numpy())
        wk = want.key_array()
        assert list(_data._dense_or(gk) if _data._dense_or(gk) is not None
                    else np.arange(50)) == list(wk)
    # ragged / scalar vectors are left to the numpy path
    assert _data._unzip_native([(0, [1.0, 2.0]), (1, [1.0])]) is None
    assert _data._unzip_native([(0, 1.0), (1, 2.0)]) is None


def test_map_cluster_id():
    """R:dbscan/dbscan.py:37-53: first label of the group, '*' stripped; noise
    or unmapped labels give -1; a broadcast wrapper or a plain dict."""
    from pypardis_amd import map_cluster_id

    class Broadcast:
        def __init__(self, v):
            self.value = v

    fwd = {"0:0": 3, "1:2": 3, "2:1": 5}
    assert map_cluster_id((10, ["0:0*", "1:2"]), Broadcast(fwd)) == (10, 3)
    assert map_cluster_id((11, ["2:1"]), fwd) == (11, 5)
    assert map_cluster_id((12, ["1:-1*", "0:0"]), fwd) == (12, -1)
    assert map_cluster_id((13, iter(["4:7"])), fwd) == (13, -1)


def test_c4_generator():
    """C4 GPS-like skew: deterministic in the seed, float32, inside the
    lon/lat box, 5% uniform noise, heavy Zipf skew (the densest eps-cell of
    a 2M sample holds > 50 points)."""
    from pypardis_amd import synth
    X, cfg = synth.make_config("C4", n=2_000_000)
    Y, _ = synth.make_config("C4", n=2_000_000)
    assert X.dtype == np.float32 and X.shape == (2_000_000, 2)
    assert np.array_equal(X, Y)
    assert X[:, 0].min() >= -180 and X[:, 0].max() < 180
    assert X[:, 1].min() >= -60 and X[:, 1].max() <= 75
    k = np.floor(X.astype(np.float64) / cfg["eps"]).astype(np.int64)
    _, c = np.unique(k[:, 0] * 1_000_000 + k[:, 1], return_counts=True)
    assert c.max() > 50
    assert cfg["eps"] == 0.001 and cfg["min_samples"] == 20 and cfg["max_partitions"] == 8
