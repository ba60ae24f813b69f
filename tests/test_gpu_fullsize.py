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
