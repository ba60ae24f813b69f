"""The windowed full-size checker (tests/window_check.py) itself, on CPU:
it accepts the oracle's own global answer and rejects corrupted ones."""
import numpy as np
import pytest
import torch

import oracle
import window_check as wc


@pytest.fixture(scope="module")
def case():
    from pypardis_amd import synth
    X, cfg = synth.make_config("C2", n=150_000)
    eps, ms = cfg["eps"], cfg["min_samples"]
    lab, core, cnt, nc = oracle.dbscan(X, eps, ms)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a.astype(dt)))
    return (torch.from_numpy(X), t(lab, np.int32), t(core, np.uint8), t(cnt, np.int32), eps, ms,
            nc)


def _run(case, lab, core, cnt, **kw):
    X, _, _, _, eps, ms, _ = case
    return wc.run_windows(X, lab, core, cnt, eps, ms, True, n_random=8, n_dense=4, n_uniform=3,
                          max_pts=20_000, **kw)


def test_accepts_oracle_answer(case):
    X, lab, core, cnt, eps, ms, nc = case
    assert wc.check_numbering(lab, core) == nc
    tallies, skipped = _run(case, lab, core, cnt)
    assert len(tallies) == 15 and not skipped
    assert sum(t["edges"] for t in tallies) > 0
    assert sum(t["border"] for t in tallies) > 0


def test_rejects_split_cluster(case):
    X, lab, core, cnt, eps, ms, nc = case
    # relabel half of the core points of the largest cluster
    big = int(torch.bincount(lab[lab >= 0].long()).argmax())
    idx = torch.nonzero((lab == big) & (core == 1)).flatten()
    bad = lab.clone()
    bad[idx[::2]] = nc
    with pytest.raises(AssertionError):
        _run(case, bad, core, cnt, seed=0)


def test_rejects_wrong_counts_and_core(case):
    X, lab, core, cnt, eps, ms, nc = case
    bad = cnt.clone()
    bad += 1
    with pytest.raises(AssertionError, match="counts"):
        _run(case, lab, core, bad)
    badc = core.clone()
    badc[:] = 1 - badc
    with pytest.raises(AssertionError, match="core"):
        _run(case, lab, badc, cnt)


def test_rejects_merged_clusters(case):
    X, lab, core, cnt, eps, ms, nc = case
    # two clusters given one label: caught by the closed-cluster census
    # (when a closed one exists) or the numbering order
    bad = lab.clone()
    bad[bad == 1] = 0
    with pytest.raises(AssertionError):
        wc.check_numbering(bad, core)
        _run(case, bad, core, cnt)


def test_counts_capped_matches_sweep():
    from pypardis_amd import synth
    X = synth.blobs_noise(5000, 2, side=3.0, n_centers=3, sigma=0.2, seed=5)
    full = oracle.counts(X, 0.05)
    assert np.array_equal(oracle.counts_capped(X, X, 0.05, 0), full)
    assert np.array_equal(oracle.counts_capped(X[:700], X, 0.05, 7), np.minimum(full[:700], 7))


def test_clique_window():
    from pypardis_amd import synth
    Xn = synth.blobs_noise(60_000, 2, side=2.0, n_centers=2, sigma=0.1, seed=9)
    eps, ms = 0.02, 10
    lab, core, cnt, nc = oracle.dbscan(Xn, eps, ms)
    X = torch.from_numpy(Xn)
    lab = torch.from_numpy(lab.astype(np.int32))
    core = torch.from_numpy(core)
    cnt = torch.from_numpy(cnt.astype(np.int32))
    c = X[int(torch.argmax(cnt))].double().numpy()
    t = wc.check_clique_window(X, lab, core, cnt, eps, ms, c)
    assert t["core"] > 10
    ids = torch.nonzero(((X.double() - torch.from_numpy(c)).abs() <= eps / 4).all(1)).flatten()
    bad = lab.clone()
    bad[ids[0]] = nc + 5
    with pytest.raises(AssertionError, match="clique"):
        wc.check_clique_window(X, bad, core, cnt, eps, ms, c)
    badc = core.clone()
    badc[ids[1]] = 0
    with pytest.raises(AssertionError, match="core"):
        wc.check_clique_window(X, lab, badc, cnt, eps, ms, c)
