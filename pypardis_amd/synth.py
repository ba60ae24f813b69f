"""Synthetic workloads named in SURVEY.md §8(d) (configs C0–C4 of BASELINE.json).

All generators are deterministic in ``seed`` and return C-contiguous float32
(n, d) arrays (C0 is float64, as in the reference's own demo data).  They are
plain numpy so the CPU oracle, the GPU tests and ``bench.py`` see the same
points.
"""
from __future__ import annotations

import numpy as np


def blobs_noise(n, d, side=100.0, n_centers=64, sigma=1.0, noise_frac=0.10,
                seed=0, dtype=np.float32, chunk=1 << 24):
    """SURVEY.md §8(d) ``blobs_noise``.

    centres ~ U[0, side]^d; (1 - noise_frac)·n points = centre[U{0..n_centers-1}]
    + N(0, sigma² I); the rest ~ U[0, side]^d.  Rows are shuffled so blob and
    noise points interleave (input order matters to sklearn's label numbering,
    so the order is part of the workload).
    """
    n = int(n)
    rng = np.random.default_rng(seed)
    centers = rng.uniform(0.0, side, size=(n_centers, d))
    n_blob = int(round((1.0 - noise_frac) * n))
    out = np.empty((n, d), dtype=dtype)
    # chunked so a 1e8-point config never holds more than one fp64 chunk
    for s in range(0, n_blob, chunk):
        e = min(n_blob, s + chunk)
        which = rng.integers(0, n_centers, size=e - s)
        out[s:e] = centers[which] + rng.normal(0.0, sigma, size=(e - s, d))
    for s in range(n_blob, n, chunk):
        e = min(n, s + chunk)
        out[s:e] = rng.uniform(0.0, side, size=(e - s, d))
    perm = rng.permutation(n)
    return np.ascontiguousarray(out[perm])


def c0_demo():
    """C0: the scikit-learn ``plot_dbscan`` demo the reference's plots use
    (SURVEY.md §4): 750 points, 3 centres, StandardScaler; fp64."""
    from sklearn.datasets import make_blobs
    from sklearn.preprocessing import StandardScaler
    X, _ = make_blobs(n_samples=750, centers=[[1, 1], [-1, -1], [1, -1]],
                      cluster_std=0.4, random_state=0)
    return np.ascontiguousarray(StandardScaler().fit_transform(X))


def embeddings(n, d=64, n_clusters=2000, clustered_frac=0.10, spread=0.1, seed=3,
               dtype=np.float32, chunk=1 << 20):
    """unit-norm embeddings.  clustered_frac·n points are
    normalize(c_j + spread·g) around n_clusters centres c_j ~ N(0, I_d); the
    rest are normalize(g), g ~ N(0, I_d).  Rows shuffled."""
    n = int(n)
    rng = np.random.default_rng(seed)
    centers = rng.normal(size=(n_clusters, d))
    n_cl = int(round(clustered_frac * n))
    out = np.empty((n, d), dtype=dtype)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        g = rng.normal(size=(e - s, d))
        k = np.arange(s, e) < n_cl
        if k.any():
            g[k] = centers[rng.integers(0, n_clusters, size=int(k.sum()))] + spread * g[k]
        out[s:e] = g / np.linalg.norm(g, axis=1, keepdims=True)
    perm = rng.permutation(n)
    return np.ascontiguousarray(out[perm])


C3_EPS = 0.114028   # tools/c3_eps.py: 0.11402826147489717, rounded to 6 digits

# BASELINE.json configs (sizes, eps, min_samples, max_partitions)
CONFIGS = {
    "C0": dict(n=750, d=2, eps=0.3, min_samples=10, max_partitions=None),
    "C1": dict(n=10_000_000, d=2, side=100.0, n_centers=64, sigma=1.0,
               noise_frac=0.10, seed=1, eps=0.05, min_samples=10,
               max_partitions=1),
    "C2": dict(n=100_000_000, d=3, side=100.0, n_centers=256, sigma=1.0,
               noise_frac=0.10, seed=2, eps=0.1, min_samples=10,
               max_partitions=8),
    # eps: the 1st percentile over 50k sampled points of the distance to the
    # 10th neighbour (self included) in the full 1M set, so ~1% of points are
    # core; computed once by tools/c3_eps.py
    "C3": dict(n=1_000_000, d=64, n_clusters=2000, clustered_frac=0.10, spread=0.1,
               seed=3, eps=C3_EPS, min_samples=10, max_partitions=1),
}


def make_config(name, n=None):
    """Points for config ``name``; ``n`` < full size gives a density-preserving
    slice: side scaled by (n/N)^(1/d) and the number of centres by n/N, so
    both the noise density and the points per blob stay those of the full
    config."""
    cfg = dict(CONFIGS[name])
    if name == "C0":
        return c0_demo(), cfg
    if name == "C3":   # slices keep the points per cluster: fewer clusters
        N = cfg["n"]
        n = N if n is None else int(n)
        k = max(1, int(round(cfg["n_clusters"] * n / N)))
        X = embeddings(n, cfg["d"], n_clusters=k, clustered_frac=cfg["clustered_frac"],
                       spread=cfg["spread"], seed=cfg["seed"])
        cfg.update(n=n, n_clusters=k)
        return X, cfg
    N = cfg["n"]
    n = N if n is None else int(n)
    side = cfg["side"] * (n / N) ** (1.0 / cfg["d"])
    n_centers = max(1, int(round(cfg["n_centers"] * n / N)))
    X = blobs_noise(n, cfg["d"], side=side, n_centers=n_centers,
                    sigma=cfg["sigma"], noise_frac=cfg["noise_frac"],
                    seed=cfg["seed"])
    cfg.update(n=n, side=side, n_centers=n_centers)
    return X, cfg
