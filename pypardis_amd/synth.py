"""Synthetic workloads named in SURVEY.md §8(d) (configs C0–C4 of BASELINE.json).

All generators are deterministic in ``seed`` and return C-contiguous float32
(n, d) arrays (C0 is float64, as in the reference's own demo data).  C0–C3
are plain numpy so the CPU oracle, the GPU tests and ``bench.py`` see the
same points; C4 (``gps_skew``, 1B points) is torch, generated on the device
for the bench and on the CPU for the oracle tests (deterministic per device
type).
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


def gps_skew(n, seed=4, n_cities=10_000, zipf=1.1, sigma0=0.02, sigma_pow=0.3,
             noise_frac=0.05, lon=(-180.0, 180.0), lat=(-60.0, 75.0), device="cpu",
             chunk=1 << 25):
    """GPS-like skewed 2-D density (lon, lat in degrees).

    ``n_cities`` centres ~ U(box); city of rank r (1-based) has Zipf weight
    r^-zipf and spread sigma0·r^sigma_pow degrees; (1 - noise_frac) of the
    points are centre + N(0, sigma²I) (longitude wrapped, latitude clamped
    into the box), the rest uniform in the box.  Each row independently is
    noise or a city point, so rows are already interleaved.

    Generated with torch on ``device`` in chunks (a 1B-point set is built on
    the GPU in seconds); the stream is deterministic in (seed, device type),
    so tests that compare against the oracle build the points on the CPU.
    Returns a float32 torch tensor (n, 2) on ``device``.
    """
    import torch
    n = int(n)
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(int(seed))
    f64 = torch.float64
    lo = torch.tensor([lon[0], lat[0]], dtype=f64, device=dev)
    span = torch.tensor([lon[1] - lon[0], lat[1] - lat[0]], dtype=f64, device=dev)
    centres = lo + span * torch.rand(n_cities, 2, generator=g, dtype=f64, device=dev)
    r = torch.arange(1, n_cities + 1, dtype=f64, device=dev)
    cdf = torch.cumsum(r ** -zipf, 0)
    cdf = cdf / cdf[-1]
    sig = sigma0 * r ** sigma_pow
    out = torch.empty(n, 2, dtype=torch.float32, device=dev)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        m = e - s
        u = torch.rand(m, generator=g, dtype=f64, device=dev)
        city = torch.searchsorted(cdf, u).clamp_(max=n_cities - 1)
        pts = centres[city] + sig[city, None] * torch.randn(m, 2, generator=g, dtype=f64,
                                                             device=dev)
        pts[:, 0] = torch.remainder(pts[:, 0] - lon[0], span[0]) + lon[0]
        pts[:, 1].clamp_(lat[0], lat[1])
        noise = torch.rand(m, generator=g, dtype=f64, device=dev) < noise_frac
        uni = lo + span * torch.rand(m, 2, generator=g, dtype=f64, device=dev)
        pts = torch.where(noise[:, None], uni, pts)
        out[s:e] = pts.to(torch.float32)
        # fp32 rounding can land a wrapped longitude on +180: keep it in [lo, hi)
        col = out[s:e, 0]
        col[col >= lon[1]] = lon[0]
        del u, city, pts, noise, uni
    return out


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
    # 1B points is the 8-GPU config; one MI355X holds it too (n < 2^30)
    "C4": dict(n=1_000_000_000, d=2, seed=4, eps=0.001, min_samples=20, max_partitions=8),
}


def make_config(name, n=None, device="cpu"):
    """Points for config ``name``; ``n`` < full size gives a density-preserving
    slice: side scaled by (n/N)^(1/d) and the number of centres by n/N, so
    both the noise density and the points per blob stay those of the full
    config."""
    cfg = dict(CONFIGS[name])
    if name == "C0":
        return c0_demo(), cfg
    if name == "C4":   # a sample of the same distribution (not density-preserving)
        n = cfg["n"] if n is None else int(n)
        cfg.update(n=n)
        return gps_skew(n, seed=cfg["seed"], device=device).numpy() if device == "cpu" \
            else gps_skew(n, seed=cfg["seed"], device=device), cfg
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
