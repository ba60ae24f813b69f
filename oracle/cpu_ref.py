"""ORACLE — TEST/BENCH INFRASTRUCTURE ONLY: the timed CPU baseline.

The reference's own pipeline restated for a multi-core host, as SURVEY.md
§8(d) / BASELINE.md prescribe (the Spark path itself cannot run here or on
the GPU box: no JVM, and the reference never travels):

  1. KD partition, the reference's min_var/mean_var rule   (oracle.kd_partition,
     R:dbscan/partition.py:33-183)
  2. 2·eps halo                                            (oracle.halo,
     R:dbscan/dbscan.py:136-151)
  3. per-neighbourhood ``sklearn.cluster.DBSCAN(eps, min_samples, metric)``
     with the reference's default algorithm='auto' (kd_tree for d <= 15,
     brute GEMM above) — the reference's arithmetic engine
     (R:dbscan/dbscan.py:28-29) — one task per neighbourhood in a process
     pool over every host core, as Spark ``local[*]`` runs ``mapPartitions``
     (one task per KD partition, so at most max_partitions cores are busy);
     BLAS held to one thread per task
  4. merge: local clusters linked through points core in two neighbourhoods;
     a point takes its owner neighbourhood's label (R:dbscan/dbscan.py:153-165
     intent).

bench.py runs this module as a child process (``python -m oracle.cpu_ref``),
never forked from its GPU-initialised process:

  python -m oracle.cpu_ref --config C2 --n 1000000 [--global-jobs]

prints one JSON object: rate, seconds, host cores and CPU model, and (with
--global-jobs) the rate of one global sklearn DBSCAN with n_jobs = cores, the
fastest CPU path for the same answer.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

from . import halo, kd_partition


def host_info():
    """Cores this process may use (affinity, capped by OMP_NUM_THREADS when
    set — a GPU box grants a share of a larger machine), nproc and the CPU
    model string."""
    nproc = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = nproc
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        avail = min(avail, int(omp))
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return dict(nproc=nproc, cores=max(1, avail), model=model)


def _sk_task(args):
    X, eps, ms, metric = args
    from sklearn.cluster import DBSCAN
    from threadpoolctl import threadpool_limits
    with threadpool_limits(1):
        db = DBSCAN(eps=eps, min_samples=ms, metric=metric, algorithm="auto", n_jobs=1).fit(X)
    core = np.zeros(len(X), bool)
    core[db.core_sample_indices_] = True
    return db.labels_.astype(np.int64), core


def run(X, eps, min_samples, max_partitions, metric="euclidean", workers=None):
    """Returns (labels, seconds, workers_used)."""
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components

    t0 = time.perf_counter()
    X = np.asarray(X)
    n = len(X)
    kd = kd_partition(X, max_partitions)
    _, _, members = halo(X, kd["box_lo"], kd["box_hi"], eps)
    P = len(members)
    workers = workers or host_info()["cores"]
    tasks = [(X[m].astype(np.float64), eps, min_samples, metric) for m in members]
    if workers > 1 and P > 1:
        with mp.get_context("fork").Pool(workers) as pool:
            local = pool.map(_sk_task, tasks, chunksize=1)
    else:
        local = [_sk_task(t) for t in tasks]
    # nodes = (neighbourhood, local cluster)
    base = np.zeros(P + 1, np.int64)
    for L, (lab, _) in enumerate(local):
        base[L + 1] = base[L] + (lab.max() + 1 if len(lab) else 0)
    pts, nodes = [], []
    for L, (lab, core) in enumerate(local):
        pts.append(members[L][core])
        nodes.append(base[L] + lab[core])
    pts = np.concatenate(pts) if pts else np.zeros(0, np.int64)
    nodes = np.concatenate(nodes) if nodes else np.zeros(0, np.int64)
    order = np.argsort(pts, kind="stable")
    pts, nodes = pts[order], nodes[order]
    same = pts[1:] == pts[:-1]
    nn = int(base[-1])
    g = coo_matrix((np.ones(int(same.sum())), (nodes[:-1][same], nodes[1:][same])), shape=(nn, nn))
    _, comp = connected_components(g, directed=False)
    labels = np.full(n, -1, np.int64)
    is_core = np.zeros(n, bool)
    owner = kd["owner"]
    for L, (lab, core) in enumerate(local):
        mem = members[L]
        own = (owner[mem] == L) & (lab >= 0)
        labels[mem[own]] = comp[base[L] + lab[own]]
        is_core[mem[owner[mem] == L]] = core[owner[mem] == L]
    # number components by their smallest core point, as sklearn would
    # (border points keep the cluster their neighbourhood's sklearn gave them)
    ok = labels >= 0
    if ok.any():
        first = np.full(nn, n, np.int64)
        okc = ok & is_core
        np.minimum.at(first, labels[okc], np.nonzero(okc)[0])
        used = np.unique(labels[ok])
        rank = np.empty(nn, np.int64)
        rank[used[np.argsort(first[used])]] = np.arange(len(used))
        labels[ok] = rank[labels[ok]]
    return labels, time.perf_counter() - t0, min(workers, P)


def global_sklearn(X, eps, min_samples, metric="euclidean", jobs=None):
    """One global sklearn DBSCAN (kd_tree / auto) with n_jobs threads: the
    fastest CPU path for the same labels.  Returns seconds."""
    from sklearn.cluster import DBSCAN
    t0 = time.perf_counter()
    DBSCAN(eps=eps, min_samples=min_samples, metric=metric, algorithm="auto",
           n_jobs=jobs or host_info()["cores"]).fit(np.asarray(X, np.float64))
    return time.perf_counter() - t0


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--global-jobs", action="store_true")
    args = ap.parse_args(argv)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from pypardis_amd import synth
    from . import build
    build()
    X, cfg = synth.make_config(args.config, n=args.n)
    P = cfg.get("max_partitions") or 1
    info = host_info()
    _, secs, busy = run(X, cfg["eps"], cfg["min_samples"], P)
    out = dict(n=args.n, seconds=secs, value=args.n / secs, max_partitions=P,
               workers=info["cores"], busy_max=busy, **info)
    if args.global_jobs:
        g = global_sklearn(X, cfg["eps"], cfg["min_samples"])
        out.update(global_seconds=g, global_value=args.n / g)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
