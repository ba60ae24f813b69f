"""Rank body for the multi-process sharded-train tests (spawned by
tests/test_distributed.py and tests/test_gpu_parity.py; gloo on 127.0.0.1)."""
from __future__ import annotations

import os
import sys

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)


def cut_points(n, world):
    """Deliberately uneven slices (rank r gets about (r + 1) shares)."""
    w = np.arange(1, world + 1, dtype=np.float64)
    c = np.concatenate([[0], np.cumsum(w) / w.sum()])
    return (c * n).astype(np.int64)


def run_rank(rank, world, port, X, eps, min_samples, metric, P, out_dir, native,
             split_method='min_var'):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from pypardis_amd.distributed import train_sharded

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cuts = cut_points(len(X), world)
        Xi = torch.from_numpy(np.ascontiguousarray(X[cuts[rank]:cuts[rank + 1]]))
        if native:
            Xi = Xi.to("cuda:0")
            ops = None
        else:
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            from sharded_ops import OracleOps
            ops = OracleOps()
        res = train_sharded(Xi, eps, min_samples, metric=metric, max_partitions=P, ops=ops,
                            split_method=split_method)
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), gid=res.gid.cpu().numpy(),
                 labels=res.labels.cpu().numpy(), core=res.core.cpu().numpy(),
                 ncl=np.int64(res.n_clusters), splits=np.array(res.splits, np.float64),
                 ebox=res.boxes, exports=np.int64(res.stats["exports"]),
                 received=np.int64(res.stats["received"]))
    finally:
        dist.destroy_process_group()


def run_world(world, X, eps, min_samples, metric, P, out_dir, native=False, timeout=600,
              split_method='min_var'):
    """Spawn `world` ranks; return the assembled (labels, core, n_clusters,
    splits) over all points."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=run_rank,
                         args=(r, world, port, X, eps, min_samples, metric, P, out_dir, native,
                               split_method))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout)
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join()
    codes = [p.exitcode for p in procs]
    if any(c != 0 for c in codes):
        raise RuntimeError(f"rank exit codes {codes}")
    n = len(X)
    labels = np.full(n, -3, np.int64)
    core = np.zeros(n, np.uint8)
    seen = np.zeros(n, np.int64)
    ncl, splits, exports, received = set(), [], 0, 0
    for r in range(world):
        z = np.load(os.path.join(out_dir, f"r{r}.npz"))
        g = z["gid"].astype(np.int64)
        labels[g] = z["labels"]
        core[g] = z["core"]
        np.add.at(seen, g, 1)
        ncl.add(int(z["ncl"]))
        splits.append(z["splits"])
        exports += int(z["exports"])
        received += int(z["received"])
    return dict(labels=labels, core=core, seen=seen, ncl=ncl, splits=splits, exports=exports,
                received=received)
