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
             split_method='min_var', api=False, keyed=False, placement=None):
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
        extra = {}
        if api:
            # the reference API: dbscan.DBSCAN(...).train(this rank's slice)
            # inside the process group; CPU runs swap the device stages for
            # the oracle stand-in (the orchestration is the product's)
            import dbscan
            from pypardis_amd import distributed
            if not native:
                distributed.NativeOps = lambda device: ops
            data = Xi
            if keyed:   # (key, vector) records with string keys
                data = [("k%06d" % (cuts[rank] + j), v) for j, v in enumerate(Xi.cpu().numpy())]
            model = dbscan.DBSCAN(eps=eps, min_samples=min_samples,
                                  metric=["euclidean", "cityblock"][metric], max_partitions=P,
                                  device=None if native else "cpu", group="world",
                                  keep_shard_records=True)
            model.train(data)
            res = model.shard
            pairs = model.assignments()
            recs = model.data.collect()   # a collective: every rank calls it
            extra = dict(n_clusters_=np.int64(model.n_clusters_),
                         data_keys=np.array([str(k) for k, _ in recs]),
                         data_recs=np.array([v for _, v in recs]),
                         data_count=np.int64(model.data.count()),
                         boxes_api=np.array([model.bounding_boxes[L].as_array()
                                             for L in sorted(model.bounding_boxes)]),
                         assign_keys=np.array([str(k) for k, _ in pairs]),
                         assign_labels=np.array([v for _, v in pairs], np.int64),
                         count=np.int64(model.result.count()))
            loc = model.labels_.cpu().numpy(), model.core_sample_mask_.cpu().numpy()
        else:
            res = train_sharded(Xi, eps, min_samples, metric=metric, max_partitions=P, ops=ops,
                                split_method=split_method, keep_owned=True, placement=placement)
            loc = res.local_labels.cpu().numpy(), res.local_core.cpu().numpy()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), gid=res.gid.cpu().numpy(),
                 labels=res.labels.cpu().numpy(), core=res.core.cpu().numpy(),
                 ncl=np.int64(res.n_clusters), splits=np.array(res.splits, np.float64),
                 ebox=res.boxes, exports=np.int64(res.stats["exports"]),
                 received=np.int64(res.stats["received"]), loc_labels=loc[0], loc_core=loc[1],
                 lo=np.int64(cuts[rank]), placement=str(res.stats.get("placement")), **extra)
    finally:
        dist.destroy_process_group()


def run_world(world, X, eps, min_samples, metric, P, out_dir, native=False, timeout=600,
              split_method='min_var', api=False, keyed=False, placement=None):
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
                               split_method, api, keyed, placement))
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
    loc_labels = np.full(n, -3, np.int64)
    loc_core = np.zeros(n, np.uint8)
    ranks = []
    for r in range(world):
        z = np.load(os.path.join(out_dir, f"r{r}.npz"))
        ranks.append(dict(z))
        lo = int(z["lo"])
        loc_labels[lo:lo + len(z["loc_labels"])] = z["loc_labels"]
        loc_core[lo:lo + len(z["loc_core"])] = z["loc_core"]
        g = z["gid"].astype(np.int64)
        labels[g] = z["labels"]
        core[g] = z["core"]
        np.add.at(seen, g, 1)
        ncl.add(int(z["ncl"]))
        splits.append(z["splits"])
        exports += int(z["exports"])
        received += int(z["received"])
    return dict(labels=labels, core=core, seen=seen, ncl=ncl, splits=splits, exports=exports,
                received=received, loc_labels=loc_labels, loc_core=loc_core, ranks=ranks)


def _rccl_rank(port, X, eps, min_samples, P, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import dbscan
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        m = dbscan.DBSCAN(eps=eps, min_samples=min_samples, max_partitions=P,
                          group=dist.group.WORLD).train(torch.from_numpy(X).cuda())
        from pypardis_amd import distributed
        assert any(isinstance(c, distributed.RcclComm) for c in distributed._rccl_cache.values())
        np.savez(os.path.join(out_dir, "rccl.npz"), labels=m.labels_.cpu().numpy(),
                 ncl=np.int64(m.n_clusters_))
    finally:
        dist.destroy_process_group()


def run_rccl_world1(X, eps, min_samples, P, out_dir, timeout=300):
    """One rank in an "nccl" process group (spawned), DBSCAN through RCCL."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = mp.get_context("spawn").Process(target=_rccl_rank,
                                        args=(port, X, eps, min_samples, P, out_dir))
    p.start()
    p.join(timeout)
    if p.is_alive():
        p.kill()
        p.join()
    if p.exitcode != 0:
        raise RuntimeError(f"rank exit code {p.exitcode}")
    z = np.load(os.path.join(out_dir, "rccl.npz"))
    return dict(labels=z["labels"], n_clusters=int(z["ncl"]))


def _rehearsal_rank(rank, world, port, x_path, eps, min_samples, P, out_dir):
    """One rank of a full-size rehearsal: gloo on the host for the
    collectives, every rank's device stages on cuda:0, the reference API
    (DBSCAN(group='world').train(slice)) exactly as bench.py --gpus N runs it."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import time

    import torch
    import torch.distributed as dist

    import dbscan
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        X = np.load(x_path, mmap_mode="r")
        cuts = cut_points(len(X), world)
        Xi = torch.from_numpy(np.ascontiguousarray(X[cuts[rank]:cuts[rank + 1]])).to("cuda:0")
        del X
        dist.barrier()
        t0 = time.perf_counter()
        m = dbscan.DBSCAN(eps=eps, min_samples=min_samples, max_partitions=P,
                          group="world").train(Xi)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        np.savez(os.path.join(out_dir, f"h{rank}.npz"), labels=m.labels_.cpu().numpy(),
                 core=m.core_sample_mask_.cpu().numpy(), ncl=np.int64(m.n_clusters_),
                 lo=np.int64(cuts[rank]), seconds=np.float64(el),
                 received=np.int64(m.shard.stats["received"]),
                 exports=np.int64(m.shard.stats["exports_total"]))
    finally:
        dist.destroy_process_group()


def run_rehearsal(world, x_path, eps, min_samples, P, out_dir, timeout=900):
    """Spawn `world` gloo ranks sharing cuda:0 over the points saved at
    x_path; returns the assembled labels / core flags in input order."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rehearsal_rank,
                         args=(r, world, port, x_path, eps, min_samples, P, out_dir))
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
    n = len(np.load(x_path, mmap_mode="r"))
    labels = np.full(n, -3, np.int64)
    core = np.zeros(n, np.uint8)
    ncl, secs, received, exports = set(), [], 0, 0
    for r in range(world):
        z = np.load(os.path.join(out_dir, f"h{r}.npz"))
        lo = int(z["lo"])
        labels[lo:lo + len(z["labels"])] = z["labels"]
        core[lo:lo + len(z["core"])] = z["core"]
        ncl.add(int(z["ncl"]))
        secs.append(float(z["seconds"]))
        received += int(z["received"])
        exports = max(exports, int(z["exports"]))
    return dict(labels=labels, core=core, ncl=ncl, seconds=secs, received=received,
                exports=exports)
