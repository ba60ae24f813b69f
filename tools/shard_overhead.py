"""Sharded-train overhead on one GPU: DBSCAN(group=WORLD).train on a 1-rank
"nccl" (RCCL) group vs the single-device train, on a config's points
(--config C2|C4, --points: the per-rank share at 8 GPUs is 12.5M of C2 or
125M of C4), with the per-phase times of distributed.train_sharded.
Diagnostic only."""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C2")
ap.add_argument("--points", type=int, default=100_000_000)
ap.add_argument("--steps", type=int, default=3)
args = ap.parse_args()
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pypardis_amd import DBSCAN, _native, synth  # noqa: E402

dev = torch.device("cuda", 0)
X, cfg = synth.make_config(args.config, n=args.points,
                           device=dev if args.config == "C4" else "cpu")
Xd = X if torch.is_tensor(X) else torch.from_numpy(X).to(dev)
del X
P = cfg.get("max_partitions") or 8
out = {"config": args.config, "points": int(Xd.shape[0])}
for name, kw in (("single", dict(n_gpus=1)), ("sharded_w1", dict(group=dist.group.WORLD))):
    m = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=P, **kw).train(Xd)
    torch.cuda.synchronize()
    stats = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=P,
                   **kw).train(Xd)
        if m.shard is not None:
            stats.append(m.shard.stats)
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / args.steps
    ctx = _native.context(0)   # one more, with the engine's per-stage events
    ctx.set_option(_native.PD_OPT_TIMING, 1)
    DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=P, **kw).train(Xd)
    torch.cuda.synchronize()
    ctx.set_option(_native.PD_OPT_TIMING, 0)
    stages = {k: round(v, 3) for k, v in ctx.timings().items()
              if v and k in ("halo", "sort", "gather", "cells", "count", "link", "merge", "roots",
                             "border", "label", "total")}
    out[name] = {"ms": ms, "stats": stats[-1] if stats else None, "stages": stages,
                 "n_clusters": m.n_clusters_}
    del m
out["ratio"] = out["sharded_w1"]["ms"] / out["single"]["ms"]
print(json.dumps(out), flush=True)
dist.destroy_process_group()
