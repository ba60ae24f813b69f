"""Sharded-train overhead on one GPU: DBSCAN(group=WORLD).train on a 1-rank
"nccl" (RCCL) group vs the single-device train, C2 (--points), with the
per-phase host laps of distributed.train_sharded.  Diagnostic only."""
import argparse
import json
import os
import time

import sys

import torch
import torch.distributed as dist

ap = argparse.ArgumentParser()
ap.add_argument("--points", type=int, default=100_000_000)
ap.add_argument("--steps", type=int, default=3)
args = ap.parse_args()
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pypardis_amd import DBSCAN, synth  # noqa: E402

X, cfg = synth.make_config("C2", n=args.points)
Xd = torch.from_numpy(X).cuda()
out = {}
for name, kw in (("single", dict(n_gpus=1)), ("sharded_w1", dict(group=dist.group.WORLD))):
    m = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=8, **kw).train(Xd)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=8, **kw).train(Xd)
    torch.cuda.synchronize()
    out[name] = {"ms": 1e3 * (time.perf_counter() - t0) / args.steps,
                 "stats": getattr(m.shard, "stats", None) if m.shard is not None else None,
                 "n_clusters": m.n_clusters_}
print(json.dumps(out))
dist.destroy_process_group()
