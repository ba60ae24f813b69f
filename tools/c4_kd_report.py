"""C4 KD imbalance and halo duplication at 8 GPUs.

C4 = 1B 2-D GPS-like points, eps 0.001, min_samples 20.  The
reference's rule splits each KD box at the first of seven candidate bounds
(mean + (i-3)*0.3*std) that best balances the two halves
(R:dbscan/partition.py:58-65), which cannot follow Zipf-distributed cities.
For max_partitions P in {8, 16, 32, 64} and each placement of the KD leaves
on the GPUs (distributed.partition_ranks: 'blocks' = neighbourhood L on GPU
L * 8 // P; 'lpt' = longest-processing-time-first on the leaves' point
counts; 'ordered' = the leaves in spatial order cut into balanced runs; the
sharded train's default when P > 8 takes 'ordered' unless LPT balances more
than 5 % better), per GPU: the points it owns, the
halo records it clusters (its neighbourhoods' 2*eps boxes), and the time of
one device train over exactly those records (pd_train, the phase-A + B work
of that rank, timed with HIP events on this one MI355X).  Prints one JSON line
(also written to --out): per-GPU figures, max/mean, and the slowest GPU's
share of the summed work (1/8 = balanced).

  python tools/c4_kd_report.py [--n 1000000000] [--out profiles/r03_c4_kd.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from pypardis_amd import KDPartitioner, _native, synth
from pypardis_amd.distributed import kd_leaf_order, leaf_sizes, partition_ranks

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000_000)
ap.add_argument("--gpus", type=int, default=8)
ap.add_argument("--parts", default="8,16,32,64")
ap.add_argument("--placements", default="blocks,lpt,ordered")
ap.add_argument("--out", default=None)
args = ap.parse_args()
W = args.gpus
dev = torch.device("cuda:0")
X, cfg = synth.make_config("C4", n=args.n, device=dev)
eps, ms = cfg["eps"], cfg["min_samples"]
ctx = _native.context(0)
report = {"config": f"C4 gps_skew n={args.n} eps={eps} min_samples={ms}", "gpus": W,
          "rule": "R:dbscan/partition.py:58-65 (7 candidate bounds, best balance)", "by_P": {}}
for P, placement in [(int(p), pl) for p in args.parts.split(",")
                     for pl in args.placements.split(",")]:
    if placement != "blocks" and P <= W:
        continue   # one leaf per GPU: the blocks placement
    t0 = time.perf_counter()
    kd = KDPartitioner(X, P)
    lab = kd.labels
    ebox = np.stack([kd.bounding_boxes[L].expand(2 * eps).as_array()
                     for L in sorted(kd.bounding_boxes)])
    owned = torch.bincount(lab.long(), minlength=P).cpu().numpy()
    weights = leaf_sizes(kd.splits, int(X.shape[0]), P) if placement != "blocks" else None
    if weights is not None:
        assert np.array_equal(weights, owned), "leaf sizes from the trace = label counts"
    part_rank, local_index = partition_ranks(P, W, weights, kd_leaf_order(kd.splits),
                                             placement if weights is not None else None)
    halo, _ = _native.halo_members(X, ebox)     # records per neighbourhood
    del _
    torch.cuda.empty_cache()
    ranks = []
    for r in range(W):
        mine = [L for L in range(P) if part_rank[L] == r]
        # the rank's records: points inside any of its neighbourhoods' boxes
        inside = torch.zeros(X.shape[0], dtype=torch.bool, device=dev)
        for L in mine:
            lo = torch.from_numpy(ebox[L, 0]).to(dev, torch.float32)
            hi = torch.from_numpy(ebox[L, 1]).to(dev, torch.float32)
            inside |= ((X >= lo) & (X <= hi)).all(1)
        idx = torch.nonzero(inside).flatten()
        del inside
        Xr = X[idx].contiguous()
        li = torch.from_numpy(local_index).to(dev)
        own = torch.where(torch.from_numpy(part_rank).to(dev)[lab[idx].long()] == r,
                          li[lab[idx].long()], torch.full_like(idx, -1)).to(torch.int32)
        del idx
        lo_, hi_ = kd.data_box
        _native.train(Xr, eps, ms, _native.PD_EUCLIDEAN, ebox[mine], owner=own,
                      data_box=np.stack([lo_, hi_]))   # warm
        ctx.set_option(_native.PD_OPT_TIMING, 1)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        _native.train(Xr, eps, ms, _native.PD_EUCLIDEAN, ebox[mine], owner=own,
                      data_box=np.stack([lo_, hi_]))
        torch.cuda.synchronize()
        wall = 1e3 * (time.perf_counter() - t1)
        tm = ctx.timings()
        ctx.set_option(_native.PD_OPT_TIMING, 0)
        ranks.append({"gpu": r, "neighbourhoods": mine,
                      "owned_points": int(owned[mine].sum()),
                      "halo_records": int(tm["records"]), "train_ms": round(wall, 2),
                      "count_ms": round(tm["count"], 2), "link_ms": round(tm["link"], 2),
                      "border_ms": round(tm["border"], 2)})
        del Xr, own
        torch.cuda.empty_cache()
    pts = np.array([x["owned_points"] for x in ranks], np.float64)
    rec = np.array([x["halo_records"] for x in ranks], np.float64)
    ms_ = np.array([x["train_ms"] for x in ranks], np.float64)
    report["by_P"][f"{P}_{placement}"] = {
        "placement": placement,
        "per_gpu": ranks,
        "owned_max_over_mean": float(pts.max() / pts.mean()),
        "records_max_over_mean": float(rec.max() / rec.mean()),
        "halo_duplication": float(rec.sum() / args.n),
        "train_ms_max_over_mean": float(ms_.max() / ms_.mean()),
        "slowest_gpu_share": float(ms_.max() / ms_.sum()),
        "implied_speedup_8gpu_vs_sum": float(ms_.sum() / ms_.max()),
        "kd_and_probe_s": round(time.perf_counter() - t0, 1),
        "neighbourhood_records": [int(h) for h in halo]}
    print(json.dumps({"P": P, **{k: v for k, v in report["by_P"][f"{P}_{placement}"].items()
                                  if k not in ("per_gpu", "neighbourhood_records")}}), flush=True)
line = json.dumps(report)
print(line, flush=True)
if args.out:
    with open(args.out, "w") as f:
        f.write(line + "\n")
