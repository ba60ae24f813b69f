"""Latency ceiling of the count sweep.

count4_kernel tests ~18 candidates per C2 record through a dependent chain:
record -> directory word -> cell start -> candidates.  Its PMC shows neither
DRAM (hbm_frac ~0.09) nor the VALU (0.44 of issue) saturated.  This tool runs
the SAME kernel (the shipped 8-waves-per-SIMD build) in replay mode
(PD_OPT_COUNT_REPLAY): after a normal train of a small density-preserving C2
slice (R records), the sweep runs again over m replicas of those records —
lane i sweeps record i mod R — so the launch has the full run's ~1e8 lanes
(full occupancy, steady state) while every load of the chain (the record,
its directory words, cell starts and candidates: R x ~40 B, a few MB) stays
in L2.  Candidate tests per second of that launch is the sweep's latency
ceiling; the full 100M-point rate over it is the fraction of that ceiling the
headline kernel reaches (bench.py's roofline.latency_frac).

Candidates per record come from one instrumented step (PD_OPT_SWEEP_STATS;
same sweep order and early exit), replicas test the same candidates.

  python tools/count_ceiling.py [--config C2|C1|C4] [--sizes 250000,500000,1000000,2000000]
                                [--full 100000000] [--out gpurun_out/count_ceiling.json]

C1 slices are density-preserving like C2's (synth.make_config).  C4 has no
density-preserving generator (its cities are fixed on the globe), so its
slices are cell samples of the full 1B-point set: the globe is cut into
0.05-degree cells (50 eps; cell borders cut ~8 % of the points' stencils) and
a hashed 1-in-k choice of cells is kept whole — local densities are the full
set's, and the mix of dense and sparse cells is its in expectation (compare
candidate_tests_per_record with the full run's); the full measurement is the
1B-point set itself.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from pypardis_amd import _native, synth

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C2", choices=["C2", "C1", "C4"])
ap.add_argument("--sizes", default="250000,500000,1000000,2000000")
ap.add_argument("--full", type=int, default=None)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--out", default=None)
args = ap.parse_args()

ctx = _native.context(0)
dev = torch.device("cuda:0")


_c4_full = None


def points(n):
    """(device points, eps, min_samples) of an n-point slice of the config."""
    global _c4_full
    if args.config != "C4":
        X, cfg = synth.make_config(args.config, n=n)
        return torch.from_numpy(X).to(dev), cfg["eps"], cfg["min_samples"]
    cfg = dict(synth.CONFIGS["C4"])
    if _c4_full is None:
        _c4_full, _ = synth.make_config("C4", device=dev)
    if n >= _c4_full.shape[0]:
        return _c4_full, cfg["eps"], cfg["min_samples"]
    # 0.05-degree cells (50 eps), a hashed 1-in-k choice of cells
    X = _c4_full
    cx = torch.floor((X[:, 0].double() + 180.0) / 0.05).long()
    cy = torch.floor((X[:, 1].double() + 60.0) / 0.05).long()
    cell = cy * 7200 + cx
    k = max(1, int(round(X.shape[0] / n)))
    keep = ((cell * 2654435761) % 4294967296) % k == 0
    return X[keep].contiguous(), cfg["eps"], cfg["min_samples"]


def measure(n, replay_lanes=None):
    Xd, eps, ms = points(n)
    ctx.set_option(_native.PD_OPT_SWEEP_STATS, 1)
    _native.cluster(Xd, eps, ms)
    st = ctx.timings()
    ctx.set_option(_native.PD_OPT_SWEEP_STATS, 0)
    cand, rec = int(st["s_count_cand"]), int(st["records"])
    _native.cluster(Xd, eps, ms)   # warm
    m = 0
    if replay_lanes:
        m = max(1, replay_lanes // rec)
        ctx.set_option(_native.PD_OPT_COUNT_REPLAY, m)
    ctx.set_option(_native.PD_OPT_TIMING, 1)
    t = []
    for _ in range(args.reps):
        _native.cluster(Xd, eps, ms)
        tm = ctx.timings()
        t.append(tm["count_kernel"] if m else tm["count"])
    ctx.set_option(_native.PD_OPT_TIMING, 0)
    ctx.set_option(_native.PD_OPT_COUNT_REPLAY, 0)
    del Xd
    torch.cuda.empty_cache()
    tc = float(np.median(t))
    lanes = rec * max(m, 1)
    tests = cand * max(m, 1)
    return {"points": n, "records": rec, "replicas": m, "lanes": lanes,
            "candidate_tests": tests, "candidate_tests_per_record": cand / rec,
            "count_ms": tc, "count_ms_all": [round(x, 4) for x in t],
            "candidate_tests_per_s": tests / (tc * 1e-3), "lanes_per_s": lanes / (tc * 1e-3)}


if args.full is None:
    args.full = synth.CONFIGS[args.config]["n"]
full = measure(args.full)
print(json.dumps(full), flush=True)
small = [measure(int(s), replay_lanes=full["records"]) for s in args.sizes.split(",")]
for r in small:
    print(json.dumps(r), flush=True)
best = max(small, key=lambda r: r["candidate_tests_per_s"])
out = {"tool": "tools/count_ceiling.py",
       "kernel": "count4_kernel (the shipped 8-waves/SIMD build, replay mode)",
       "config": f"{args.config} " + ("hashed 1-in-k samples of 0.05-degree cells of the full set"
                                       if args.config == "C4" else "density-preserving slices") +
                 ", max_partitions=1 (pd_cluster), replicated to the full run's lane count",
       "l2_resident_replay": small, "full": full,
       "ceiling_candidate_tests_per_s": best["candidate_tests_per_s"],
       "ceiling_points": best["points"],
       "latency_frac": full["candidate_tests_per_s"] / best["candidate_tests_per_s"]}
line = json.dumps(out)
print(line, flush=True)
if args.out:
    with open(args.out, "w") as f:
        f.write(line + "\n")
