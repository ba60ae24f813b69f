"""Latency ceiling of the count sweep.

count4_kernel tests ~18 candidates per C2 record through a dependent chain:
record -> directory word -> cell start -> candidates.  Its PMC shows neither
DRAM (hbm_frac ~0.09) nor the VALU (0.44 of issue) saturated.  This tool runs
the SAME kernel (the shipped 8-waves-per-SIMD build, PD_OPT_TIMING events
around its launch) on density-preserving C2 slices small enough that each
XCD's share of the sorted records, directory and cell starts stays in its
4 MiB L2 (0.5M / 1M / 2M points: 1-4 MB of records per XCD), where every
load of the chain is an L2 hit, at full occupancy (>= 8k waves), and reports
candidate tests per second.  The best of those rates is the kernel's ceiling
with L2-resident operands; the full 100M-point rate over it is the fraction of
that ceiling the headline kernel reaches (bench.py's latency_frac).

Candidates per run come from one extra instrumented step (PD_OPT_SWEEP_STATS,
same sweep order and early exit), the time from the shipped kernel.

  python tools/count_ceiling.py [--sizes 500000,1000000,2000000] [--full 100000000]
                                [--out gpurun_out/count_ceiling.json]
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
ap.add_argument("--sizes", default="500000,1000000,2000000")
ap.add_argument("--full", type=int, default=100_000_000)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--out", default=None)
args = ap.parse_args()

ctx = _native.context(0)
dev = torch.device("cuda:0")


def measure(n):
    X, cfg = synth.make_config("C2", n=n)
    Xd = torch.from_numpy(X).to(dev)
    del X
    eps, ms = cfg["eps"], cfg["min_samples"]
    ctx.set_option(_native.PD_OPT_SWEEP_STATS, 1)
    _native.cluster(Xd, eps, ms)
    st = ctx.timings()
    ctx.set_option(_native.PD_OPT_SWEEP_STATS, 0)
    cand, rec = st["s_count_cand"], st["records"]
    _native.cluster(Xd, eps, ms)   # warm
    ctx.set_option(_native.PD_OPT_TIMING, 1)
    t = []
    for _ in range(args.reps):
        _native.cluster(Xd, eps, ms)
        t.append(ctx.timings()["count"])
    ctx.set_option(_native.PD_OPT_TIMING, 0)
    del Xd
    torch.cuda.empty_cache()
    tc = float(np.median(t))
    return {"points": n, "records": int(rec), "candidate_tests": int(cand),
            "count_ms": tc, "count_ms_all": [round(x, 4) for x in t],
            "candidate_tests_per_s": cand / (tc * 1e-3), "records_per_s": rec / (tc * 1e-3),
            "waves": int((rec + 63) // 64)}


small = [measure(int(s)) for s in args.sizes.split(",")]
for r in small:
    print(json.dumps(r), flush=True)
full = measure(args.full)
print(json.dumps(full), flush=True)
best = max(small, key=lambda r: r["candidate_tests_per_s"])
out = {"tool": "tools/count_ceiling.py", "kernel": "count4_kernel (8 waves/SIMD build)",
       "config": "C2 density-preserving slices, max_partitions=1 (pd_cluster)",
       "l2_resident": small, "full": full,
       "ceiling_candidate_tests_per_s": best["candidate_tests_per_s"],
       "ceiling_points": best["points"],
       "latency_frac": full["candidate_tests_per_s"] / best["candidate_tests_per_s"]}
line = json.dumps(out)
print(line, flush=True)
if args.out:
    with open(args.out, "w") as f:
        f.write(line + "\n")
