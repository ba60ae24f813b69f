"""C4 (GPS-like skew, 2-D) at growing sizes: one warm train per size with
per-stage HIP-event times, printed as one JSON line per size (flushed), so a
slow stage shows up before the largest size runs.

  C4_SIZES=10000000,100000000 python tools/c4_probe.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pypardis_amd import DBSCAN, _native, synth

sizes = [int(s) for s in os.environ.get("C4_SIZES", "10000000").split(",")]
P = int(os.environ.get("C4_P", "8"))
reps = int(os.environ.get("C4_REPS", "2"))
dev = torch.device("cuda:0")
ctx = _native.context(0)
if os.environ.get("C4_XSUB"):
    ctx.set_option(_native.PD_OPT_XSUB, int(os.environ["C4_XSUB"]))
if os.environ.get("C4_WINDOW"):
    ctx.set_option(_native.PD_OPT_CENTRE_WINDOW, int(os.environ["C4_WINDOW"]))
if os.environ.get("C4_ROTATE"):
    ctx.set_option(_native.PD_OPT_COUNT_ROTATE, int(os.environ["C4_ROTATE"]))
if os.environ.get("C4_VARIANT"):
    ctx.set_option(_native.PD_OPT_SWEEP_VARIANT, int(os.environ["C4_VARIANT"]))
for n in sizes:
    t = time.perf_counter()
    X, cfg = synth.make_config("C4", n=n, device=dev)
    if os.environ.get("C4_NOISE"):   # experiment: another noise fraction
        X = synth.gps_skew(n, seed=cfg["seed"], noise_frac=float(os.environ["C4_NOISE"]),
                           device=dev)
    torch.cuda.synchronize()
    gen = time.perf_counter() - t
    out = {"n": n, "gen_s": round(gen, 2)}
    for rep in range(reps):
        ctx.set_option(_native.PD_OPT_TIMING, 1 if rep == reps - 1 else 0)
        torch.cuda.synchronize()
        t = time.perf_counter()
        m = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=P).train(X)
        torch.cuda.synchronize()
        out[f"train_s{rep}"] = round(time.perf_counter() - t, 4)
    ctx.set_option(_native.PD_OPT_TIMING, 0)
    tm = ctx.timings()
    out["stages_ms"] = {k: round(v, 2) for k, v in tm.items() if not k.startswith("s_")}
    if os.environ.get("C4_STATS"):
        ctx.set_option(_native.PD_OPT_SWEEP_STATS, 1)
        DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=P).train(X)
        torch.cuda.synchronize()
        ctx.set_option(_native.PD_OPT_SWEEP_STATS, 0)
        out["sweep_stats"] = {k: int(v) for k, v in ctx.timings().items() if k.startswith("s_")}
    out["n_clusters"] = m.n_clusters_
    out["core"] = int(m.core_sample_mask_.sum().item())
    out["noise"] = int((m.labels_ < 0).sum().item())
    out["part_sizes"] = torch.bincount(m.partitioner.labels.long(), minlength=P).tolist()
    print(json.dumps(out), flush=True)
    del X, m
    torch.cuda.empty_cache()
