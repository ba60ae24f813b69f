#!/usr/bin/env python3
"""Benchmark: BASELINE.json's metric on its headline config.

  metric : points clustered/sec (whole node), 100M 3-D pts; % HBM roofline
  config : C2 = blobs_noise(1e8, 3, side=100, 256 centres, sigma=1, 10% noise,
           seed=2), eps=0.1, min_samples=10, max_partitions=8
  step   : one full DBSCAN.train over the device-resident points — KD
           partition (3 BFS levels of GPU passes), 2·eps halo, per-neighbourhood
           DBSCAN, merge, global labels (labels stay in HBM).

  python bench.py [--gpus N --steps K --warmup W] [--points N] [--no-cpu]

For N > 1 (torch.distributed.run, one rank per GPU, RCCL) the same 100M
points are split by index over the ranks and the step is the sharded train
(pypardis_amd/distributed.py: KD levels with all-reduced moments/counts,
routing + all-to-all-v of the halo records, per-GPU clustering of its
max_partitions/N neighbourhoods, all-gather label merge, global ranks):
strong scaling, value = total points / max-over-ranks time.

Roofline object: the neighbour-count kernel (count2_kernel in engine.hip, or
count_kernel with --sweep-variant bit 0 clear).
achieved = B_nc / t, B_nc = records * (3^d*4d + 4d + 4) + (cells + 1) * 4 bytes
(340 B per record in 3-D), t = the kernel's HIP-event time on
its own stream, averaged over the timed steps.  traffic = FETCH_SIZE*2 +
WRITE_SIZE per launch from profiles/*pmc*.json when present (gfx950 FETCH_SIZE
reads half the bytes of wide streaming loads: MI355X_MICROARCH.md §HBM).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0
MFMA_BF16_PEAK_TFLOPS = 2500.0   # dense bf16 (MI355X_MICROARCH.md; no sparsity)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--points", type=int, default=None, help="override point count")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-n", type=int, default=None,
                    help="CPU baseline sample size (default 1M points; 20k for d > 15)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--link-mode", type=int, default=None, help="PD_OPT_LINK_MODE override")
    ap.add_argument("--sweep-variant", type=int, default=None,
                    help="PD_OPT_SWEEP_VARIANT override (bit 0 count, 1 link, 2 border)")
    ap.add_argument("--count-rotate", type=int, default=None,
                    help="PD_OPT_COUNT_ROTATE override (0 = count sweeps always start at the row)")
    ap.add_argument("--jump-rounds", type=int, default=None, help="PD_OPT_JUMP_ROUNDS override")
    ap.add_argument("--centre-window", type=int, default=None,
                    help="PD_OPT_CENTRE_WINDOW override (link mode 3 centre-row union)")
    ap.add_argument("--rehearse", action="store_true",
                    help="N>1 on one GPU: gloo backend, every rank on cuda:0 (correctness "
                         "rehearsal of the sharded path; not a measurement)")
    return ap.parse_args()


def default_cpu_n(d):
    return 20_000 if d > 15 else 1_000_000


def b_nc(records, cells, d):
    per = (3 ** d) * 4 * d + 4 * d + 4
    return records * per + (cells + 1) * 4, per


def load_pmc(kernel="count_kernel", config="C2"):
    """Per-launch HBM bytes of `kernel` from the newest PMC summary of the same
    config that has it (profiles/rNN_vMM_pmc[_cK]_summary.json; no _cK tag =
    C2; newest = highest (round, version))."""
    import re

    def order(f):
        m = re.search(r"r(\d+)_v(\d+)", os.path.basename(f))
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)

    def tag(f):
        m = re.search(r"pmc_(c\d)_", os.path.basename(f))
        return m.group(1).upper() if m else "C2"

    for f in sorted(glob.glob(os.path.join(HERE, "profiles", "*pmc*.json")), key=order,
                    reverse=True):
        if tag(f) != config:
            continue
        try:
            k = json.load(open(f)).get(kernel)
        except Exception:
            continue
        if k and "hbm_bytes_per_launch" in k:
            return dict(bytes_per_launch=k["hbm_bytes_per_launch"], source=os.path.basename(f))
    return None


def cpu_baseline(cfg_name, n_sample, n_full):
    import oracle
    from oracle import cpu_ref
    from pypardis_amd import synth
    X, cfg = synth.make_config(cfg_name, n=n_sample)
    oracle.build()
    labels, secs, workers = cpu_ref.run(X, cfg["eps"], cfg["min_samples"],
                                        cfg.get("max_partitions") or 1)
    out = {"value": n_sample / secs, "unit": "points/s", "cores": workers, "kind": "port",
           "seconds": secs,
           "sample": (f"{cfg_name} {'sample of the same distribution (NOT density-preserving: ' if cfg_name == 'C4' else 'density-preserving slice'}"
                      f"{'sparser than the full set, so the CPU rate is optimistic)' if cfg_name == 'C4' else ''}, {n_sample} pts, "
                      f"max_partitions={cfg.get('max_partitions')}: numpy KD + halo, "
                      f"sklearn 1.7.2 DBSCAN (algorithm='auto') per neighbourhood in a "
                      f"{workers}-process pool, 1 BLAS thread each (Spark local[*] emulation), "
                      "owner-rule merge")}
    if X.shape[1] > 15:   # brute force: O(n^2) work, the rate falls as 1/n
        out["extrapolated_full_value"] = out["value"] * n_sample / n_full
        out["sample"] += f"; brute O(n^2): at the full {n_full} pts x{n_sample / n_full:.3g}"
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse:
        local_rank = 0
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    from pypardis_amd import DBSCAN, _native, synth

    # C4 (1B points) is generated on the device: a host-side build of 1B
    # points would dominate the run; the other configs are numpy
    X, cfg = synth.make_config(args.config, n=args.points,
                               device=dev if args.config == "C4" else "cpu")
    n, d = X.shape
    eps, ms, P = cfg["eps"], cfg["min_samples"], cfg.get("max_partitions") or 1
    ctx = _native.context(local_rank)
    if args.sweep_variant is not None:
        ctx.set_option(_native.PD_OPT_SWEEP_VARIANT, args.sweep_variant)
    if args.centre_window is not None:
        ctx.set_option(_native.PD_OPT_CENTRE_WINDOW, args.centre_window)
    if args.count_rotate is not None:
        ctx.set_option(_native.PD_OPT_COUNT_ROTATE, args.count_rotate)
    if args.link_mode is not None:
        ctx.set_option(_native.PD_OPT_LINK_MODE, args.link_mode)
    if args.jump_rounds is not None:
        ctx.set_option(_native.PD_OPT_JUMP_ROUNDS, args.jump_rounds)
    if world > 1:
        from pypardis_amd.distributed import NativeOps, train_sharded
        lo, hi = rank * n // world, (rank + 1) * n // world
        Xd = X[lo:hi].clone() if torch.is_tensor(X) else \
            torch.from_numpy(np.ascontiguousarray(X[lo:hi])).to(dev)
        ops = NativeOps(dev)

        def step():
            return train_sharded(Xd, eps, ms, max_partitions=max(P, world), ops=ops)
    else:
        Xd = X if torch.is_tensor(X) else torch.from_numpy(X).to(dev)

        def step():
            return DBSCAN(eps=eps, min_samples=ms, max_partitions=P).train(Xd)
    del X

    for _ in range(args.warmup):
        m = step()
    torch.cuda.synchronize()
    ctx.set_option(_native.PD_OPT_TIMING, 1)
    stage_sum = {}
    count_ms = []
    rec = cells = 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m = step()
        t = ctx.timings()
        for k, v in t.items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
        count_ms.append(t["count"])
        rec, cells = int(t["records"]), int(t["cells_n"])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    ctx.set_option(_native.PD_OPT_TIMING, 0)
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device="cpu" if args.rehearse else dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    sweep = None
    if world == 1:   # one extra, untimed step with the instrumented sweeps
        ctx.set_option(_native.PD_OPT_SWEEP_STATS, 1)
        step()
        torch.cuda.synchronize()
        ctx.set_option(_native.PD_OPT_SWEEP_STATS, 0)
        sweep = {k: int(v) for k, v in ctx.timings().items()
                 if k.startswith("s_") or k in ("records", "core_records")}
    ms_step = 1e3 * el / args.steps
    value = n * args.steps / el
    ncl = m.n_clusters if world > 1 else m.n_clusters_

    if rank == 0:
        t_cnt = float(np.mean(count_ms))
        if d <= 4:
            alg_bytes, per = b_nc(rec, cells, d)
            achieved = alg_bytes / (t_cnt * 1e-3) / 1e9
            variant = args.sweep_variant if args.sweep_variant is not None \
                else _native.SWEEP_VARIANT_DEFAULT
            kname = "count2_kernel" if variant & 1 else "count_kernel"
            pmc = load_pmc(kname, args.config)
            roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS,
                    "traffic": pmc["bytes_per_launch"] if pmc else None, "kernel": kname,
                    "kernel_ms": t_cnt, "bytes_per_record": per, "records": rec,
                    "cells": cells, "algorithmic_bytes": alg_bytes}
            dtype = "f64"
        else:
            # dense tiles (dense.hip): the count pass's Gram tiles, 2 d flops
            # per pair over the 64 x 64 wave tiles it computes (the engine
            # reports them in cells_n; the projection window prunes the rest
            # of the n^2 pairs); the MFMA executes 3 split-bf16 products
            # with d padded to 16 ks
            ks = 1 if d <= 16 else 2 if d <= 32 else 4 if d <= 64 else 8
            n_pad = -(-n // 64) * 64
            tiles = cells if cells > 0 else (n_pad // 64) ** 2
            alg = 2.0 * d * 64 * 64 * tiles
            exe = 3 * 2.0 * 64 * 64 * 16 * ks * tiles
            achieved = alg / (t_cnt * 1e-3) / 1e12
            pmc = load_pmc("tile_kernel_m0", args.config)   # the count-pass launch
            roof = {"bound": "mfma", "achieved": achieved, "peak": MFMA_BF16_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": achieved / MFMA_BF16_PEAK_TFLOPS,
                    "traffic": pmc["bytes_per_launch"] if pmc else None,
                    "kernel": "tile_kernel (count pass)", "kernel_ms": t_cnt,
                    "algorithmic_flops": alg, "mfma_executed_flops": exe,
                    "wave_tiles": tiles, "tiles_all_pairs": (n_pad // 64) ** 2,
                    "tile_fraction": tiles / (n_pad // 64) ** 2,
                    "mfma_executed_tflops": exe / (t_cnt * 1e-3) / 1e12,
                    "mfma_utilisation": exe / (t_cnt * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFLOPS}
            dtype = "bf16x3 (split bf16 MFMA, fp32 accumulate) + f64 recheck"
        stages = {k: round(v / args.steps, 3) for k, v in stage_sum.items()
                  if k not in ("records", "cells_n", "grid_cells", "key_bits", "core_records")
                  and not k.startswith("s_")}
        # KD partition + host work around pd_train (wall time, not events)
        stages["outside_train"] = round(ms_step - stages.get("total", 0.0), 3)
        cpu = None
        if world == 1 and not args.no_cpu:
            try:
                cpu = cpu_baseline(args.config, min(args.cpu_n or default_cpu_n(d), n), n)
            except Exception as e:   # report, never fake
                cpu = {"value": None, "error": repr(e)}
        out = {
            "metric": "points clustered/sec (whole node), 100M 3-D pts, 1/2/4/8 GPUs; % HBM roofline",
            "value": value,
            "unit": "points/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic",
            "config": {"workload": f"{args.config}: "
                                   f"{'gps_skew' if args.config == 'C4' else 'blobs_noise' if d <= 4 else 'embeddings'} "
                                   f"n={n} d={d} eps={eps} min_samples={ms} max_partitions={P}",
                       "n_points": n, "d": d, "eps": eps, "min_samples": ms,
                       "max_partitions": P, "input": "fp32 device-resident",
                       "parallelism": f"kd-sharded{world}" if world > 1 else "single"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "stages_ms": stages,
            "n_clusters": ncl,
            "shard_stats": m.stats if world > 1 else None,
            "sweep_stats": sweep,
        }
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
