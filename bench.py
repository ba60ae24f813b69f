#!/usr/bin/env python3
"""Benchmark: BASELINE.json's metric on its headline config.

  metric : points clustered/sec (whole node), 100M 3-D pts; % HBM roofline
  config : C2 = blobs_noise(1e8, 3, side=100, 256 centres, sigma=1, 10% noise,
           seed=2), eps=0.1, min_samples=10, max_partitions=8
  step   : one full DBSCAN.train over the device-resident points — KD
           partition (3 BFS levels of GPU passes), 2·eps halo, per-neighbourhood
           DBSCAN, merge, global labels (labels stay in HBM).

  python bench.py [--gpus N --steps K --warmup W] [--config C2|C1|C3|C4]
                  [--points N] [--no-cpu] [--no-host]

`python bench.py --gpus N` (N > 1) outside a torchrun environment starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py <same args>`
as a CHILD process (this process never imports torch or touches a GPU, and
never execs) and exits with its status; rank 0's JSON line is the line.

For N > 1 (torch.distributed.run, one rank per GPU) the same points are split
by index over the ranks and each rank calls DBSCAN(...).train(its slice) in
the process group: the sharded train over RCCL through libpardis's pd_comm_*
(KD levels with all-reduced moments/counts, routing + all-to-all-v of the halo
records, per-GPU clustering of its neighbourhoods, all-gather of the merge
exports, global ranks, labels returned to the ranks holding the points):
strong scaling, value = total points / max-over-ranks time.

Roofline object — the neighbour-count kernel (count2_kernel, engine.hip):
  frac / achieved: the algorithmic MODEL of SURVEY.md §8(d), B_nc = records *
      (3^d*4d + 4d + 4) + (cells + 1) * 4 bytes, over the kernel's HIP-event
      time on its own stream.  It charges every candidate cell's coordinates
      once per record with no cache reuse: a work model, not a DRAM reading;
  traffic / hbm_frac / l2_hit: MEASURED, from the newest PMC summary of the
      same kernel and config (profiles/rNN_vMM_pmc[_cK]_summary.json, made by
      tools/pmc_run.sh): traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per
      launch (gfx950 FETCH_SIZE counts half the bytes of wide reads:
      MI355X_MICROARCH.md §HBM), hbm_frac = traffic / kernel time / 8 TB/s;
  limiter: candidate tests per record and per second (the kernel's work unit).
stage_roofline gives the link stage the same measured accounting.

Other legs (single process): cpu_baseline — the reference's algorithm on the
host cores, in a child process started before the GPU is touched
(python -m oracle.cpu_ref); host_input — the same train from host numpy (H2D
inside the step) and from a list of (key, vector) records.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0
MFMA_BF16_PEAK_TFLOPS = 2500.0   # dense bf16 (MI355X_MICROARCH.md; no sparsity)
MFMA_FP8_PEAK_TFLOPS = 5000.0    # dense e4m3 (32x32x64 f8f6f4: 2x bf16 per clock)
BASELINE_METRIC = "points clustered/sec (whole node), 100M 3-D pts, 1/2/4/8 GPUs; % HBM roofline"
LINK_KERNELS = ("init_kernel", "window_uf_kernel", "cell_word_root_kernel",
                "mid_cell_word_root_kernel", "big_cell_word_root_kernel", "verify_screen_kernel",
                "flag_list_kernel", "cell_verify_kernel", "pair_kernel")
L2_PEAK_GBS = 34500.0            # MI355X_MICROARCH.md §L2: ~34.5 TB/s aggregate


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--points", type=int, default=None, help="override point count")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-host", action="store_true", help="skip the host-input legs")
    ap.add_argument("--cpu-n", type=int, default=None,
                    help="CPU baseline sample size (default 1M; 10M for C4; 20k for d > 15)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--dir-budget", type=int, default=None,
                    help="PD_OPT_DIR_BUDGET override (bytes of the eps-grid directory)")
    ap.add_argument("--count-rotate", type=int, default=None,
                    help="PD_OPT_COUNT_ROTATE override (0 = count sweeps always start at the row)")
    ap.add_argument("--dense-screen", type=int, default=None,
                    help="PD_OPT_DENSE_SCREEN override (1 e4m3, 0 bf16 hi.hi)")
    ap.add_argument("--dir-paged", type=int, default=None,
                    help="PD_OPT_DIR_PAGED override (1 paged, 0 flat, -1 auto)")
    ap.add_argument("--label-buckets", type=int, default=None,
                    help="PD_OPT_LABEL_BUCKETS override (0: one scattered label write per record)")
    ap.add_argument("--centre-window", type=int, default=None,
                    help="PD_OPT_CENTRE_WINDOW override (link window length)")
    ap.add_argument("--xsub", type=int, default=None,
                    help="PD_OPT_XSUB override (axis-0 sub-cells per eps)")
    ap.add_argument("--halo-passes", type=int, default=None,
                    help="PD_OPT_HALO_PASSES override (1 single pass, 2 tile counts + scan)")
    ap.add_argument("--kd-fuse", type=int, default=None,
                    help="PD_OPT_KD_FUSE override (1: counts + children's moments in one pass)")
    ap.add_argument("--verify-fused", type=int, default=None,
                    help="PD_OPT_VERIFY_FUSED override (1: cell verify over every cell, screen inline)")
    ap.add_argument("--halo-tree", type=int, default=None,
                    help="PD_OPT_HALO_TREE override (1: box tests only near split planes)")
    ap.add_argument("--kd-replay", type=int, default=None,
                    help="PD_OPT_KD_REPLAY override (1: KD passes replay the splits, no labels)")
    ap.add_argument("--rehearse", action="store_true",
                    help="N>1 on one GPU: gloo backend, every rank on cuda:0 (correctness "
                         "rehearsal of the sharded path; not a measurement)")
    return ap.parse_args()


def default_cpu_n(cfg_name, d):
    if d > 15:
        return 20_000
    return 10_000_000 if cfg_name == "C4" else 1_000_000


def b_nc(records, cells, d):
    per = (3 ** d) * 4 * d + 4 * d + 4
    return records * per + (cells + 1) * 4, per


def _order(f):
    m = re.search(r"r(\d+)_v(\d+)", os.path.basename(f))
    return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)


def load_pmc(config="C2"):
    """Newest PMC summary of `config` (profiles/rNN_vMM_pmc[_cK]_summary.json;
    no _cK tag = C2; newest = highest (round, version)): (dict, file name)."""
    def tag(f):
        m = re.search(r"pmc_(c\d)_", os.path.basename(f))
        return m.group(1).upper() if m else "C2"

    for f in sorted(glob.glob(os.path.join(HERE, "profiles", "*pmc*summary*.json")), key=_order,
                    reverse=True):
        if tag(f) != config:
            continue
        try:
            return json.load(open(f)), os.path.basename(f)
        except Exception:
            continue
    return None, None


def load_ceiling(config="C2"):
    """Newest count-sweep latency ceiling of `config`
    (profiles/rNN_vMM_count_ceiling[_cK].json, tools/count_ceiling.py): the
    shipped count kernel on L2-resident slices of that config (its "config"
    field names it)."""
    fs = sorted(glob.glob(os.path.join(HERE, "profiles", "*count_ceiling*.json")), key=_order)
    for f in reversed(fs):
        try:
            c = json.load(open(f))
        except Exception:
            continue
        if str(c.get("config", "C2")).split()[0] == config:
            return c, os.path.basename(f)
    return None, None


def pmc_fields(k):
    """Measured per-launch HBM bytes and L2 hit rate from one kernel's counters.
    hbm_bytes doubles FETCH_SIZE (the guide's gfx950 correction, calibrated
    for 16-B-per-lane streaming reads); hbm_bytes_raw does not — for narrower
    gathers the true figure lies between the two."""
    out = {}
    if "FETCH_SIZE" in k or "WRITE_SIZE" in k:
        out["hbm_bytes"] = (2 * k.get("FETCH_SIZE", 0.0) + k.get("WRITE_SIZE", 0.0)) * 1024
        out["hbm_bytes_raw"] = (k.get("FETCH_SIZE", 0.0) + k.get("WRITE_SIZE", 0.0)) * 1024
    h, m = k.get("TCC_HIT_sum"), k.get("TCC_MISS_sum")
    if h is not None and m is not None and h + m > 0:
        out["l2_hit"] = h / (h + m)
    return out


def calibration():
    fs = sorted(glob.glob(os.path.join(HERE, "profiles", "*cpu_calibration*.json")), key=_order)
    if not fs:
        return None
    try:
        c = json.load(open(fs[-1]))
    except Exception:
        return None
    c["source"] = os.path.basename(fs[-1])
    return c


def cpu_baseline(cfg_name, n_sample, n_full, d):
    """The reference's algorithm on the host cores (oracle/cpu_ref.py), in a
    child process started before this process touches the GPU."""
    cmd = [sys.executable, "-m", "oracle.cpu_ref", "--config", cfg_name, "--n", str(n_sample)]
    if d <= 15:
        cmd.append("--global-jobs")
    p = subprocess.Popen(cmd, cwd=HERE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    t0 = time.time()
    while True:   # a heartbeat on stderr while the host cores work
        try:
            out, err = p.communicate(timeout=30)
            break
        except subprocess.TimeoutExpired:
            if time.time() - t0 > 1800:
                p.kill()
                out, err = p.communicate()
                return {"value": None, "error": "CPU baseline timed out (1800 s)"}
            print(f"[bench] CPU baseline running ({time.time() - t0:.0f} s)", file=sys.stderr,
                  flush=True)
    if p.returncode != 0:
        return {"value": None, "error": (err or out)[-2000:]}
    c = json.loads(out.strip().splitlines()[-1])
    if cfg_name == "C4":
        desc = ("sample of the same distribution at 1% of the full size; its cities are "
                "100x sparser, so neighbour lists are 100x shorter than at 1B: the rate is "
                "an optimistic extrapolation to the full set")
    else:
        desc = "density-preserving slice"
    out = {"value": c["value"], "unit": "points/s", "cores": c["workers"], "kind": "port",
           "seconds": c["seconds"], "nproc": c["nproc"], "cpu_model": c["model"],
           "sample": (f"{cfg_name} {desc}, {n_sample} pts, max_partitions={c['max_partitions']}: "
                      f"numpy KD + halo, sklearn DBSCAN (algorithm='auto') per neighbourhood in "
                      f"a {c['workers']}-process pool (Spark local[*] runs one task per KD "
                      f"partition, so at most {c['busy_max']} are busy), 1 BLAS thread each, "
                      f"owner-rule merge; host: {c['nproc']} CPUs visible ({c['model']}), "
                      f"{c['workers']} usable")}
    if "global_value" in c:
        out["global_sklearn_value"] = c["global_value"]
        out["global_sklearn_note"] = (f"one global sklearn DBSCAN, n_jobs={c['workers']}: the "
                                      "fastest CPU path to the same labels (not the reference's "
                                      "partitioned pipeline)")
    cal = calibration()
    if cal:
        out["calibration"] = {k: cal[k] for k in ("n", "reference_seconds",
                                                  "cpu_ref_seconds_1_worker",
                                                  "ratio_reference_over_cpu_ref", "source")}
        out["sample"] += (f"; calibration ({cal['n']} pts, one process each, build container): "
                          f"the reference itself {cal['reference_seconds']:.1f} s, this port "
                          f"{cal['cpu_ref_seconds_1_worker']:.1f} s")
    if d > 15:   # brute force: O(n^2) work, the rate falls as 1/n
        out["extrapolated_full_value"] = out["value"] * n_sample / n_full
        out["sample"] += f"; brute O(n^2): at the full {n_full} pts x{n_sample / n_full:.3g}"
    elif cfg_name == "C4":
        out["extrapolated"] = True
    return out


def grid_roofline(rec, cells, d, t_cnt, sweep, pmc, pmc_src, stages, cfg_name="C2"):
    alg_bytes, per = b_nc(rec, cells, d)
    if not t_cnt > 0:   # no kernel time recorded (never expected): no rate, no crash
        t_cnt = 1e30
    achieved = alg_bytes / (t_cnt * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "frac_kind": "model: algorithmic B_nc, every candidate cell read once per record",
            "traffic": None, "kernel": "count4_kernel", "kernel_ms": t_cnt,
            "bytes_per_record": per, "records": rec, "cells": cells,
            "algorithmic_bytes": alg_bytes, "pmc_source": pmc_src}
    k = (pmc or {}).get("count4_kernel") or (pmc or {}).get("count2_kernel")
    if k:
        f = pmc_fields(k)
        if "hbm_bytes" in f:
            roof["traffic"] = f["hbm_bytes"]
            roof["traffic_raw"] = f["hbm_bytes_raw"]
            roof["traffic_note"] = ("2*FETCH_SIZE + WRITE_SIZE per launch (the guide's gfx950 "
                                   "correction for 16-B streaming reads; this kernel's "
                                   "candidate loads are narrower, so the true DRAM bytes lie "
                                   "between traffic_raw and traffic)")
            roof["hbm_frac"] = f["hbm_bytes"] / (t_cnt * 1e-3) / (HBM_PEAK_GBS * 1e9)
        if "l2_hit" in f:
            roof["l2_hit"] = f["l2_hit"]
        req = k.get("TCP_TCC_READ_REQ_sum")
        if req:
            # L1 -> L2 read requests of 64-128 B (request size uncalibrated):
            # the L2 fraction at 128 B is an upper bound
            roof["l2_read_requests"] = req
            roof["l2_frac"] = req * 128 / (t_cnt * 1e-3) / (L2_PEAK_GBS * 1e9)
            roof["l2_frac_at_64B"] = req * 64 / (t_cnt * 1e-3) / (L2_PEAK_GBS * 1e9)
            roof["l2_note"] = ("TCP_TCC_READ_REQ_sum x 128 B (x 64 B) per launch / kernel time "
                               "/ the guide's 34.5 TB/s aggregate L2 rate")
    if sweep and sweep.get("s_count_cand") and rec:
        cand = sweep["s_count_cand"]
        roof["limiter"] = {
            "kind": "issue/latency of the candidate tests (gathers served by L2), not DRAM "
                    "bandwidth: compare hbm_frac with frac",
            "candidate_tests": cand, "candidate_tests_per_record": cand / rec,
            "candidate_tests_per_s": cand / (t_cnt * 1e-3),
            "records_per_s": rec / (t_cnt * 1e-3)}
        ceil, ceil_src = load_ceiling(cfg_name)
        if not (ceil and ceil.get("ceiling_candidate_tests_per_s")):
            # each config's sweep (its candidate lists and cell occupancy)
            # needs its own ceiling
            roof["latency_frac"] = None
            roof["latency_note"] = f"no latency ceiling measured for {cfg_name}"
        else:
            # the same kernel with every load of its chain an L2 hit
            roof["latency_frac"] = (cand / (t_cnt * 1e-3)) / ceil["ceiling_candidate_tests_per_s"]
            roof["latency_ceiling"] = {
                "candidate_tests_per_s": ceil["ceiling_candidate_tests_per_s"],
                "points": ceil.get("ceiling_points"), "source": ceil_src,
                "note": f"count4_kernel on a {cfg_name} slice ({ceil.get('config', '')}) "
                        "whose records, directory and cell starts fit each XCD's L2, "
                        "replicated to the full run's lanes (tools/count_ceiling.py)"}
    stage = None
    if pmc and stages.get("link"):
        kb = {}
        for name in LINK_KERNELS:
            if name in pmc:
                f = pmc_fields(pmc[name])
                if "hbm_bytes" in f:
                    kb[name] = f["hbm_bytes"]
        if kb:
            tot = sum(kb.values())
            stage = {"stage": "link", "ms": stages["link"], "hbm_bytes": tot,
                     "achieved_gbs": tot / (stages["link"] * 1e-3) / 1e9,
                     "hbm_frac": tot / (stages["link"] * 1e-3) / (HBM_PEAK_GBS * 1e9),
                     "kernels_hbm_bytes": kb,
                     "bound": "latency of dependent union-find gathers and atomics",
                     "pmc_source": pmc_src}
    return roof, stage


def dense_roofline(n, d, t_cnt, cells, pmc, pmc_src, refined=None, screen=1):
    # dense tiles (dense.hip): the count pass's Gram tiles, 2 d flops per pair
    # over the 64 x 64 wave tiles it computes (the engine reports them in
    # cells_n; the projection window prunes the rest of the n^2 pairs).  The
    # MFMA executes the screen on every tile — e4m3 32x32x64 (d padded to 64,
    # at the fp8 rate; screen 1, the default) or bf16 hi.hi (d padded to 16
    # ks) — and the split-bf16 product on the tiles the screen keeps
    # (grid_cells): from scratch after the e4m3 screen (three products), the
    # two remaining ones after the hi.hi screen.  `frac` prices the
    # algorithmic flops at the bf16 peak (the exact product's dtype; the
    # fp8-peak fraction is beside it); `mfma_utilisation` is the MFMA pipe
    # time those executed flops take at their dtype's peak over the kernel time
    ks = 1 if d <= 16 else 2 if d <= 32 else 4 if d <= 64 else 8
    ks8 = (ks + 3) // 4
    n_pad = -(-n // 64) * 64
    tiles = cells if cells > 0 else (n_pad // 64) ** 2
    refined = tiles if refined is None else refined
    alg = 2.0 * d * 64 * 64 * tiles
    if screen == 1:
        exe8 = 2.0 * 64 * 64 * 64 * ks8 * tiles
        exe16 = 2.0 * 64 * 64 * 16 * ks * 3 * refined
    else:
        exe8 = 0.0
        exe16 = 2.0 * 64 * 64 * 16 * ks * (tiles + 2 * refined)
    if not t_cnt > 0:   # no kernel time recorded (never expected): no rate, no crash
        t_cnt = 1e30
    achieved = alg / (t_cnt * 1e-3) / 1e12
    pipe_s = exe8 / (MFMA_FP8_PEAK_TFLOPS * 1e12) + exe16 / (MFMA_BF16_PEAK_TFLOPS * 1e12)
    roof = {"bound": "mfma", "achieved": achieved, "peak": MFMA_BF16_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": achieved / MFMA_BF16_PEAK_TFLOPS,
            "frac_kind": "algorithmic: 2 d flops per computed pair, at the bf16 peak",
            "frac_fp8_peak": achieved / MFMA_FP8_PEAK_TFLOPS,
            "screen": "e4m3 32x32x64" if screen == 1 else "bf16 hi.hi",
            "traffic": None,
            "kernel": "tile_kernel (count pass)", "kernel_ms": t_cnt,
            "algorithmic_flops": alg, "mfma_executed_flops_fp8": exe8,
            "mfma_executed_flops_bf16": exe16,
            "wave_tiles": tiles, "refined_tiles": refined,
            "tiles_all_pairs": (n_pad // 64) ** 2,
            "tile_fraction": tiles / (n_pad // 64) ** 2,
            "mfma_utilisation": pipe_s / (t_cnt * 1e-3),
            "pmc_source": pmc_src}
    k = (pmc or {}).get("tile_kernel_m0")
    if k:
        f = pmc_fields(k)
        roof["traffic"] = f.get("hbm_bytes")
        if "hbm_bytes" in f:
            roof["hbm_frac"] = f["hbm_bytes"] / (t_cnt * 1e-3) / (HBM_PEAK_GBS * 1e9)
        if "l2_hit" in f:
            roof["l2_hit"] = f["l2_hit"]
    return roof


def train_roofline(pmc, pmc_src, ms_step):
    """The whole train's measured HBM bytes (every kernel's per-launch bytes
    from the PMC summary x its launches per train) over the step time: the
    step's own fraction of the 8 TB/s peak, beside the one-kernel roofline."""
    if not pmc or "_meta" not in pmc or not ms_step:
        return None
    tot, per = 0.0, {}
    for k, v in pmc.items():
        if k.startswith("_") or "hbm_bytes_per_launch" not in v:
            continue
        b = v["hbm_bytes_per_launch"] * v.get("dispatches_per_train", 0.0)
        if b > 0:
            per[k] = b
            tot += b
    if tot <= 0:
        return None
    top = dict(sorted(per.items(), key=lambda kv: -kv[1])[:8])
    return {"bytes_per_train": tot, "achieved_gbs": tot / (ms_step * 1e-3) / 1e9,
            "peak": HBM_PEAK_GBS, "frac": tot / (ms_step * 1e-3) / (HBM_PEAK_GBS * 1e9),
            "kind": "measured: sum over every kernel of (2*FETCH_SIZE + WRITE_SIZE) x launches "
                    "per train, over ms_per_step",
            "top_kernels_bytes": top, "pmc_source": pmc_src}


def host_legs(DBSCAN, eps, ms, P, Xh):
    """The same train from host memory: a numpy array (H2D inside the step),
    and a list of (key, vector) records — the reference's RDD element form
    (R:dbscan/dbscan.py:104-109) — with the ingest (as_points) timed apart."""
    import torch
    from pypardis_amd._data import as_points
    out = {}
    DBSCAN(eps=eps, min_samples=ms, max_partitions=P).train(Xh)   # warm
    torch.cuda.synchronize()
    reps = 2
    t0 = time.perf_counter()
    for _ in range(reps):
        DBSCAN(eps=eps, min_samples=ms, max_partitions=P).train(Xh)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    out["numpy"] = {"points": len(Xh), "ms_per_step": 1e3 * t, "value": len(Xh) / t,
                    "note": "DBSCAN.train(numpy array): H2D copy of the points inside the step"}
    nr = min(len(Xh), 1_000_000)
    recs = list(zip(range(nr), Xh[:nr]))
    t0 = time.perf_counter()
    pts = as_points(recs)
    torch.cuda.synchronize()
    t_in = time.perf_counter() - t0
    t0 = time.perf_counter()
    DBSCAN(eps=eps, min_samples=ms, max_partitions=P).train(pts)
    torch.cuda.synchronize()
    t_tr = time.perf_counter() - t0
    out["records"] = {"records": nr, "ingest_s": t_in, "ingest_records_per_s": nr / t_in,
                      "train_s": t_tr, "value": nr / (t_in + t_tr),
                      "note": "list of (int key, ndarray) records: vectorised unzip + stack + "
                              "H2D (ingest), then train"}
    return out


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n, argv):
    """One process per GPU for `--gpus n` without torchrun around us: the
    rank processes come from torch.distributed.run started as a child (no
    exec; this process has not imported torch), each with WORLD_SIZE / RANK /
    LOCAL_RANK set, so they run main()'s rank path.  Returns the child's exit
    status (rank 0 prints the JSON line to the stdout we share)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    print(f"[bench] launching {n} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env, cwd=HERE)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" in os.environ and args.gpus not in (1, world):
        print(f"[bench] --gpus {args.gpus} inside a torchrun job of {world} ranks: "
              f"the job's {world} ranks are measured", file=sys.stderr, flush=True)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    from pypardis_amd import synth
    cfgd = synth.CONFIGS[args.config]
    n_cfg = args.points or cfgd["n"]
    d_cfg = cfgd["d"]
    cpu = None
    if world == 1 and not args.no_cpu:
        # before the GPU is initialised, so the child inherits no HIP state
        try:
            cpu = cpu_baseline(args.config,
                               min(args.cpu_n or default_cpu_n(args.config, d_cfg), n_cfg),
                               n_cfg, d_cfg)
        except Exception as e:   # report, never fake
            cpu = {"value": None, "error": repr(e)}

    import torch
    import torch.distributed as dist

    if args.rehearse:
        local_rank = 0
    if world > 1 and local_rank >= torch.cuda.device_count():
        raise SystemExit(f"[bench] rank {rank}: local rank {local_rank} but "
                         f"{torch.cuda.device_count()} GPU(s) visible (--rehearse runs every "
                         f"rank on cuda:0 over gloo)")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    from pypardis_amd import DBSCAN, _native

    # C4 (1B points) is generated on the device: a host-side build of 1B
    # points would dominate the run; the other configs are numpy
    X, cfg = synth.make_config(args.config, n=args.points,
                               device=dev if args.config == "C4" else "cpu")
    n, d = X.shape
    eps, ms, P = cfg["eps"], cfg["min_samples"], cfg.get("max_partitions") or 1
    ctx = _native.context(local_rank)
    for opt, val in ((_native.PD_OPT_CENTRE_WINDOW, args.centre_window),
                     (_native.PD_OPT_COUNT_ROTATE, args.count_rotate),
                     (_native.PD_OPT_DIR_BUDGET, args.dir_budget),
                     (_native.PD_OPT_LABEL_BUCKETS, args.label_buckets),
                     (_native.PD_OPT_DIR_PAGED, args.dir_paged),
                     (_native.PD_OPT_DENSE_SCREEN, args.dense_screen),
                     (_native.PD_OPT_XSUB, args.xsub),
                     (_native.PD_OPT_HALO_PASSES, args.halo_passes),
                     (_native.PD_OPT_KD_FUSE, args.kd_fuse),
                     (_native.PD_OPT_VERIFY_FUSED, args.verify_fused),
                     (_native.PD_OPT_HALO_TREE, args.halo_tree),
                     (_native.PD_OPT_KD_REPLAY, args.kd_replay)):
        if val is not None:
            ctx.set_option(opt, val)
    Xh = None
    if world > 1:   # this rank's slice; DBSCAN.train in the process group shards
        lo, hi = rank * n // world, (rank + 1) * n // world
        Xd = X[lo:hi].clone() if torch.is_tensor(X) else \
            torch.from_numpy(np.ascontiguousarray(X[lo:hi])).to(dev)
    else:
        Xd = X if torch.is_tensor(X) else torch.from_numpy(X).to(dev)
        Xh = None if torch.is_tensor(X) else X
    del X

    grp = {"group": dist.group.WORLD} if world > 1 else {}

    def step():
        return DBSCAN(eps=eps, min_samples=ms, max_partitions=max(P, world), **grp).train(Xd)

    for _ in range(args.warmup):
        m = step()
    torch.cuda.synchronize()
    ctx.set_option(_native.PD_OPT_TIMING, 1)
    stage_sum = {}
    count_ms = []
    rec = cells = 0
    directory = None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m = step()
        t = ctx.timings()
        for k, v in t.items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
        # the roofline kernel's own event time (dense: the tile kernel alone;
        # grid: the count stage is the count2 launch)
        count_ms.append(t["count_kernel"] if t.get("count_kernel", 0) > 0 else t["count"])
        rec, cells, gcells = int(t["records"]), int(t["cells_n"]), int(t["grid_cells"])
        directory = {"paged": bool(t["dir_paged"]), "words": int(t["dir_words"]),
                     "key_bits": int(t["key_bits"])}
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
        # the window union tallies candidates, hits and unions only (the
        # other s_link_* slots belonged to the retired link modes)
        for k in ("s_link_core", "s_link_same", "s_link_find_same", "s_count_staged"):
            if not sweep.get(k):
                sweep.pop(k, None)
    ms_step = 1e3 * el / args.steps
    value = n * args.steps / el
    ncl = m.n_clusters_
    shard_stats = m.shard.stats if m.shard is not None else None
    rccl_ranks = None
    if world > 1:
        # the slowest rank's per-phase times, and the rank count RCCL itself
        # reports for the communicator the train ran on (0: gloo rehearsal)
        allst = [None] * world
        dist.all_gather_object(allst, (el, shard_stats))
        slow = max(range(world), key=lambda r: allst[r][0])
        shard_stats = dict(allst[slow][1] or {}, rank=slow,
                           rank_seconds=[round(a[0], 4) for a in allst])
        if not args.rehearse:
            from pypardis_amd import distributed
            comm = distributed.make_comm(dist.group.WORLD, dev)
            rccl_ranks = comm.comm.size()[0] if hasattr(comm, "comm") else 0
        else:
            rccl_ranks = 0
    del m

    host = None
    if world == 1 and not args.no_host and d <= 4:
        host = host_legs(DBSCAN, eps, ms, P, Xh if Xh is not None else Xd.cpu().numpy())

    if rank == 0:
        t_cnt = float(np.mean(count_ms))
        stages = {k: round(v / args.steps, 3) for k, v in stage_sum.items()
                  if k not in ("records", "cells_n", "grid_cells", "key_bits", "core_records",
                               "dir_paged", "dir_words")
                  and not k.startswith("s_")}
        if not stages.get("count_kernel"):
            stages.pop("count_kernel", None)   # dense path only
        # KD partition + host work around pd_train (wall time, not events)
        stages["outside_train"] = round(ms_step - stages.get("total", 0.0), 3)
        pmc, pmc_src = load_pmc(args.config)
        stage_roof = None
        if d <= 4:
            roof, stage_roof = grid_roofline(rec, cells, d, t_cnt, sweep, pmc, pmc_src, stages,
                                             args.config)
            dtype = f"{'f32' if Xd.dtype == torch.float32 else 'f64'} coords, f64 predicate"
        else:
            roof = dense_roofline(n, d, t_cnt, cells, pmc, pmc_src, refined=gcells,
                                  screen=1 if args.dense_screen is None else args.dense_screen)
            dtype = ("e4m3 screen (32x32x64 f8f6f4)" if args.dense_screen in (None, 1)
                     else "bf16 hi.hi screen") + \
                ", split-bf16 x3 where it keeps a pair (fp32 accumulate), f64 recheck"
        if args.config == "C2" and n == cfgd["n"]:
            metric = BASELINE_METRIC
        else:
            metric = (f"points clustered/sec (whole node), {n} {d}-D pts ({args.config}); "
                      f"% {'HBM' if d <= 4 else 'MFMA'} roofline")
        kind = {"C4": "gps_skew"}.get(args.config, "blobs_noise" if d <= 4 else "embeddings")
        out = {
            "metric": metric,
            "value": value,
            "unit": "points/s",
            "n_gpus": world,
            "rccl_ranks": rccl_ranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic",
            "config": {"workload": f"{args.config}: {kind} n={n} d={d} eps={eps} "
                                   f"min_samples={ms} max_partitions={P}",
                       "n_points": n, "d": d, "eps": eps, "min_samples": ms,
                       "max_partitions": P,
                       "input": f"{str(Xd.dtype).replace('torch.', '')} device-resident",
                       "parallelism": f"kd-sharded{world}" if world > 1 else "single",
                       "transport": (("gloo rehearsal, every rank on cuda:0" if args.rehearse
                                      else "RCCL (pd_comm)") if world > 1 else None)},
            "roofline": roof,
            "train_roofline": train_roofline(pmc, pmc_src, ms_step) if world == 1 else None,
            "stage_roofline": stage_roof,
            "cpu_baseline": cpu,
            "host_input": host,
            "stages_ms": stages,
            "n_clusters": ncl,
            "shard_stats": shard_stats,
            "sweep_stats": sweep,
            "directory": directory if d <= 4 else None,
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
