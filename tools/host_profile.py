"""Host time of one DBSCAN.train step (C2 by default): where the Python and
C++ host code spend the time the GPU waits for between the KD build and the
fused train.  Wraps _native.kd_build / _native.train_tree with wall-clock
stamps (both return after a stream sync, so their spans include GPU time)
and runs cProfile over a few steps.

  python tools/host_profile.py [--config C2] [--steps 5] [--out FILE]
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pypardis_amd import DBSCAN, _native, synth

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C2")
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--out", default=None)
args = ap.parse_args()

X, cfg = synth.make_config(args.config)
Xd = torch.from_numpy(X).cuda()
del X
stamps = {}


def wrap(name):
    f = getattr(_native, name)

    def g(*a, **k):
        stamps.setdefault(name + "_in", []).append(time.perf_counter())
        r = f(*a, **k)
        stamps.setdefault(name + "_out", []).append(time.perf_counter())
        return r
    setattr(_native, name, g)


wrap("kd_build")
wrap("train_tree")


def step():
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"],
           max_partitions=cfg["max_partitions"]).train(Xd)
    torch.cuda.synchronize()
    stamps.setdefault("step_in", []).append(t0)
    stamps.setdefault("step_out", []).append(time.perf_counter())


for _ in range(2):
    step()
for k in list(stamps):
    stamps[k].clear()
pr = cProfile.Profile()
pr.enable()
for _ in range(args.steps):
    step()
pr.disable()


def med(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


res = {
    "config": args.config, "steps": args.steps,
    "step_ms": med([b - a for a, b in zip(stamps["step_in"], stamps["step_out"])]) * 1e3,
    "before_kd_ms": med([b - a for a, b in zip(stamps["step_in"], stamps["kd_build_in"])]) * 1e3,
    "kd_build_ms": med([b - a for a, b in zip(stamps["kd_build_in"], stamps["kd_build_out"])]) * 1e3,
    "kd_to_train_ms": med([b - a for a, b in zip(stamps["kd_build_out"], stamps["train_tree_in"])]) * 1e3,
    "train_tree_ms": med([b - a for a, b in zip(stamps["train_tree_in"], stamps["train_tree_out"])]) * 1e3,
    "after_train_ms": med([b - a for a, b in zip(stamps["train_tree_out"], stamps["step_out"])]) * 1e3,
}
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(json.dumps(res), flush=True)
print(s.getvalue())
if args.out:
    with open(args.out, "w") as f:
        f.write(json.dumps(res) + "\n" + s.getvalue())
