"""Time the KD partition passes in isolation on C2 (100M 3-D points): the
fused first level (bbox + moments), the counts pass, the split + moments
passes of levels 1 and 2, the final split, and torch's X.sum() / copy as
streaming references.  HIP events on the current stream, mean of 10.

  python tools/kd_bench.py [n]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pypardis_amd import _native, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
X, cfg = synth.make_config("C2", n=n)
Xd = torch.from_numpy(X).cuda()
del X
lab = torch.zeros(n, dtype=torch.int32, device="cuda")
ctx = _native.context()
GB = Xd.numel() * 4 / 1e9


def timeit(f, reps=10):
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


res = {}
res["torch_sum"] = timeit(lambda: Xd.sum())
Y = torch.empty_like(Xd)
res["torch_copy"] = timeit(lambda: Y.copy_(Xd))
del Y
res["level0_bbox_moments"] = timeit(lambda: _native.kd_pass(Xd, lab, None, [0], True, True,
                                                            ctx=ctx))
# labels for two halves / quarters
mid = float(np.median(Xd[:1_000_000, 0].cpu().numpy()))
lab.zero_()
_native.kd_split(Xd, lab, [0], [0], [mid], [1], ctx=ctx)
bounds = np.tile(np.linspace(-40, 40, 7), (2, 1))
res["counts_2sel"] = timeit(lambda: _native.kd_counts(Xd, lab, [0, 1], [1, 1], bounds, ctx=ctx))
lab0 = lab.clone()


def pass_ng2():
    lab.copy_(lab0)
    _native.kd_pass(Xd, lab, ([0], [0], [mid], [1]), [0, 1], ctx=ctx)


t_copy = timeit(lambda: lab.copy_(lab0))
res["pass_split1_ng2"] = timeit(pass_ng2) - t_copy
lab.copy_(lab0)
_native.kd_pass(Xd, lab, ([0, 1], [1, 1], [0.0, 0.0], [2, 3]), [0, 1, 2, 3], ctx=ctx)
lab1 = lab.clone()


def pass_ng4():
    lab.copy_(lab1)
    _native.kd_pass(Xd, lab, ([0, 1, 2, 3], [2, 2, 2, 2], [0.0] * 4, [4, 5, 6, 7]), [], ctx=ctx)


res["split_only_4"] = timeit(pass_ng4) - t_copy
res["counts_4sel"] = timeit(lambda: _native.kd_counts(Xd, lab1, [0, 1, 2, 3], [2] * 4,
                                                      np.tile(np.linspace(-40, 40, 7), (4, 1)),
                                                      ctx=ctx))


def pass_ng4m():
    lab.copy_(lab0)
    _native.kd_pass(Xd, lab, ([0, 1], [1, 1], [0.0, 0.0], [2, 3]), [0, 1, 2, 3], ctx=ctx)


res["pass_split2_ng4"] = timeit(pass_ng4m) - t_copy
for k, v in res.items():
    print("%-22s %7.3f ms  X-stream %6.2f TB/s" % (k, v, GB / v))
