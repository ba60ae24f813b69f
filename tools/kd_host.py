"""Where the C2 step's time outside pd_train goes: KDPartitioner alone
(its GPU passes + host decisions), the whole DBSCAN.train, and pd_train's
own event total.  Wall clock, mean of 10 after warm-up.

  python tools/kd_host.py [n]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pypardis_amd import DBSCAN, KDPartitioner, _native, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
X, cfg = synth.make_config("C2", n=n)
Xd = torch.from_numpy(X).cuda()
del X
ctx = _native.context()


def wall(f, reps=10):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / reps


t_kd = wall(lambda: KDPartitioner(Xd, 8))
t_train = wall(lambda: DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"],
                              max_partitions=8).train(Xd))
ctx.set_option(_native.PD_OPT_TIMING, 1)
DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=8).train(Xd)
torch.cuda.synchronize()
tot = ctx.timings()["total"]
ctx.set_option(_native.PD_OPT_TIMING, 0)
print("KDPartitioner %.3f ms | train %.3f ms | pd_train events %.3f ms | train - kd - pd_train "
      "%.3f ms" % (t_kd, t_train, tot, t_train - t_kd - tot))
