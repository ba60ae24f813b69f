"""Experiment: link strategies on the C2 workload, interleaved in one process."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from pypardis_amd import DBSCAN, _native, synth
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
X, cfg = synth.make_config("C2", n=n)
Xd = torch.from_numpy(X).cuda(); del X
ctx = _native.context()
ctx.set_option(_native.PD_OPT_TIMING, 1)
variants = [("x1", 0, 4, 1), ("x2", 0, 4, 2), ("x4", 0, 4, 4), ("x2_sweep", 1, 0, 2), ("x2_j8", 0, 8, 2)]
ref = None
res = {v[0]: [] for v in variants}
for rnd in range(3):
    for name, mode, jr, xs in variants:
        ctx.set_option(_native.PD_OPT_XSUB, xs)
        ctx.set_option(_native.PD_OPT_LINK_MODE, mode)
        ctx.set_option(_native.PD_OPT_JUMP_ROUNDS, jr)
        m = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=8).train(Xd)
        t = ctx.timings()
        res[name].append((t["link"], t["merge"], t["roots"], t["border"], t["total"], t["count"], t["sort"], t["cells"]))
        if mode != 1:
            if ref is None:
                ref = m.labels_.clone()
            assert torch.equal(ref, m.labels_), name
for k, v in res.items():
    a = np.array(v)
    print(f"{k:12s} sort={np.median(a[:,6]):5.2f} cells={np.median(a[:,7]):5.2f} count={np.median(a[:,5]):6.2f} link={np.median(a[:,0]):8.2f} merge={np.median(a[:,1]):7.2f} roots={np.median(a[:,2]):6.2f} border={np.median(a[:,3]):6.2f} total={np.median(a[:,4]):8.2f} ms")
