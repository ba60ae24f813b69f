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
variants = [("uf_only", 2, 0), ("sweep_only", 1, 0), ("mn+j0", 0, 0), ("mn+j1", 0, 1), ("mn+j2", 0, 2), ("mn+j4", 0, 4)]
ref = None
res = {v[0]: [] for v in variants}
for rnd in range(3):
    for name, mode, jr in variants:
        ctx.set_option(_native.PD_OPT_LINK_MODE, mode)
        ctx.set_option(_native.PD_OPT_JUMP_ROUNDS, jr)
        m = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"], max_partitions=8).train(Xd)
        t = ctx.timings()
        res[name].append((t["link"], t["merge"], t["roots"], t["border"], t["total"], t["count"]))
        if mode != 1:
            if ref is None:
                ref = m.labels_.clone()
            assert torch.equal(ref, m.labels_), name
for k, v in res.items():
    a = np.array(v)
    print(f"{k:12s} count={np.median(a[:,5]):6.2f} link={np.median(a[:,0]):8.2f} merge={np.median(a[:,1]):7.2f} roots={np.median(a[:,2]):6.2f} border={np.median(a[:,3]):6.2f} total={np.median(a[:,4]):8.2f} ms")
