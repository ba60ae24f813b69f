"""One warm C2 train (for rocprofv3 --pmc / --kernel-trace runs)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pypardis_amd import DBSCAN, _native, synth

n = int(os.environ.get("PROF_N", "100000000"))
name = os.environ.get("PROF_CFG", "C2")
X, cfg = synth.make_config(name, n=n, device="cuda" if name == "C4" else "cpu")
Xd = X if torch.is_tensor(X) else torch.from_numpy(X).cuda()
del X
for _ in range(int(os.environ.get("PROF_REPS", "2"))):
    m = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"],
               max_partitions=cfg.get("max_partitions") or 1).train(Xd)
torch.cuda.synchronize()
print("clusters", m.n_clusters_)
