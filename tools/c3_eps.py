"""Measure C3's eps: the 1st percentile, over a 50k-point
sample, of the distance to the 10th nearest neighbour (self included) in the
full 1M-point C3 set.  CPU (torch matmul, chunked); prints the value that
pypardis_amd/synth.py records as C3_EPS."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pypardis_amd import synth  # noqa: E402

cfg = dict(synth.CONFIGS["C3"])
X = synth.embeddings(cfg["n"], cfg["d"], n_clusters=cfg["n_clusters"],
                     clustered_frac=cfg["clustered_frac"], spread=cfg["spread"], seed=cfg["seed"])
rng = np.random.default_rng(0)
q = rng.choice(len(X), 50_000, replace=False)
Xt = torch.from_numpy(X.astype(np.float64))
n2 = (Xt * Xt).sum(1)
kth = []
for s in range(0, len(q), 500):
    Q = Xt[q[s:s + 500]]
    d2 = (Q * Q).sum(1)[:, None] + n2[None, :] - 2.0 * Q @ Xt.T
    kth.append(torch.topk(d2, 10, dim=1, largest=False).values[:, -1].clamp_min(0).sqrt())
kth = torch.cat(kth).numpy()
print(repr(float(np.percentile(kth, 1.0))))
