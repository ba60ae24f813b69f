"""Full-size rehearsals of the multi-GPU train on one MI355X.

BASELINE.json's C2 ("100M 3-D blobs, max_partitions=8, one KD partition per
GPU with RCCL label merge over xGMI") and C4 ("1B 2-D points ... across
8xMI355X") are multi-GPU configurations.  The node that runs them is not
available here, so the sharded path runs exactly as bench.py --gpus N runs it
(DBSCAN(group=...).train(this rank's slice), one process per rank) with W
ranks sharing cuda:0 and gloo carrying the collectives through the host:
device-decided KD with gathered partials, route / pack / exchange of the
halo records, per-rank clustering, the export merge, results back to the
holding ranks.  The assembled labels and core flags must equal the
single-device train's bit for bit (which the windowed oracle checks of
test_gpu_fullsize.py pin to sklearn's)."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _single(X, cfg):
    from pypardis_amd import DBSCAN
    Xd = X if torch.is_tensor(X) else torch.from_numpy(X).cuda()
    m = DBSCAN(eps=cfg["eps"], min_samples=cfg["min_samples"],
               max_partitions=cfg["max_partitions"]).train(Xd)
    return (m.labels_.cpu().numpy().astype(np.int64), m.core_sample_mask_.cpu().numpy(),
            m.n_clusters_)


@pytest.fixture(scope="module")
def c2_full(tmp_path_factory):
    from pypardis_amd import synth
    X, cfg = synth.make_config("C2")
    lab, core, ncl = _single(X, cfg)
    path = str(tmp_path_factory.mktemp("c2") / "x.npy")
    np.save(path, X)
    del X
    return path, cfg, lab, core, ncl


@pytest.mark.parametrize("world", [2, 4])
def test_c2_full_sharded_rehearsal(c2_full, tmp_path, world):
    from dist_worker import run_rehearsal
    path, cfg, lab, core, ncl = c2_full
    out = run_rehearsal(world, path, cfg["eps"], cfg["min_samples"], cfg["max_partitions"],
                        str(tmp_path))
    assert out["ncl"] == {ncl}
    assert out["exports"] > 0          # clusters cross the ranks: the merge is exercised
    assert out["received"] > len(lab)  # halo copies travel to both sides
    assert torch.equal(torch.from_numpy(out["labels"]), torch.from_numpy(lab))
    assert torch.equal(torch.from_numpy(out["core"]), torch.from_numpy(core))
    print(f"C2 100M, {world} ranks: per-rank seconds {out['seconds']}")


def test_c4_sample_sharded_rehearsal(tmp_path):
    """A 200M-point C4 sample (the 1B generator's distribution: Zipf cities,
    dense centres), P = 8 over 4 ranks."""
    from dist_worker import run_rehearsal
    from pypardis_amd import synth
    X, cfg = synth.make_config("C4", n=200_000_000, device="cuda")
    lab, core, ncl = _single(X, cfg)
    path = str(tmp_path / "x.npy")
    np.save(path, X.cpu().numpy())
    del X
    torch.cuda.empty_cache()
    out = run_rehearsal(4, path, cfg["eps"], cfg["min_samples"], cfg["max_partitions"],
                        str(tmp_path))
    os.remove(path)
    assert out["ncl"] == {ncl}
    assert torch.equal(torch.from_numpy(out["labels"]), torch.from_numpy(lab))
    assert torch.equal(torch.from_numpy(out["core"]), torch.from_numpy(core))
    print(f"C4 200M, 4 ranks: per-rank seconds {out['seconds']}")
