"""Calibrate oracle/cpu_ref.py against the reference itself (build container
only — the reference never travels): the unmodified reference pipeline
(R:dbscan/*.py) run under the in-memory RDD stand-in of
tests/golden/make_golden.py, and cpu_ref with one worker, on the same 1M-point
C2 density-preserving slice (78.0 s for the reference).

  PYTHONHASHSEED=0 python tools/calibrate_cpu_ref.py [n] > profiles/r02_cpu_calibration.json

The ratio reference_seconds / cpu_ref_seconds (both one process) says how
much faster the restatement is than the reference's own Python + sklearn
work at equal cores; bench.py quotes it beside its cpu_baseline.
"""
import json
import os
import sys
import time

sys.dont_write_bytecode = True
os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from oracle import cpu_ref  # noqa: E402
from pypardis_amd import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    X, cfg = synth.make_config("C2", n=n)
    eps, ms, P = cfg["eps"], cfg["min_samples"], cfg["max_partitions"]
    oracle.build()
    import make_golden
    ref, _, _, _ = make_golden.load_reference()
    rows = [(i, X[i].astype(np.float64)) for i in range(n)]
    t0 = time.perf_counter()
    m = ref.DBSCAN(eps=eps, min_samples=ms, metric="euclidean", max_partitions=P)
    m.train(make_golden.FakeContext(1).parallelize(rows))
    a = m.assignments()
    t_ref = time.perf_counter() - t0
    assert len(a) == n
    lab, t_port, _ = cpu_ref.run(X, eps, ms, P, workers=1)
    lab_o, core_o, _, _ = oracle.dbscan(X, eps, ms)
    core_o = core_o.astype(bool)
    info = cpu_ref.host_info()
    print(json.dumps(dict(
        n=n, config="C2 density-preserving slice", max_partitions=P, metric="euclidean",
        reference_seconds=t_ref, cpu_ref_seconds_1_worker=t_port,
        ratio_reference_over_cpu_ref=t_ref / t_port,
        cpu_ref_core_labels_equal_global_sklearn=bool(np.array_equal(lab[core_o], lab_o[core_o])),
        cpu_ref_noise_equal=bool(np.array_equal(lab < 0, lab_o < 0)),
        host=info, note="reference = unmodified R:dbscan/*.py under the RDD stand-in of "
                        "tests/golden/make_golden.py, one process; cpu_ref = oracle/cpu_ref.py "
                        "with one worker (same algorithm, numpy KD + halo, sklearn per "
                        "neighbourhood, owner-rule merge)")))


if __name__ == "__main__":
    main()
