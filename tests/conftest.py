import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def golden_names():
    return sorted(f[4:-4] for f in os.listdir(GOLDEN) if f.startswith("ref_") and f.endswith(".npz"))


def load_golden(name, prefix="ref"):
    import numpy as np
    z = np.load(os.path.join(GOLDEN, f"{prefix}_{name}.npz"))
    return {k: z[k] for k in z.files}


def rotation_names():
    """Goldens of KDPartitioner(split_method='rotation') (make_golden_rotation.py)."""
    return sorted(f[4:-4] for f in os.listdir(GOLDEN) if f.startswith("rot_") and f.endswith(".npz"))
