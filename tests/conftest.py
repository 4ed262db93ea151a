import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


def golden_cases():
    """Names of the aggregation fixtures made by tests/golden/make_golden.py."""
    names = []
    for p in sorted(glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))):
        name = os.path.splitext(os.path.basename(p))[0]
        if name != "relpose" and not name.startswith("ref_"):
            names.append(name)
    return names


def load_golden(name):
    with np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def rel_err(got, ref):
    """max |got - ref| / max |ref| (the parity metric: relative to the tensor's max-abs)."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    if ref.size == 0:
        return 0.0
    scale = max(np.abs(ref).max(), 1e-30)
    return float(np.abs(got - ref).max() / scale)


@pytest.fixture(scope="session")
def cuda_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU visible")
    return torch.device("cuda:0")
