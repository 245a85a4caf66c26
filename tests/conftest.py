import glob
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def golden_names(kind="admm"):
    """Committed golden cases: triple_decomp_ADMM (g*.npz), the same solver with
    opts.model='qi' (qi*.npz), triple_decomp_ALS (als*.npz) or the nonconvex
    test.m solver (nc*.npz)."""
    pat = {"admm": "g*.npz", "qi": "qi*.npz", "als": "als*.npz", "ncvx": "nc*.npz"}[kind]
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, pat)))


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["opts"] = json.loads(str(d["opts"]))
    d["r"] = int(d["r"])
    d["k"] = int(d["k"])
    return d


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    nb = np.linalg.norm(b.ravel())
    return np.linalg.norm((a - b).ravel()) / (nb if nb > 0 else 1.0)


@pytest.fixture(scope="session")
def gpu_available():
    try:
        import tritd
        return tritd.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def synth():
    from tritd import synth as s
    return s
