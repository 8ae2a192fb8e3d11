import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libcsmom.so on cuda:0)")


def load_golden(name):
    return np.load(GOLDEN / f"{name}.npz", allow_pickle=False)


def golden_tags(z):
    return sorted({k.split("_")[0] for k in z.files if k.startswith("J") and "s" in k.split("_")[0]})


def parse_tag(tag):
    return int(tag[1:tag.index("s")]), int(tag[tag.index("s") + 1:])


def bits_equal(a, b):
    """Bitwise equality of float arrays, NaN positions compared as NaN (payload-agnostic)."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    if a.shape != b.shape:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    return bool((na == nb).all() and (a[~na].view(np.uint64) == b[~nb].view(np.uint64)).all())


def max_rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    m = ~(np.isnan(a) | np.isnan(b))
    if not m.any():
        return 0.0
    return float(np.max(np.abs(a[m] - b[m]) / np.maximum(np.abs(b[m]), 1e-300)))


@pytest.fixture(scope="session")
def engine():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import csmom
    return csmom.Engine(0)
