import json
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
GOLDEN = REPO / "tests" / "golden"
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU); run with -m gpu")


@pytest.fixture(scope="session")
def golden_meta():
    return json.loads((GOLDEN / "scenes.json").read_text())


@pytest.fixture(scope="session")
def golden_renders():
    with np.load(GOLDEN / "renders.npz") as z:
        return {k: z[k] for k in z.files}


def cpu_flags():
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("flags"):
                fl = line.split(":", 1)[1].split()
                return sorted(f for f in fl if f.startswith("avx512") or f in ("avx2", "fma"))
    except OSError:
        pass
    return []


def same_platform(meta) -> bool:
    """NumPy's SIMD sin/pow are ulp-exact only on the same NumPy version and CPU dispatch target
    as the container that generated the fixtures."""
    return meta.get("numpy") == np.__version__ and meta.get("cpu_flags") == cpu_flags()


def golden_png(name):
    from PIL import Image

    return np.asarray(Image.open(GOLDEN / name).convert("RGB"))
