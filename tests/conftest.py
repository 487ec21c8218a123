import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running pin (still part of the default suites)")


def _ensure_built():
    lib = os.path.join(ROOT, "aniso_amd", "libaniso_mi355x.so")
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")])
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "aniso_amd", "csrc"), "-j8"])


_ensure_built()


def main_coeffs(xy):
    """main.cpp:34-40 coefficient functions."""
    import numpy as np

    x = xy[:, 0]
    ss = 16 * 0.5 * (1 - np.cos(2 * np.pi * x))
    return ss, ss + 0.2


def gaussian_charge(xy):
    """main.cpp:29-32 source function."""
    import numpy as np

    return np.exp(-25 * ((xy[:, 0] - 0.5) ** 2 + (xy[:, 1] - 0.5) ** 2))


def rough_coeffs(xy, seed):
    """Piecewise-varying sigma (not smooth across squares) to exercise the line integral."""
    import numpy as np

    rng = np.random.default_rng(seed)
    ss = rng.uniform(0.5, 6.0, xy.shape[0])
    return ss, ss + rng.uniform(0.1, 2.0, xy.shape[0])


@pytest.fixture(scope="session")
def root():
    return ROOT
