"""Shared pytest setup: the `gpu` marker, paths to the drop-in package, the
oracle and the golden fixtures."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "beta-sgp_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def ref_kwargs(fx):
    """The kwargs dict stored (as a repr of plain literals) in a fixture."""
    import ast
    return ast.literal_eval(str(fx["kwargs"]))


@pytest.fixture(scope="session")
def ngc():
    d = golden("ngc7027_inputs.npz")
    return d["gn"], d["psf"], d["bg"][0][0], d["obj"]
