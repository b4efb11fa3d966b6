import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def load_pkg():
    """Import the hyphenated package directory `arpack-ng_amd/` as `arpack_ng_amd`."""
    if "arpack_ng_amd" in sys.modules:
        return sys.modules["arpack_ng_amd"]
    d = os.path.join(ROOT, "arpack-ng_amd")
    spec = importlib.util.spec_from_file_location("arpack_ng_amd", os.path.join(d, "__init__.py"),
                                                  submodule_search_locations=[d])
    m = importlib.util.module_from_spec(spec)
    sys.modules["arpack_ng_amd"] = m
    spec.loader.exec_module(m)
    return m


@pytest.fixture(scope="session")
def pkg():
    return load_pkg()


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def get(name):
        return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
    return get
