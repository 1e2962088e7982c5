import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def pncx():
    """The HIP library; on a GPU box a load failure is an error, not a skip."""
    from pnetcdf_amd import pncx as P
    P.lib()
    return P


@pytest.fixture
def knob():
    """knob(name, value): set an A/B switch of libpncx (pncx_knob_set, read
    once from PNCX_<name> at load) for this test; restored afterwards."""
    from pnetcdf_amd import pncx as P
    saved = {}

    def set_(name, value):
        if name not in saved:
            saved[name] = P.knob_get(name)
        P.knob_set(name, int(value))

    yield set_
    for name, value in saved.items():
        P.knob_set(name, value)
