import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.dirname(os.path.abspath(__file__))):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def pytest_configure(config):
    # torch bundles its own HIP runtime (libamdhip64, ROCm 7.0) while libfm_hip.so links the system one
    # (ROCm 7.2) under the same soname: whichever loads first serves both.  Import torch before any test
    # loads libfm_hip.so, so the tests that also use torch (device-resident frames) see a working GPU
    # whatever order they run in -- the order bench.py uses too.
    try:
        import torch  # noqa: F401
    except Exception:  # noqa: BLE001 - torch is optional for the CPU tests
        pass
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle

    oracle.build()
    return oracle
