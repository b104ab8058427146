import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: large-size GPU property tests")


@pytest.fixture(scope="session")
def oracle_port():
    import oracle
    if not oracle.available("port"):
        oracle.build(ref=False)
    return oracle.Oracle("port")


@pytest.fixture(scope="session")
def gpu_lib():
    from cp_pfdr_graph_d1_amd import pfdr
    lib = pfdr.load()
    n = lib.pfdr_device_count()
    if n is None or n < 1:
        pytest.fail("-m gpu test without a visible HIP device")
    return pfdr.Lib()
