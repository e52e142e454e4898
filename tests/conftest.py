import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_addoption(parser):
    # A/B runs only (tools/build_variant.sh): run the suite against another build of the engine
    parser.addoption("--sgx-lib", default=None, help="path of an alternate libsgx.so build")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsgx.so on cuda:0)")
    config.addinivalue_line("markers", "slow: large inputs (full BASELINE sizes)")
    alt = config.getoption("--sgx-lib")
    if alt:
        import sparkucx_amd._lib as L

        L.LIB_PATH = os.path.abspath(alt)


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def sgx_lib():
    import sparkucx_amd

    if not os.path.exists(sparkucx_amd._lib.LIB_PATH):
        import __graft_entry__

        __graft_entry__.build()
    sparkucx_amd.lib()
    return sparkucx_amd


@pytest.fixture(scope="session")
def engine(sgx_lib):
    eng = sgx_lib.ShuffleEngine(device=0)
    yield eng
    eng.close()
