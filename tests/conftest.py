import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs the product kernels")


@pytest.fixture(scope="session")
def oracle_built():
    from oracle import oracle as O
    if not os.path.exists(O.ORACLE_SO):
        O.build()
    return O


@pytest.fixture(scope="session")
def product():
    import libyafaray_amd as Y
    if not os.path.exists(Y.LIB_PATH):
        Y.build()
    return Y


def experiments_built() -> bool:
    """Whether libyafaray4.so carries the measured-and-dropped pipelines (-DYAF_EXPERIMENTS: k_trace_brute,
    ray sorting, k_path, in-place NEE shadow rays, the bounded gather walk); the product build does not."""
    import libyafaray_amd as Y
    return "YAF_EXPERIMENTS" in Y.build_info()


@pytest.fixture
def experiments(product):
    if not experiments_built():
        pytest.skip("needs a -DYAF_EXPERIMENTS build of libyafaray4.so (tools/build_variants.sh)")
    return True
