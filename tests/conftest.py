import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) -- run with -m gpu")
    # the sanitizer run (scripts/asan_cpu_suite.sh) points the tests at the host-ASan engine build
    eng = os.environ.get("SDR_TEST_ENGINE_LIB")
    if eng:
        from stereo_depth_ruler_amd import _lib
        _lib.use_library(eng)


def hyp_examples(n: int) -> int:
    """A hypothesis test's example count: n, times SDR_HYP_SCALE for a wider survey on the box
    (the round's logs: profiles/r6_parity_survey/)."""
    return max(1, int(n * float(os.environ.get("SDR_HYP_SCALE", "1"))))


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    O.build()
    return O
