import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "cpu: CPU-only test")
    config.addinivalue_line("markers", "slow: long-running test")
    # the C++ data-index extension (host code, seconds to build) is needed by the CPU data tests;
    # build it in-tree once in the controller process (not in xdist workers) if it is missing
    if not hasattr(config, "workerinput"):
        from scaling_amd import _build

        if not _build.data_ext_path().exists():
            _build.build_data(verbose=False)


@pytest.fixture(autouse=True)
def _reset_logger():
    yield
