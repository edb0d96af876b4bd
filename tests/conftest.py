import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs the C-ABI hot path")


@pytest.fixture(scope="session")
def lvo():
    from lvo_amd_loader import lvo as mod
    return mod


@pytest.fixture
def gpu_ctx_factory(lvo):
    """Creates HIP contexts for one test (destroyed at its end); fails (never skips silently) when
    the HIP library or GPU is missing."""
    ctxs = []

    def make(scan_line=64, **over):
        p = lvo.abi.default_params(scan_line)
        for k, v in over.items():
            setattr(p, k, v)
        c = lvo.Context(p, device=0)
        ctxs.append(c)
        return c

    yield make
    for c in ctxs:
        c.close()
