import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Hardware queues: the GPU box exports GPU_MAX_HW_QUEUES=4 (HIP's default).
# The single-process groups of the GPU tests use at most 3 ranks, one stream
# each, so every rank's stream has a queue of its own at that setting; the
# multi-process tests leave the budget to rdc_amd.launcher / the library.
# fail fast instead of waiting out the production timeout
os.environ.setdefault("RDC_TIMEOUT", "30")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O
