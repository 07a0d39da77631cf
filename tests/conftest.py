import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "rootless-coll-mpi-ops_amd")
for p in (REPO, PKG, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librlo_hip.so on the device)")
    config.addinivalue_line("markers", "slow: long CPU test")


def pytest_collection_modifyitems(session, config, items):
    """The drop-in tests run first.  They start 4-8 MPI processes, each holding a persistent
    kernel on its own HIP queue; once this pytest process has used the GPU it keeps up to
    GPU_MAX_HW_QUEUES idle queues of its own, and with those the 8-rank run of testcases.c was
    seen to stall (no rank reached its progress loop; hardware queues oversubscribed is the
    likely cause: the same run passes when this process has not touched the GPU).  bench.py runs its
    drop-in leg before opening the GPU for the same reason."""
    items.sort(key=lambda it: 0 if os.path.basename(str(it.fspath)) == "test_gpu_dropin.py" else 1)


@pytest.fixture(scope="session")
def golden():
    import json

    d = os.path.join(REPO, "tests", "golden")

    def load(name):
        with open(os.path.join(d, name)) as f:
            return json.load(f)

    return load
