import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


@pytest.fixture(scope="session")
def oracle_group():
    import eg_oracle as O
    return O.production_group()


# No GPU framework besides libeg_hip.so is brought up in the test process: device buffers come from
# the library itself (GroupContext.device_buffer / to_device, eg_dev_alloc), so the process holds
# one HIP runtime (torch is imported by the CPU tests for its gloo process group only).


@pytest.fixture(scope="session")
def group():
    from electionguard.core import productionGroup
    return productionGroup(0)


def be2i(row) -> int:
    return int.from_bytes(bytes(row), "big")
