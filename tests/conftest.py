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


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    # torch bundles its own libamdhip64.so.7: it must bring up its HIP runtime BEFORE
    # libeg_hip.so pulls in the system one, or torch sees no GPU (tests that hand torch
    # device tensors to the C ABI need both).  bench.py has the same order.  Session-wide, so
    # no test order (a fixture opening a context directly) can load the library first.
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()


@pytest.fixture(scope="session")
def group():
    from electionguard.core import productionGroup
    return productionGroup(0)


def be2i(row) -> int:
    return int.from_bytes(bytes(row), "big")
