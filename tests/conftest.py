import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — runs on the GPU box")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the in-tree engine and oracle libraries once (fast no-op when up to date)."""
    from koordinator_amd.build import build_all
    build_all()
    # torch's HIP runtime (its own copy) first: it does not initialise once the engine library has created a
    # context in this process, and some GPU tests hand torch tensors to the engine
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
