import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the checker (oracle) and the host-side generator; the HIP library is built
    by __graft_entry__.build() (hipcc) and only loaded here."""
    import oracle
    oracle.build()
    from birdnest.audio_amd import build as b
    b.build_synth()
    yield


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
