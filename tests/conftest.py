import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and libfmt.so")


@pytest.fixture(scope="session")
def orc():
    import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """A process that uses torch's device buffers beside libfmt.so (test_map_replay_device_buffers_and_bad_keys)
    initialises torch's HIP runtime (the one bundled with the torch wheel) before libfmt.so opens the
    device through the image's ROCm: the other order leaves torch with "No HIP GPUs are available" on
    some boxes. bench.py initialises torch first too."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        try:
            import torch

            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:  # (no torch GPU runtime: the torch-using tests fail on their own)
            pass
    yield
