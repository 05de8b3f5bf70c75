import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE_DATA = "/root/reference/data"
# the reference's bundled fixture (/root/reference/data), decoded by our own t7 reader and
# committed as packed .npz (tools/pack_fixture.py): present wherever the repo is, including
# the GPU box, where the reference tree is not mounted
PACKED_FIXTURE = os.path.join(ROOT, "tests", "fixtures")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running test")
    # an empty hipGraph capture is the symptom of a capture on the wrong device or stream:
    # SegmentedStep never produces one on purpose, so any occurrence fails the test
    config.addinivalue_line("filterwarnings", "error:The CUDA Graph is empty")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


HAS_GPU = _has_gpu()


def pytest_collection_modifyitems(config, items):
    if HAS_GPU:
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def ref_data():
    if not os.path.isdir(REFERENCE_DATA):
        pytest.skip("reference fixture data not mounted")
    return REFERENCE_DATA


@pytest.fixture(scope="session")
def packed_fixture():
    return PACKED_FIXTURE
