import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "proud-slam_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_DIR = os.path.join(REPO, "tests", "golden")
GOLDEN_CASES = ["A_voxels_center", "B_room0_small", "B_room0_det", "C_scannet_small"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running test")


def load_golden(name):
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN_DIR, f"{name}.npz"), allow_pickle=False))


@pytest.fixture(params=GOLDEN_CASES)
def golden(request):
    return request.param, load_golden(request.param)
