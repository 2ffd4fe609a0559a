import os
import sys

import pytest

# Load torch (and its HIP runtime) before libptamd.so: the library then binds
# to that same libamdhip64 (matched by SONAME) instead of pulling a second HIP
# runtime into the process when a test later hands it torch device memory.
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "discovering-path-tracer_amd")
for p in (PKG, os.path.join(ROOT, "tests"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def box_obj_bytes():
    path = os.path.join(ROOT, "tests", "golden", "box.obj")
    with open(path, "rb") as f:
        return f.read()
