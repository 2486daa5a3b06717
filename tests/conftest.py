import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session", autouse=True)
def _built_libraries():
    """Build the oracle (and the product library if hipcc is present and it is missing)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = os.path.join(ROOT, "pf_monocular_pose_estimator_amd", "libpfmpe.so")
    if not os.path.exists(lib) and os.path.exists("/opt/rocm/bin/hipcc"):
        subprocess.run(["make", "-s", "-j5", "-C", os.path.join(ROOT, "pf_monocular_pose_estimator_amd")], check=True)
    yield
