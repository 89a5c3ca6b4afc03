import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU check")


def _ensure_built():
    libs = [os.path.join(ROOT, "ray_tracying_amd", "lib", n) for n in ("librt_hip.so", "librt_host.so")]
    libs.append(os.path.join(ROOT, "oracle", "liboracle.so"))
    if not all(os.path.exists(p) for p in libs):
        subprocess.run(["make", "-j8", "-C", ROOT], check=True, capture_output=True)


@pytest.fixture(scope="session", autouse=True)
def built():
    _ensure_built()
    yield


@pytest.fixture(scope="session")
def gpu():
    import ray_tracying_amd as rt
    n = rt.device_count()
    if n < 1:
        pytest.fail("no HIP device visible: the gpu tests must run on an MI355X")
    return n
