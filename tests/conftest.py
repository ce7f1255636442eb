import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running test")
    # Build the native extension once per session (no-op when up to date).
    r = subprocess.run(["make", "-j8", "-C", ROOT], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + r.stdout[-3000:] + r.stderr[-3000:])


@pytest.fixture(scope="session")
def hamlet() -> bytes:
    with open(os.path.join(ROOT, "data", "hamlet.txt"), "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def cli() -> str:
    return os.path.join(ROOT, "build", "MapReduce")
