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


@pytest.fixture(autouse=True, scope="session")
def _private_cache_dir(tmp_path_factory):
    """Per-session cache directory (partition maps, sparse line indexes): tests never read
    or write the user's ~/.cache/locust.  A test that wants its own sets LOCUST_CACHE_DIR."""
    if "LOCUST_CACHE_DIR" in os.environ:
        yield
        return
    os.environ["LOCUST_CACHE_DIR"] = str(tmp_path_factory.mktemp("locust_cache"))
    try:
        yield
    finally:
        os.environ.pop("LOCUST_CACHE_DIR", None)
