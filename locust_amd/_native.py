"""Loader for the native extension (``locust_amd/_locust*.so`` + ``_lib/liblocust.so``).

The extension is built in-tree by ``make`` (or ``python __graft_entry__.py``, which runs it).  Import fails
loudly when it is missing: there is no pure-Python fallback for the engine, so a GPU test
can never silently pass on a Python stand-in.
"""
from __future__ import annotations

import os
import subprocess
import sys

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(jobs: int = 8, quiet: bool = True) -> None:
    """Compile every HIP/C++ source for gfx950 (``make -j``) in the repo root."""
    cmd = ["make", f"-j{jobs}", "-C", REPO_ROOT]
    out = subprocess.run(cmd, capture_output=quiet, text=True)
    if out.returncode != 0:
        msg = (out.stdout or "") + (out.stderr or "") if quiet else ""
        raise RuntimeError(f"native build failed ({' '.join(cmd)}):\n{msg[-4000:]}")


def load():
    try:
        from . import _locust  # noqa: F401
    except ImportError as e:  # pragma: no cover - exercised only on a broken checkout
        raise ImportError(
            "locust_amd native extension is not built; run `make -j8` in "
            f"{REPO_ROOT} (or `python __graft_entry__.py`). Original error: {e}"
        ) from e
    return sys.modules[__name__.rsplit(".", 1)[0] + "._locust"]


def cli_path() -> str:
    """Path of the ``MapReduce`` CLI binary built next to the package."""
    return os.path.join(REPO_ROOT, "build", "MapReduce")
