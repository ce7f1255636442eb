"""__graft_entry__.build() in a clean tree: the build must run before anything imports the
package (locust_amd/__init__.py loads the extension, which a clean tree does not have yet)."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_build_runs_make_before_importing_the_package(tmp_path):
    tree = tmp_path / "tree"
    (tree / "locust_amd").mkdir(parents=True)
    shutil.copy(os.path.join(ROOT, "__graft_entry__.py"), tree)
    for f in ("__init__.py", "_native.py"):
        shutil.copy(os.path.join(ROOT, "locust_amd", f), tree / "locust_amd")
    # a stand-in `make` that records its call and builds nothing
    bin_dir = tmp_path / "bin"
    bin_dir.mkdir()
    marker = tmp_path / "make_called"
    (bin_dir / "make").write_text(f"#!/bin/sh\necho \"$@\" > {marker}\n")
    (bin_dir / "make").chmod(0o755)
    env = dict(os.environ, PATH=f"{bin_dir}:{os.environ['PATH']}")
    p = subprocess.run([sys.executable, "-c", "import __graft_entry__ as g; g.build()"], cwd=tree,
                       env=env, capture_output=True, text=True, timeout=120)
    assert marker.exists(), p.stderr[-2000:]  # make ran first
    assert f"-C {tree}" in marker.read_text()
    # the stand-in built nothing, so the import after it fails loudly (no Python fallback)
    assert p.returncode != 0 and "native extension is not built" in p.stderr
