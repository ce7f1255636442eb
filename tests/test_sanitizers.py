"""Host-only AddressSanitizer/UBSan build: the CPU engine, loaders,
spill I/O, generator and CLI run clean under ASan.  (GPU ASan / xnack+ is not available
on the GPU pool.)"""
import os
import subprocess

import pytest

from locust_amd.utils import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "build", "asan", "MapReduce")


@pytest.fixture(scope="module")
def asan_cli():
    r = subprocess.run(["make", "-C", ROOT, "asan"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return ASAN


def run(cmd, **kw):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    return subprocess.run(cmd, capture_output=True, env=env, timeout=300, **kw)


def test_cpu_pipeline_under_asan(asan_cli, hamlet):
    r = run([asan_cli, os.path.join(ROOT, "data", "hamlet.txt"), "--backend", "cpu"])
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    out = r.stdout.decode()
    ent = oracle.wordcount(hamlet)[0]
    body = out[out.index("print key:"):out.rindex("\nDone")].rstrip("\n")
    assert body == oracle.format_cpu(ent).decode().rstrip("\n")


def test_stage_split_and_generator_under_asan(asan_cli, tmp_path):
    g = tmp_path / "g.txt"
    r = run([asan_cli, "--gen", str(g), "--gen-lines", "5000", "--seed", "3"])
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    for fmt in ("text", "binary"):
        r = run([asan_cli, str(g), "0", "2500", "7", "1", "--backend", "cpu", "--spill-dir",
                 str(tmp_path), "--spill-format", fmt])
        assert r.returncode == 0, r.stderr.decode()[-3000:]
        spill = tmp_path / ("out.7.kv" if fmt == "binary" else "out.7.txt")
        r = run([asan_cli, str(g), "0", "0", "7", "2", "--backend", "cpu", "--inputs", str(spill)])
        assert r.returncode == 0, r.stderr.decode()[-3000:]


def test_gpu_backend_fails_loudly_in_host_build(asan_cli):
    r = run([asan_cli, os.path.join(ROOT, "data", "hamlet.txt")])
    assert r.returncode == 2 and b"no GPU backend" in r.stderr
