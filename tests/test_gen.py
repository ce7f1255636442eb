"""Synthetic text generator (the 1M-line / 10 GB BASELINE configs' input)."""
import os
import subprocess

import pytest

import locust_amd as lc
from locust_amd.utils import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_deterministic_and_thread_independent():
    a = lc._C.gen_text(lines=5000, seed=3, threads=1)
    b = lc._C.gen_text(lines=5000, seed=3, threads=4)
    assert a == b
    assert a != lc._C.gen_text(lines=5000, seed=4)


def test_exact_lines_and_width():
    t = lc._C.gen_text(lines=3001, seed=1)
    lines = t.split(b"\n")
    assert t.endswith(b"\n") and len(lines) == 3002 and lines[-1] == b""
    assert max(len(x) for x in lines) <= 99  # the reference's 100-byte line slot


def test_bytes_mode_cuts_at_a_line():
    t = lc._C.gen_text(bytes=100000, seed=2)
    assert len(t) <= 100000 and len(t) > 99000 and t.endswith(b"\n")
    assert lc._C.gen_text(lines=5000, seed=2).startswith(t)


def test_block_sharding():
    """A rank can generate just its shard: blocks of 1,024 lines are independent."""
    whole = lc._C.gen_text(lines=4096, seed=9)
    parts = b"".join(lc._C.gen_text(lines=1024, seed=9, first_block=k) for k in range(4))
    assert parts == whole


def test_shape_is_hamlet_like():
    t = lc._C.gen_text(lines=20000, seed=5)
    ent, ntok, _ = oracle.wordcount(t)
    per_line = ntok / 20000
    assert 4 < per_line < 10  # Hamlet: 7.4 tokens per line
    counts = sorted((c for _k, _v, c in ent), reverse=True)
    assert counts[0] > 20 * counts[100]  # Zipfian head
    assert any(k[:1].isupper() for k, _v, _c in ent)  # case variants are distinct keys
    assert any(b"!" in k or b"?" in k for k, _v, _c in ent)  # non-delimiters stay in tokens


def test_host_text_roundtrip():
    h = lc._C.HostText.generate(lines=2000, seed=11)
    assert h.to_bytes() == lc._C.gen_text(lines=2000, seed=11)
    assert h.lines == 2000
    b = lc._C.HostText.from_bytes(b"a b\nc\n")
    assert b.size == 6 and b.lines == 2 and b.to_bytes() == b"a b\nc\n"


def test_cli_generator_matches(tmp_path):
    out = tmp_path / "g.txt"
    cli = os.path.join(ROOT, "build", "MapReduce")
    r = subprocess.run([cli, "--gen", str(out), "--gen-lines", "3000", "--seed", "4"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == lc._C.gen_text(lines=3000, seed=4)
    r = subprocess.run([cli, "--gen", str(out), "--gen-bytes", "50000", "--seed", "4"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == lc._C.gen_text(bytes=50000, seed=4)


def test_cpu_engine_on_generated_text():
    t = lc._C.gen_text(lines=3000, seed=6)
    r = lc.wordcount_text(t, backend="cpu")
    assert r.entries() == oracle.wordcount(t)[0]
