"""The reference's 40-B record (KeyIntValuePair, /root/reference/MapReduce/src/KeyValue.h:
13-18) as a real file format: the kiv stage-1 spill and the --export-kiv results, checked
byte by byte with `struct` (key[30] NUL padded, 2 pad bytes, int value @32, int count @36)."""
import os
import struct
import subprocess

import pytest

import locust_amd as lc
from locust_amd.utils import oracle

REC = struct.Struct("<30s2xii")
assert REC.size == 40


def parse(path):
    data = open(path, "rb").read()
    magic, version, recsize, count, _ = struct.unpack_from("<8sIIQQ", data, 0)
    assert magic == b"LCSTKIV1" and version == 1 and recsize == 40
    assert len(data) == 32 + 40 * count
    return [REC.unpack_from(data, 32 + 40 * i) for i in range(count)]


def test_spill_roundtrip_and_layout(tmp_path):
    recs = [(b"alpha", 3), (b"b", 1), (b"x" * 29, 7)]
    p = str(tmp_path / "s.kiv")
    lc._C.write_spill(p, recs, "kiv")
    raw = parse(p)
    assert [(k.rstrip(b"\0"), v, c) for k, v, c in raw] == [(k, n, 0) for k, n in recs]
    assert lc._C.read_spill(p) == recs
    assert lc._C.read_kiv(p) == [(k, n, 0) for k, n in recs]


def test_too_long_key_is_refused(tmp_path):
    with pytest.raises(Exception):
        lc._C.write_spill(str(tmp_path / "bad.kiv"), [(b"y" * 30, 1)], "kiv")


def test_cli_export_and_kiv_stage_split(hamlet, cli, tmp_path):
    text = oracle.window(hamlet, 0, 1500)
    src = tmp_path / "h.txt"
    src.write_bytes(text)
    ent = oracle.wordcount(text)[0]
    out = tmp_path / "res.kiv"
    r = subprocess.run([cli, str(src), "--backend", "cpu", "--quiet", "--export-kiv", str(out)],
                       capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert [(k.rstrip(b"\0"), v, c) for k, v, c in parse(out)] == ent
    # stage 1 writes out.<node>.kiv, stage 2 reads it back
    d = str(tmp_path)
    r1 = subprocess.run([cli, str(src), "0", "1500", "4", "1", "--backend", "cpu", "--spill-dir", d,
                         "--spill-format", "kiv"], capture_output=True, timeout=120)
    assert r1.returncode == 0, r1.stderr
    spill = os.path.join(d, "out.4.kiv")
    recs = parse(spill)
    assert sum(v for _k, v, _c in recs) == sum(c for _k, _v, c in ent)
    r2 = subprocess.run([cli, str(src), "0", "0", "4", "2", "--backend", "cpu", "--spill-dir", d,
                         "--spill-format", "kiv"], capture_output=True, timeout=120)
    assert r2.returncode == 0, r2.stderr
    assert oracle.format_gpu(ent) in r2.stdout or oracle.format_cpu(ent) in r2.stdout
