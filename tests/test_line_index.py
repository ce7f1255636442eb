"""Line and byte windows of stage 1 without an O(offset) prefix scan.

* find_line_window keeps a per-file sparse line index -- the newline count at every 8 MiB
  block start -- in the cache directory, keyed by the file's identity; a later window
  starts scanning at the last indexed block before its first line, so only the first
  window past a block pays for it.  The answers must not depend on what the cache holds.
* byte_window / ``--byte-range A:B`` moves both ends to line starts exactly as file_shards
  cuts, so windows [a0, a1), [a1, a2), ... of ANY offsets hold every line once: a launcher
  needs the file size only (the reference's per-node ranges, main.cu:369-374)."""
import glob
import os
import random
import subprocess

import pytest

import locust_amd as lc
from locust_amd.utils import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MiB = 1 << 20


def _starts(text: bytes) -> list[int]:
    """Byte offset of every line start, plus len(text) as the end sentinel."""
    s = [0]
    i = text.find(b"\n")
    while i >= 0:
        if i + 1 < len(text):
            s.append(i + 1)
        i = text.find(b"\n", i + 1)
    if not text:
        s = []
    return s + [len(text)]


def _expect(text: bytes, starts: list[int], s: int, e: int):
    nl = len(starts) - 1  # lines
    e = nl if e < 0 else max(e, s)
    if s >= nl:
        return len(text), len(text), 0
    return starts[s], starts[min(e, nl)], min(e, nl) - s


@pytest.fixture(scope="module")
def big(tmp_path_factory):
    """~26 MiB (4 blocks of 8 MiB) of irregular lines; last line without a newline."""
    rng = random.Random(11)
    parts, n = [], 0
    while n < 26 * MiB:
        ln = b"x" * rng.choice([0, 1, 5, 40, 200, 3000]) + b"\n"
        parts.append(ln)
        n += len(ln)
    text = b"".join(parts) + b"unterminated tail"
    f = tmp_path_factory.mktemp("lix") / "big.txt"
    f.write_bytes(text)
    return str(f), text, _starts(text)


def _cases(starts, rng):
    nl = len(starts) - 1
    c = [(0, 0), (0, 1), (0, -1), (nl - 1, -1), (nl - 1, nl), (nl, nl + 1), (nl + 5, -1),
         (nl // 2, nl // 2 + 1), (nl - 3, nl + 100), (5, 5)]
    c += [tuple(sorted(rng.sample(range(nl + 3), 2))) for _ in range(25)]
    c += [(rng.randrange(nl), -1) for _ in range(5)]
    return c


@pytest.mark.parametrize("order", ["forward", "backward", "random"])
def test_line_window_with_index_cache(big, tmp_path, monkeypatch, order):
    path, text, starts = big
    monkeypatch.setenv("LOCUST_CACHE_DIR", str(tmp_path / "c"))
    rng = random.Random({"forward": 1, "backward": 2, "random": 3}[order])
    cases = _cases(starts, rng)
    if order == "forward":
        cases.sort()
    elif order == "backward":
        cases.sort(reverse=True)
    for s, e in cases:
        assert tuple(lc._C.find_line_window(path, s, e)) == _expect(text, starts, s, e), (s, e)
    files = glob.glob(str(tmp_path / "c" / "lines-*.bin"))
    assert len(files) == 1  # one index for the file, grown in place
    # a cold cache, a disabled cache and a warm one agree
    monkeypatch.setenv("LOCUST_LINE_CACHE", "0")
    for s, e in cases[:8]:
        assert tuple(lc._C.find_line_window(path, s, e)) == _expect(text, starts, s, e)


def test_line_index_cache_invalidated_by_edit(tmp_path, monkeypatch):
    monkeypatch.setenv("LOCUST_CACHE_DIR", str(tmp_path / "c"))
    f = tmp_path / "t.txt"
    a = b"".join(b"a" * (i % 50) + b"\n" for i in range(400000))  # ~10 MiB
    f.write_bytes(a)
    nl = a.count(b"\n")
    assert lc._C.find_line_window(str(f), 0, -1)[2] == nl
    p1 = lc._C.line_index_cache_path(str(f))
    assert p1 and os.path.exists(p1)
    b = b"\n" * 1000 + a  # same path, new content: a new identity, never the stale index
    f.write_bytes(b)
    assert lc._C.line_index_cache_path(str(f)) != p1
    assert lc._C.find_line_window(str(f), 0, -1)[2] == nl + 1000
    assert tuple(lc._C.find_line_window(str(f), 1000, 1001)) == (1000, 1001, 1)
    # a damaged cache file is ignored and rewritten
    p2 = lc._C.line_index_cache_path(str(f))
    with open(p2, "r+b") as fh:
        fh.seek(48)
        fh.write(b"\xff" * 8)
    assert lc._C.find_line_window(str(f), 5, 9)[2] == 4
    monkeypatch.setenv("LOCUST_LINE_CACHE", "0")
    assert lc._C.line_index_cache_path(str(f)) == ""


@pytest.mark.parametrize("text", [b"", b"\n", b"abc", b"a\nb", b"a\nb\n", b"\n\n\nx\n\n"])
def test_byte_window_small(tmp_path, text):
    f = tmp_path / "t.txt"
    f.write_bytes(text)
    n = len(text)
    for a in range(n + 2):
        for b in range(a, n + 2):
            w = lc._C.byte_window(str(f), a, b)
            want_a = lc._C.line_start_at(str(f), a)
            assert w[0] == want_a and w[1] >= w[0]
            # a line start: 0, after a newline, or the end
            assert w[0] in (0, n) or text[w[0] - 1:w[0]] == b"\n"


def test_byte_windows_partition_lines(big):
    path, text, starts = big
    rng = random.Random(4)
    n = len(text)
    for parts in (1, 2, 3, 7, 16):
        cuts = sorted({0, n, *[rng.randrange(n) for _ in range(parts - 1)]})
        pieces = [lc._C.byte_window(path, a, b) for a, b in zip(cuts, cuts[1:])]
        assert pieces[0][0] == 0 and pieces[-1][1] == n
        for (a0, b0, _), (a1, _b1, _) in zip(pieces, pieces[1:]):
            assert b0 == a1  # adjacent: every line once
        assert all(p[0] in starts for p in pieces)
    # file_shards is the even-cut special case
    P = 5
    sh = lc._C.file_shards(path, P)
    for k, (off, nb) in enumerate(sh):
        w = lc._C.byte_window(path, n * k // P, n * (k + 1) // P)
        assert (w[0], w[1]) == (off, off + nb)


@pytest.mark.parametrize("windows", [2, 3, 8])
def test_cli_byte_range_stage_split(cli, hamlet, tmp_path, windows):
    """Stage 1 on byte ranges cut anywhere (the file size is all a launcher needs), then one
    stage 2: the single-stage output, val included."""
    f = os.path.join(ROOT, "data", "hamlet.txt")
    n = os.path.getsize(f)
    rng = random.Random(windows)
    cuts = [0] + sorted(rng.randrange(n) for _ in range(windows - 1)) + [n]
    spills, lines = [], 0
    for k, (a, b) in enumerate(zip(cuts, cuts[1:])):
        js = tmp_path / f"m{k}.json"
        rng_arg = f"{a}:{b}" if k < windows - 1 else f"{a}:"
        p = subprocess.run([cli, f, "0", "0", str(k), "1", "--byte-range", rng_arg,
                            "--spill-dir", str(tmp_path), "--spill-format", "binary",
                            "--backend", "cpu", "--json", str(js)],
                           capture_output=True, timeout=120)
        assert p.returncode == 0, p.stderr.decode()
        assert b"Using custom start" not in p.stdout  # no positional line window
        import json

        d = json.loads(js.read_text())
        assert d["byte_range_begin"] == a and d["byte_begin"] == lc._C.line_start_at(f, a)
        assert d["delimiters"] == oracle.DEFAULT_DELIMS.decode()
        lines += d["lines"]
        spills.append(str(tmp_path / f"out.{k}.kv"))
    assert lines == hamlet.count(b"\n") + (0 if hamlet.endswith(b"\n") else 1)
    p = subprocess.run([cli, f, "0", "0", "0", "2", "--inputs", ",".join(spills),
                        "--backend", "cpu", "--output-format", "gpu"], capture_output=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr.decode()
    ent, _ntok, _ = oracle.wordcount(hamlet)
    got = [l for l in p.stdout.split(b"\n") if l.startswith(b"print key:")]
    assert got == oracle.format_gpu(ent).rstrip(b"\n").split(b"\n")


def test_cli_byte_range_refusals(cli, tmp_path):
    f = os.path.join(ROOT, "data", "hamlet.txt")
    for args in (["--byte-range", "5:3", "0", "0", "0", "1"], ["--byte-range", "x", "0", "0", "0", "1"],
                 ["--byte-range", "0:10"], ["--byte-range", "0:10", "0", "0", "0", "1", "--ref-compat"]):
        p = subprocess.run([cli, f, *args, "--spill-dir", str(tmp_path), "--backend", "cpu"],
                           capture_output=True, timeout=60)
        assert p.returncode != 0, args


def test_count_newlines_simd_matches_python():
    """count_newlines (AVX2 / SSE2 byte-lane counters, 255 rounds per fold) against
    bytes.count at every alignment and length around the vector and fold boundaries."""
    import random

    rng = random.Random(7)
    base = bytes(rng.choice(b"ab\n\n \xff\x0a\x8a") for _ in range(300_000))
    for off in range(0, 40):
        for n in list(range(0, 140)) + [255 * 128 - 1, 255 * 128, 255 * 128 + 129, 200_000]:
            chunk = base[off:off + n]
            assert lc._C.count_newlines(chunk) == chunk.count(b"\n"), (off, n)
    allnl = b"\n" * (255 * 128 * 3 + 77)  # every lane at its 255 limit before a fold
    assert lc._C.count_newlines(allnl) == len(allnl)
    for t in (b"", b"a", b"a\n", b"\n", b"a\n\nb", b"a\nb\n"):
        assert lc._C.count_lines(t) == len(t.split(b"\n")) - (1 if t.endswith(b"\n") or not t else 0)
