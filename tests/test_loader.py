"""The file loader (csrc/io/io.cpp): whole files by parallel preads, line windows read
block by block only up to their last line, and the streamed file source -- every result
the same as the in-memory window of the whole text (the reference's loadFile semantics,
main.cu:40-64, B1 under ref_compat)."""
import os

import pytest

import locust_amd as lc

CASES = [b"", b"a\n", b"a", b"\n\n\n", b"x y\nz", b"one\ntwo\nthree\n"]
WINDOWS = [(-1, -1), (0, 700), (0, 0), (5, 3), (4000, 5000), (0, 4463), (0, 4462), (0, 1),
           (1, 2), (4462, 4463), (4461, 4463), (0, -1), (3, -1), (2, 3), (0, 2), (1, 10)]


@pytest.mark.parametrize("ref_compat", [False, True])
def test_load_lines_matches_in_memory_window(tmp_path, hamlet, ref_compat):
    for i, text in enumerate(CASES + [hamlet, hamlet.rstrip(b"\n")]):
        f = tmp_path / f"t{i}.txt"
        f.write_bytes(text)
        for s, e in WINDOWS:
            got = lc._C.load_lines(str(f), s, e, ref_compat)
            want = lc._C.text_window(text, s, e, ref_compat)
            assert got[:3] == want[:3], (i, s, e, ref_compat)
            if s < 0:
                assert got[3] == want[3]


def test_window_stops_at_its_last_line(tmp_path):
    """A window near the start of a large file reads only its first blocks."""
    big = tmp_path / "big.txt"
    with open(big, "wb") as f:
        f.write(b"alpha beta\n" * 100)
        f.truncate(1 << 30)  # a 1 GiB sparse tail of NUL bytes, never read
    got = lc._C.load_lines(str(big), 10, 20, False)
    assert got[0] == b"alpha beta\n" * 10 and got[1] == 10 and got[2] == 10
    assert got[3] < 1000  # lines scanned, not the whole file


def test_file_source_chunks(tmp_path, hamlet):
    """The streamed source hands out whole lines only, whatever the chunk size."""
    f = tmp_path / "h.txt"
    f.write_bytes(hamlet + b"tail without newline")
    for cap in (4096, 65536, 1 << 20):
        parts, lines = lc._C.file_source_chunks(str(f), cap)
        assert b"".join(parts) == hamlet + b"tail without newline"
        assert all(p.endswith(b"\n") for p in parts[:-1]) and all(len(p) <= cap for p in parts)
        assert lines == hamlet.count(b"\n") + 1


def test_file_source_read_pool(tmp_path, hamlet):
    """Pieces of several MiB are read by the source's persistent reader threads: slices of
    one read land in order and every piece still ends on a line boundary."""
    f = tmp_path / "big.txt"
    body = hamlet * 40  # ~7.6 MB
    f.write_bytes(body)
    for threads in (1, 3, 8):
        parts, lines = lc._C.file_source_chunks(str(f), 3 << 20, threads)
        assert b"".join(parts) == body
        assert all(p.endswith(b"\n") for p in parts) and len(parts) >= 3
        assert lines == body.count(b"\n")
