"""Compact result records: the ordered kernels drain their output to
host memory as variable-length runs of 8-B words (csrc/include/locust/kv.hpp), one segment
per virtual partition, and EntryList decodes them on the fly.  Here: the host decoder on
hand-built segments against the packed-key oracle; the GPU twin (the kernels' own compact
output byte-identical to the CPU engine, and the wire bytes it saves) is
tests/test_gpu_engine.py::test_compact_output_*."""
import struct

import pytest

import locust_amd as lc
from locust_amd.utils import oracle


def _pack(key: bytes):
    key = key.ljust(32, b"\0")
    return [struct.unpack(">Q", key[8 * j:8 * j + 8])[0] for j in range(4)]


def _record(key: bytes, count: int):
    """kv.hpp's compact record, written independently: short form (count < 2^24) packs key
    bytes 0-3 into the header word, then key bytes 4.. in 8-byte words; long form keeps a
    56-bit count and the packed key words."""
    kb = len(key.rstrip(b"\0"))
    if count < (1 << 24):
        head = (int.from_bytes(key[:4].ljust(4, b"\0"), "big") << 32) | (count << 8) | (kb << 1)
        rest = key[4:kb]
        extra = [int.from_bytes(rest[i:i + 8].ljust(8, b"\0"), "big") for i in range(0, len(rest), 8)]
        return [head] + extra
    w = _pack(key)
    return [(count << 8) | (kb << 1) | 1] + w[:(kb + 7) // 8]


def test_decode_segments_with_gaps_and_empty():
    keys = [(b"a", 3), (b"abcd", 5), (b"abcde", 1 << 24), (b"abcdefgh", 1), (b"abcdefghi", 7),
            (b"abcdefghijkl", 2), (b"abcdefghijklm", 3), (b"b" * 17, 2), (b"b" * 20, 1 << 30),
            (b"z" * 29, 4), (b"z" * 31, 9), (b"zz", 1)]
    words, segs = [], []
    # segment 0: two records; then a gap (the kernel leaves room for 40-B records); an
    # empty segment; segment 2: the rest
    seg0 = _record(*keys[0]) + _record(*keys[1])
    words += seg0 + [0xdeadbeef] * 5
    segs.append((0, 2))
    segs.append((len(words), 0))
    start = len(words)
    for k, c in keys[2:]:
        words += _record(k, c)
    segs.append((start, len(keys) - 2))
    r = lc._C.Result.from_compact(words, segs, val_base=100)
    assert r.compact and r.num_unique == len(keys)
    ent = r.entries()
    assert [(k, c) for k, _v, c in ent] == keys
    vals = [v for _k, v, _c in ent]
    assert vals[0] == 100 and vals == [100 + sum(c for _k, c in keys[:i]) for i in range(len(keys))]
    # the wire bytes are the records' words, not the gap
    assert r.wire_bytes == 8 * (len(seg0) + sum(len(_record(k, c)) for k, c in keys[2:]))
    assert r.wire_bytes < 40 * len(keys)
    # the formatted output is the oracle's
    want = [(k, 100 + sum(c for _k, c in keys[:i]), c) for i, (k, c) in enumerate(keys)]
    assert r.format() == b"".join(b"print key: %s \t val: %d \t count: %d\n" % e for e in want)


def test_decode_hamlet_sized(hamlet):
    ent = oracle.wordcount(hamlet)[0]
    words, segs, at = [], [], 0
    for i in range(0, len(ent), 97):  # 97-entry segments
        chunk = ent[i:i + 97]
        segs.append((len(words), len(chunk)))
        for k, _v, c in chunk:
            words += _record(k, c)
    r = lc._C.Result.from_compact(words, segs)
    assert r.entries() == ent
    assert r.wire_bytes / len(ent) < 15  # English keys: one or two words per entry (14.1 B)


@pytest.mark.gpu
def test_gpu_compact_long_counts():
    """Counts of 2^24 and more take the long record form (kv.hpp): two keys past it -- one
    of 2 bytes, one of 13 -- through the large-pass ordered kernel, next to short-form keys."""
    n1, n2 = (1 << 24) + 8, (1 << 24) + 16
    text = (b"aa aa aa aa aa aa aa aa\n" * (n1 // 8) + b"bbbbbbbbbbbbb bbbbbbbbbbbbb\n" * (n2 // 2)
            + b"".join(b"zebra%d\n" % i for i in range(1000)))
    r = lc.wordcount_text(text, backend="gpu")
    assert r.compact
    ent = r.entries()
    assert ent[0] == (b"aa", 0, n1) and ent[1] == (b"bbbbbbbbbbbbb", n1, n2)
    assert len(ent) == 1002 and all(c == 1 for _k, _v, c in ent[2:])
    assert sorted(k for k, _v, _c in ent[2:]) == sorted(b"zebra%d" % i for i in range(1000))
