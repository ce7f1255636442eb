"""The stage split's spill indexes on the launcher side (no native module needed).

Stage 1 writes next to every combined spill a sparse index, ``<spill>.idx``
(csrc/io/io.cpp IndexHeader / IndexRecord: every stride-th record's packed key, record
number, byte offset and the token count before it).  The launcher reads only these -- a
few KiB per spill -- to plan the R key-range reducers exactly as every reducer will
(``plan_splitters`` mirrors ``plan_reducer_splitters``, csrc/engine/stage.cpp), and to
find the byte slice of each spill that reducer r reads (``reducer_slices``): from the
last sample below its range (whose count_before is exact) to the first record at or past
its range's end.  The reducer hosts then pull only those slices peer to peer from the
mapper daemons (sparse files at the spill's own offsets, so the index stays valid);
nothing but the indexes and the result lines passes through the launcher.  Reference:
the shuffle the reference never shipped (/root/reference/README.md:24-29).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

IDX_MAGIC = b"LCSTIDX1"
SPILL_MAGIC = b"LCSTSPL1"
KEY_WORDS = 4
RECORD_BYTES = 40      # binary spill record: 4 key words + count
HEADER = struct.Struct("<8sIIQQQQQQ")   # 64 B
SAMPLE = struct.Struct("<4QQQQQ")       # 64 B
BEYOND = (2**64 - 1,) * KEY_WORDS       # past every key


@dataclass
class SpillIndex:
    sorted: bool
    distinct: bool
    records: int
    total_count: int
    spill_bytes: int
    stride: int
    # (key words, record, offset, count_before)
    samples: list = field(default_factory=list)


def parse_index(data: bytes) -> SpillIndex:
    if len(data) < HEADER.size:
        raise ValueError("short spill index")
    magic, ver, flags, records, total, sbytes, ns, stride, _r = HEADER.unpack_from(data, 0)
    if magic != IDX_MAGIC or ver != 1 or stride < 1 or len(data) < HEADER.size + ns * SAMPLE.size:
        raise ValueError("not a spill index")
    smp = []
    for i in range(ns):
        v = SAMPLE.unpack_from(data, HEADER.size + i * SAMPLE.size)
        smp.append((tuple(v[:KEY_WORDS]), v[4], v[5], v[6]))
    return SpillIndex(bool(flags & 1), bool(flags & 2), records, total, sbytes, stride, smp)


def plan_splitters(idx: list[SpillIndex], reducers: int) -> list[tuple]:
    """reducers - 1 splitter keys cutting all samples at equal record weight (equal keys are
    one unit, so the cut does not depend on the order of `idx`)."""
    if reducers < 1:
        raise ValueError("reducers must be >= 1")
    allw, total = [], 0
    for x in idx:
        s = x.samples
        for j, (key, rec, _off, _cb) in enumerate(s):
            nxt = s[j + 1][1] if j + 1 < len(s) else x.records
            w = nxt - rec if nxt > rec else 1
            allw.append((key, w))
            total += w
    allw.sort(key=lambda t: t[0])
    spl, before, j = [], 0, 0
    for i in range(1, reducers):
        while j < len(allw) and before * reducers < total * i:
            k0 = allw[j][0]
            while j < len(allw) and allw[j][0] == k0:
                before += allw[j][1]
                j += 1
        spl.append(allw[j][0] if j < len(allw) else BEYOND)
    return spl


def reducer_range(spl: list[tuple], r: int):
    """[lo, hi) of reducer r (None: open)."""
    return (spl[r - 1] if r > 0 else None), (spl[r] if r < len(spl) else None)


def reducer_slices(x: SpillIndex, lo, hi) -> list[tuple[int, int]]:
    """Byte ranges (offset, length) of a binary spill that the reducer of [lo, hi) reads:
    the header, then from the last sample below lo to the first record at or past hi
    (inclusive: the reader stops on it)."""
    s = x.samples
    if not s:
        return [(0, x.spill_bytes)]
    first = s[0][2]
    j = 0
    if lo is not None:
        j = max(0, sum(1 for smp in s if smp[0] < lo) - 1)   # samples are in key order
    start = s[j][2]
    end = x.spill_bytes
    if hi is not None:
        q = next((i for i, smp in enumerate(s) if smp[0] >= hi), None)
        if q is not None:
            end = min(x.spill_bytes, s[q][2] + RECORD_BYTES)
    out = [(0, first)]
    if end > start:
        if start <= first:
            out = [(0, end)]
        else:
            out.append((start, end - start))
    return out


def range_record_bytes(records: list[tuple], lo, hi) -> int:
    """Bytes of the binary records (key words, count) with lo <= key < hi (tests, stats)."""
    return RECORD_BYTES * sum(1 for k, _c in records
                              if (lo is None or k >= lo) and (hi is None or k < hi))


def read_binary_spill(data: bytes) -> list[tuple]:
    """(key words, count) records of a binary spill (tests)."""
    magic, ver, kw, count, _r = struct.unpack_from("<8sIIQQ", data, 0)
    if magic != SPILL_MAGIC or ver != 1 or kw != KEY_WORDS:
        raise ValueError("not a binary spill")
    rec = struct.Struct("<4QQ")
    return [(tuple(v[:4]), v[4]) for v in (rec.unpack_from(data, 32 + i * RECORD_BYTES)
                                          for i in range(count))]
