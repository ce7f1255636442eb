"""Independent pure-Python WordCount oracle.

Shares no code with the native engine: tokenization is a direct re-statement of BSD
``strtok_r`` semantics over the reference's delimiter set (main.cu:138), with the
20-emit cap (main.cu:141) and key truncation at 29 bytes.  Sorting is Python's bytes
order == unsigned-byte lexicographic == the reference's KIVComparator (KeyValue.h:20-33).
"""
from __future__ import annotations

from collections import Counter

DEFAULT_DELIMS = b" ,.-;:'()\"\t"


def split_lines(text: bytes) -> list[bytes]:
    lines = text.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    return lines


def tokenize(line: bytes, delims: bytes = DEFAULT_DELIMS, emits: int = 20,
             max_key: int = 29) -> tuple[list[bytes], bool]:
    """Tokens of one line and whether the emit cap dropped any."""
    line = line.split(b"\0", 1)[0]  # strtok_r stops at NUL
    dset = set(delims)
    out: list[bytes] = []
    cur = bytearray()
    for c in line:
        if c in dset:
            if cur:
                out.append(bytes(cur))
                cur = bytearray()
        else:
            cur.append(c)
    if cur:
        out.append(bytes(cur))
    dropped = len(out) > emits
    return [t[:max_key] for t in out[:emits]], dropped


def wordcount(text: bytes, delims: bytes = DEFAULT_DELIMS, emits: int = 20, max_key: int = 29):
    """Returns (entries, num_tokens, overflow_lines): entries = [(key, val, count)] sorted."""
    counter: Counter = Counter()
    overflow = 0
    for line in split_lines(text):
        toks, dropped = tokenize(line, delims, emits, max_key)
        counter.update(toks)
        overflow += dropped
    entries = []
    pos = 0
    for key in sorted(counter):
        entries.append((key, pos, counter[key]))
        pos += counter[key]
    return entries, pos, overflow


def format_gpu(entries) -> bytes:
    """The reference GPU build's result lines (main.cu:132)."""
    return b"".join(b"print key: %s \t val: %d \t count: %d\n" % (k, v, c) for k, v, c in entries)


def format_cpu(entries) -> bytes:
    """The reference CPU build's result lines (main.cu:286)."""
    return b"".join(b"print key: %s \t value: %d\n" % (k, c) for k, _v, c in entries)


def window(text: bytes, line_start: int = -1, line_end: int = -1, ref_compat: bool = False) -> bytes:
    """Lines [line_start, line_end) of text, with the reference's last-line quirk if asked."""
    lines = split_lines(text)
    total = len(lines)
    if line_start < 0:
        first, last = 0, total - (1 if ref_compat and total else 0)
    else:
        first = min(line_start, total)
        last = total if line_end < 0 else min(max(line_end, line_start), total)
        if ref_compat and 0 <= line_end and line_end >= total and last > first:
            last -= 1
    sel = lines[first:last]
    return b"".join(l + b"\n" for l in sel)
