"""The device string library (csrc/include/locust/dstring.hpp) from Python: the host build
of the same ``__host__ __device__`` functions the map kernels run on the GPU (reference
util.cu:3-139 -- d_strlen, d_strcmp, d_strcpy, d_strtok_r, reverse/itoa), a tokenizer
with the reference's delimiter rules, and a device-vs-host cross-check that runs every
function on the GPU (one thread per string) and reports where the two builds differ.
"""
from __future__ import annotations

from dataclasses import dataclass

from .._native import load

_C = load()

#: the reference's delimiter set (space, tab and ,.-;:'()" -- dstring.hpp kDefaultDelims)
DEFAULT_DELIMS = " ,.-;:'()\"\t"
#: KeyIntValuePair::key[30]: 29 characters and the NUL (KeyValue.h:13-18)
MAX_KEY_LEN = 29

strtok_r_tokens = _C.strtok_r_tokens
itoa = _C.itoa
strcmp = _C.strcmp
pack_key = _C.pack_key


def tokenize(line: bytes | str, delims: str = DEFAULT_DELIMS) -> list[bytes]:
    """The tokens d_strtok_r yields for `line` (the reference's map() loop, util.cu:101-139),
    as byte strings, in order."""
    b = line.encode() if isinstance(line, str) else bytes(line)
    return [bytes(t) for t in strtok_r_tokens(b, delims)]


@dataclass
class StringMismatch:
    """One field where the GPU build of a string function disagreed with the host build."""
    index: int
    field: str
    device: object
    host: object


def _host_row(s: bytes, nxt: bytes | None, n: int, delims: str):
    starts = [j for j in range(len(s)) if chr(s[j]) not in delims
              and (j == 0 or chr(s[j - 1]) in delims)]
    return {
        "len": len(s),
        "cmp_next": None if nxt is None else strcmp(s, nxt),
        "copy": s[:MAX_KEY_LEN],
        "copy_len": max(0, len(s) - MAX_KEY_LEN),
        "ntok": len(starts),
        "offsets": starts[:8],
        "itoa": itoa(n, 10),
    }


def device_check(strings: list[bytes], ints: list[int] | None = None,
                 delims: str = DEFAULT_DELIMS) -> list[StringMismatch]:
    """Run strlen / strcmp (with the next string) / bounded strcpy / strtok_r / itoa on the
    GPU for every string (device_string_selftest) and compare each field with the host
    build.  Returns the mismatches (empty: the two builds agree).  Needs a GPU."""
    strings = [bytes(s).replace(b"\0", b"") for s in strings]
    ints = list(ints) if ints is not None else [len(s) for s in strings]
    if len(ints) != len(strings):
        raise ValueError("device_check: one int per string")
    rows = _C.device_string_selftest(strings, ints, delims)
    bad: list[StringMismatch] = []
    for i, (s, row) in enumerate(zip(strings, rows)):
        ln, cmp_next, copy_len, copy, ntok, offs, it = row
        dev = {"len": ln, "cmp_next": cmp_next if i + 1 < len(strings) else None,
               "copy": bytes(copy), "copy_len": copy_len, "ntok": ntok, "offsets": list(offs),
               "itoa": it}
        host = _host_row(s, strings[i + 1] if i + 1 < len(strings) else None, ints[i], delims)
        for k, hv in host.items():
            if dev[k] != hv:
                bad.append(StringMismatch(i, k, dev[k], hv))
    return bad
