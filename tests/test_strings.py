"""Device string library (host side of the __host__ __device__ functions), SURVEY §4 item 1."""
import random

import pytest

from locust_amd.ops import itoa, pack_key, strcmp, strtok_r_tokens
from locust_amd.utils.oracle import DEFAULT_DELIMS


def py_strtok(line: bytes, delims: bytes):
    out, cur = [], bytearray()
    for c in line.split(b"\0", 1)[0]:
        if c in delims:
            if cur:
                out.append(bytes(cur))
                cur = bytearray()
        else:
            cur.append(c)
    if cur:
        out.append(bytes(cur))
    return out


@pytest.mark.parametrize("line", [
    b"", b"   ", b"word", b"  lead and trail  ", b"a,b.c-d;e:f'g(h)i\"j\tk",
    b"to be, or not to be: that is the question",
    b"--..,,", b"x" * 80, b"one,,,,two;;;three",
])
def test_strtok_r_cases(line):
    assert strtok_r_tokens(line, DEFAULT_DELIMS.decode()) == py_strtok(line, DEFAULT_DELIMS)


def test_strtok_r_random():
    rng = random.Random(1)
    alphabet = b"abcXYZ019 ,.-;:'()\"\t"
    for _ in range(2000):
        line = bytes(rng.choice(alphabet) for _ in range(rng.randint(0, 60)))
        assert strtok_r_tokens(line, DEFAULT_DELIMS.decode()) == py_strtok(line, DEFAULT_DELIMS)


@pytest.mark.parametrize("n,base", [(0, 10), (7, 10), (-42, 10), (2147483647, 10),
                                    (-2147483648, 10), (255, 16), (5, 2), (35, 36)])
def test_itoa(n, base):
    digits = "0123456789abcdefghijklmnopqrstuvwxyz"
    def ref(n, b):
        if n == 0:
            return "0"
        neg = n < 0 and b == 10
        u = -n if neg else n & 0xFFFFFFFF
        s = ""
        while u:
            s = digits[u % b] + s
            u //= b
        return ("-" if neg else "") + s
    assert itoa(n, base) == ref(n, base)


def test_strcmp_unsigned_order():
    assert strcmp(b"abc", b"abc") == 0
    assert strcmp(b"ab", b"abc") == -1
    assert strcmp(b"b", b"abc") == 1
    assert strcmp(b"Z", b"a") == -1  # uppercase sorts first
    assert strcmp(b"\xe9", b"z") == 1  # unsigned bytes


def test_pack_key_order_matches_bytes_order():
    rng = random.Random(7)
    keys = [bytes(rng.choice(b"abAB\x7f\x80\xff") for _ in range(rng.randint(1, 31)))
            for _ in range(500)]
    packed = sorted(keys, key=lambda k: pack_key(k))
    assert packed == sorted(keys)


@pytest.mark.gpu
def test_device_string_library_matches_host():
    """the same cases on the device (one thread per string)."""
    import locust_amd as lc

    rng = random.Random(5)
    alphabet = b"abcXYZ019 ,.-;:'()\"\t\x80\xff"
    cases = [b"", b"   ", b"word", b"  lead and trail  ", b"a,b.c-d;e:f'g(h)i\"j\tk",
             b"x" * 60, b"one,,,,two;;;three"]
    cases += [bytes(rng.choice(alphabet) for _ in range(rng.randint(0, 100))).replace(b"\0", b"")
              for _ in range(3000)]
    ints = [rng.randint(-2**31, 2**31 - 1) for _ in cases]
    rows = lc._C.device_string_selftest(cases, ints, DEFAULT_DELIMS.decode())
    for i, (s, row) in enumerate(zip(cases, rows)):
        ln, cmp_next, copy_len, copy, ntok, offs, it = row
        assert ln == len(s)
        if i + 1 < len(cases):
            assert cmp_next == strcmp(s, cases[i + 1])
        assert copy == s[:29] and copy_len == max(0, len(s) - 29)  # chars that did not fit
        starts = [j for j in range(len(s)) if s[j] not in DEFAULT_DELIMS
                  and (j == 0 or s[j - 1] in DEFAULT_DELIMS)]
        assert ntok == len(py_strtok(s, DEFAULT_DELIMS)) == len(starts)
        assert offs == starts[:8]
        assert it == str(ints[i]) and it == itoa(ints[i], 10)


def test_ops_tokenize_matches_oracle():
    """locust_amd.ops.strings.tokenize (host build of d_strtok_r) against the Python strtok."""
    from locust_amd.ops import strings as S

    rng = random.Random(11)
    alphabet = b"abcXYZ019 ,.-;:'()\"\t"
    for _ in range(500):
        s = bytes(rng.choice(alphabet) for _ in range(rng.randint(0, 80)))
        assert S.tokenize(s) == py_strtok(s, DEFAULT_DELIMS)
    assert S.DEFAULT_DELIMS.encode() == DEFAULT_DELIMS


@pytest.mark.gpu
def test_ops_device_check_reports_no_mismatch():
    """The cross-check helper finds the device and host builds in agreement."""
    from locust_amd.ops import strings as S

    rng = random.Random(12)
    cases = [b"", b"a b", b"x" * 40] + [bytes(rng.randrange(1, 256) for _ in range(rng.randint(0, 60)))
                                         for _ in range(500)]
    assert S.device_check(cases, [rng.randint(-2**31, 2**31 - 1) for _ in cases]) == []
