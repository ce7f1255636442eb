"""CPU reference pipeline vs the independent Python oracle."""
import random

import pytest

import locust_amd as lc
from locust_amd.utils import oracle


def run_cpu(text, **kw):
    return lc.wordcount_text(text, backend="cpu", **kw)


@pytest.mark.parametrize("start,end,tokens,unique,the", [
    (0, 700, 4896, 1566, 143),
    (-1, -1, 32940, 5608, 930),
])
def test_hamlet_counts(hamlet, start, end, tokens, unique, the):
    text = oracle.window(hamlet, start, end)
    r = run_cpu(text)
    assert (r.num_tokens, r.num_unique) == (tokens, unique)
    d = {k: c for k, _v, c in r.entries()}
    assert d[b"the"] == the


def test_hamlet_ref_compat_drops_last_line(hamlet):
    r = lc.wordcount_file(lc.REPO_ROOT + "/data/hamlet.txt", backend="cpu", ref_compat=True)
    assert (r.num_tokens, r.num_unique) == (32938, 5607)
    d = {k: c for k, _v, c in r.entries()}
    assert d[b"THE"] == 1


def test_matches_oracle_entries(hamlet):
    text = oracle.window(hamlet, 100, 1400)
    assert run_cpu(text).entries() == oracle.wordcount(text)[0]


def test_emit_cap_and_truncation():
    line = b" ".join(b"w%d" % i for i in range(30))
    text = line + b"\n" + b"x" * 40 + b" short\n"
    r = run_cpu(text)
    ent, ntok, overflow = oracle.wordcount(text)
    assert r.entries() == ent
    assert r.num_tokens == ntok == 22
    assert r.overflow_lines == overflow == 1
    assert r.truncated == 1


def test_random_texts():
    rng = random.Random(3)
    words = [b"alpha", b"Beta", b"gamma", b"d", b"e-mail", b"x" * 35, b"it's"]
    for _ in range(20):
        lines = []
        for _ in range(rng.randint(0, 50)):
            n = rng.randint(0, 30)
            lines.append(b" ".join(rng.choice(words) for _ in range(n)))
        text = b"\n".join(lines) + (b"\n" if rng.random() < 0.5 else b"")
        assert run_cpu(text).entries() == oracle.wordcount(text)[0]


def test_empty_input():
    r = run_cpu(b"")
    assert r.num_tokens == 0 and r.entries() == []


def test_nul_cr_high_bytes():
    """Embedded NUL ends the line's tokens (main.cu:55-59 copies with my_strcpy); '\\r' and
    bytes >= 0x80 are key bytes."""
    rng = random.Random(8)
    words = [b"abc", b"a\0b", b"\0", b"cr\r", b"\xff\xfe", b"caf\xc3\xa9", b"L" * 31, b"it's"]
    for _ in range(20):
        lines = []
        for _ in range(rng.randint(1, 40)):
            n = rng.choice([0, 1, 5, 20, 21, 25])
            lines.append(rng.choice([b" ", b"\0", b"\t"]).join(rng.choice(words) for _ in range(n)))
        text = b"\n".join(lines) + b"\n"
        ent, ntok, overflow = oracle.wordcount(text)
        r = run_cpu(text)
        assert r.entries() == ent and r.num_tokens == ntok and r.overflow_lines == overflow
