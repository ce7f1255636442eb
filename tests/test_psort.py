"""Partitioned LDS radix sort (psort.hip): the reference algorithm's Process stage on the
small-input fast map's partition table, against the oracle and against the device-wide
LSD sort (LOCUST_PSORT=0).  Covers partitions over the LDS capacity (device-wide fallback),
keys reaching the third and fourth packed words, keys of exactly 8/16/24 bytes, a retuned
partition map, graph replay, the reference-semantics timers and the map-stage entry point."""
import os
import random

import pytest

import locust_amd as lc
from locust_amd.utils import oracle

pytestmark = pytest.mark.gpu


def radix(text, **kw):
    return lc.wordcount_text(text, backend="gpu", sort="radix", check=True, **kw)


def lines_of(words, per=10):
    return b"".join(b" ".join(words[i:i + per]) + b"\n" for i in range(0, len(words), per))


@pytest.mark.parametrize("graph", [0, 1])
def test_hamlet_radix_repeated_with_retune(hamlet, graph):
    """Whole Hamlet on one engine, job after job: the first job sorts with the first-byte
    partition map, later ones with the map retuned from its output (and replayed graphs)."""
    cfg = lc.make_config("gpu", sort="radix", check=True, graph=graph)
    eng = lc._C.GpuEngine(cfg, len(hamlet) + 1, 5000)
    want = oracle.wordcount(hamlet)[0]
    for text in (hamlet, hamlet, oracle.window(hamlet, 0, 700), hamlet, hamlet):
        r = eng.run(text)
        assert r.entries() == oracle.wordcount(text)[0]
    assert eng.run(hamlet).entries() == want


def test_partition_over_lds_capacity_falls_back():
    """One first byte with > kPsortMax (5,120) tokens: that partition overflows and the
    device-wide sort redoes the pass; the result is identical."""
    rng = random.Random(3)
    words = [b"a%d" % rng.randint(0, 5000) for _ in range(20000)]
    words += [b"b%d" % rng.randint(0, 50) for _ in range(3000)]
    text = lines_of(words)
    ent, ntok, _ = oracle.wordcount(text)
    r = radix(text, graph=0)
    assert r.num_tokens == ntok and r.entries() == ent
    r = radix(text, graph=1)
    assert r.entries() == ent


@pytest.mark.parametrize("width", [7, 8, 9, 15, 16, 17, 23, 24, 25, 29, 35])
def test_long_keys_reach_every_word(width):
    """Keys sharing long prefixes differ only in their 2nd/3rd/4th packed word; truncation
    at 29 bytes makes some of them equal."""
    rng = random.Random(width)
    stem = b"x" * max(width - 3, 0)
    words = [stem + bytes(rng.choice(b"abc") for _ in range(min(3, width))) for _ in range(6000)]
    words += [bytes(rng.choice(b"xy") for _ in range(rng.randint(1, width))) for _ in range(3000)]
    rng.shuffle(words)
    text = lines_of(words, 15)
    ent, ntok, _ = oracle.wordcount(text)
    r = radix(text)
    assert r.num_tokens == ntok and r.entries() == ent


def test_psort_matches_device_wide_sort(hamlet, monkeypatch):
    """A/B: identical output with the partitioned sort and the device-wide LSD sort."""
    rng = random.Random(17)
    vocab = [bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyzABC'") for _ in range(rng.randint(1, 14)))
             for _ in range(4000)]
    texts = [hamlet, oracle.window(hamlet, 100, 900),
             lines_of([rng.choice(vocab) for _ in range(30000)], 12)]
    for text in texts:
        a = radix(text, graph=0)
        monkeypatch.setenv("LOCUST_PSORT", "0")
        b = radix(text, graph=0)
        monkeypatch.delenv("LOCUST_PSORT")
        assert a.entries() == b.entries() == oracle.wordcount(text)[0]


def test_ref_timers_and_map_stage(hamlet):
    """The reference-semantics timed run and the stage-1 entry point also sort with the
    partitioned kernel, including the overflow fallback."""
    big = lines_of([b"a%d" % (i % 7000) for i in range(20000)])
    for text in (hamlet, big):
        r = radix(text, ref_timers=True, graph=0)
        assert r.entries() == oracle.wordcount(text)[0]
        eng = lc.Engine(lc.make_config("gpu", sort="radix"), len(text) + 1, text.count(b"\n") + 1)
        toks = eng.map_stage(text)
        assert len(toks) == oracle.wordcount(text)[1]
        assert toks == sorted(toks)


def test_single_partition_all_equal_and_tiny():
    for text in (b"same " * 5000 + b"\n", b"x\n", b"a b\n", b"b a a\n" * 3):
        r = radix(text)
        assert r.entries() == oracle.wordcount(text)[0]
