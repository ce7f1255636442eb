"""GPU pipeline vs oracle: every kernel path (map compat/fast, reduce lds/global, planned
and device-planned radix passes), edge cases, and sizes around the reference's 32,768-thread
truncation (bug B3)."""
import random

import pytest

import locust_amd as lc
from locust_amd.utils import oracle

pytestmark = pytest.mark.gpu

PATHS = [
    dict(map_path="fast", reduce_path="lds", sort="dict"),
    dict(map_path="compat", reduce_path="lds", sort="dict"),
    dict(map_path="fast", reduce_path="lds"),
    dict(map_path="fast", reduce_path="global"),
    dict(map_path="compat", reduce_path="lds"),
    dict(map_path="compat", reduce_path="global"),
    dict(map_path="fast", reduce_path="lds", sync_plan=False),
    dict(map_path="fast", reduce_path="lds", sort="dict", zero_copy_text=0),
    dict(map_path="fast", reduce_path="lds", sort="dict", zero_copy_text=1),
]


def gpu(text, **kw):
    return lc.wordcount_text(text, backend="gpu", check=True, **kw)


@pytest.mark.parametrize("opts", PATHS, ids=lambda o: "-".join(f"{v}" for v in o.values()))
@pytest.mark.parametrize("start,end", [(0, 700), (-1, -1)])
def test_hamlet_matches_oracle(hamlet, opts, start, end):
    text = oracle.window(hamlet, start, end)
    ent, ntok, _ = oracle.wordcount(text)
    r = gpu(text, **opts)
    assert r.num_tokens == ntok
    assert r.entries() == ent
    assert r.format() == oracle.format_gpu(ent)


def test_hamlet_known_numbers(hamlet):
    r = gpu(hamlet)
    assert (r.num_tokens, r.num_unique) == (32940, 5608)
    d = {k: (v, c) for k, v, c in r.entries()}
    assert d[b"the"][1] == 930 and d[b"THE"][1] == 2
    # B3 regression: keys whose runs start past index 32,768 get their own heads
    for k in (b"yours", b"yourself", b"yourselves", b"youth", b"zone"):
        assert k in d


@pytest.mark.parametrize("opts", PATHS[:5], ids=["dict", "compat-dict", "fast-lds", "fast-global", "compat-lds"])
def test_random_texts(opts):
    rng = random.Random(11)
    words = [b"alpha", b"Beta", b"gamma", b"d", b"e-mail", b"x" * 35, b"it's", b"\xc3\xa9t\xc3\xa9"]
    for trial in range(12):
        lines = []
        for _ in range(rng.randint(0, 400)):
            n = rng.choice([0, 1, 5, 19, 20, 21, 40])
            sep = rng.choice([b" ", b",  ", b"--", b"\t"])
            lines.append(sep.join(rng.choice(words) for _ in range(n)))
        text = b"\n".join(lines) + (b"\n" if trial % 2 else b"")
        ent, ntok, overflow = oracle.wordcount(text)
        r = gpu(text, **opts)
        assert r.entries() == ent
        assert r.num_tokens == ntok
        assert r.overflow_lines == overflow


@pytest.mark.parametrize("sort", ["radix", "dict"])
@pytest.mark.parametrize("ntok", [1, 2, 4095, 4096, 8192, 8193, 32768, 32769, 100003])
def test_sizes_around_tiles(ntok, sort):
    rng = random.Random(ntok)
    vocab = [bytes(rng.choice(b"abcdefghij") for _ in range(rng.randint(1, 12))) for _ in range(3000)]
    toks = [rng.choice(vocab) for _ in range(ntok)]
    text = b"\n".join(b" ".join(toks[i:i + 10]) for i in range(0, ntok, 10)) + b"\n"
    ent, n, _ = oracle.wordcount(text)
    assert n == ntok
    assert gpu(text, sort=sort).entries() == ent


@pytest.mark.parametrize("nuniq", [32768, 32769, 70000])
def test_dict_many_distinct_keys(nuniq):
    # distinct-key counts around the rank-sort / radix-fallback boundary
    rng = random.Random(nuniq)
    vocab = [b"k%07d%s" % (i, bytes(rng.choice(b"xyz") for _ in range(rng.randint(0, 20)))) for i in range(nuniq)]
    toks = vocab + [rng.choice(vocab) for _ in range(nuniq // 3)]
    rng.shuffle(toks)
    text = b"\n".join(b" ".join(toks[i:i + 8]) for i in range(0, len(toks), 8))
    ent, n, _ = oracle.wordcount(text)
    r = gpu(text, sort="dict")
    assert r.num_unique == nuniq and r.entries() == ent


def test_long_lines_segment_boundaries():
    # lines far longer than a 1 KiB wave segment and the 4 KiB tile: the carried per-line
    # ordinal (20-emit cap) must survive segment and tile boundaries.
    rng = random.Random(5)
    lines = []
    for _ in range(50):
        n = rng.randint(0, 3000)
        lines.append(b" " * rng.randint(0, 3000) + b" ".join(b"w%d" % rng.randint(0, 50) for _ in range(n)))
    text = b"\n".join(lines)
    ent, ntok, overflow = oracle.wordcount(text)
    r = gpu(text)
    assert r.entries() == ent and r.overflow_lines == overflow


NASTY_WORDS = [b"abc", b"a\0b", b"\0", b"x\0\0y", b"cr\r", b"\r", b"\xff\xfe", b"\x80z",
               b"caf\xc3\xa9", b"L" * 31, b"M" * 29, b"N" * 30, b"q" * 70, b"it's", b"\x01\x7f"]


@pytest.mark.parametrize("opts", PATHS[:6], ids=["dict", "compat-dict", "fast-lds", "fast-global",
                                                 "compat-lds", "compat-global"])
def test_nul_cr_high_bytes_long_tokens(opts):
    """An embedded NUL ends its line's token stream (my_strcpy stops there, main.cu:55-59);
    '\r' and bytes >= 0x80 are ordinary key bytes; tokens over 29 bytes are truncated."""
    rng = random.Random(77)
    for trial in range(10):
        lines = []
        for _ in range(rng.randint(1, 300)):
            n = rng.choice([0, 1, 3, 19, 20, 21, 25])
            sep = rng.choice([b" ", b", ", b"\t", b"\0", b" \0 "])
            lines.append(sep.join(rng.choice(NASTY_WORDS) for _ in range(n)))
        text = b"\n".join(lines) + (b"\n" if trial % 2 else b"")
        ent, ntok, overflow = oracle.wordcount(text)
        r = gpu(text, **opts)
        assert r.entries() == ent, trial
        assert r.num_tokens == ntok
        assert r.overflow_lines == overflow


@pytest.mark.parametrize("sort", ["dict", "radix"])
def test_nul_across_segments_and_tiles(sort):
    """A NUL far before a wave segment / tile boundary still kills the rest of the line,
    and the next line starts live again (the carried dead state resets at '\n')."""
    rng = random.Random(9)
    lines = []
    for i in range(60):
        pre = b" ".join(b"p%d" % rng.randint(0, 30) for _ in range(rng.randint(0, 25)))
        post = b" ".join(b"d%d" % rng.randint(0, 30) for _ in range(rng.randint(0, 900)))
        pad = b" " * rng.randint(0, 5000)
        nul = b"\0" if i % 3 else b" "
        lines.append(pre + pad + nul + pad + post)
    text = b"\n".join(lines) + b"\n"
    ent, ntok, overflow = oracle.wordcount(text)
    r = gpu(text, sort=sort)
    assert r.entries() == ent and r.num_tokens == ntok and r.overflow_lines == overflow


def test_empty_and_delimiter_only():
    for text in (b"", b"\n\n\n", b" ,.;\n--\n"):
        r = gpu(text)
        assert r.num_tokens == 0 and r.entries() == []


@pytest.mark.parametrize("kind,n", [("equal_runs", 50000), ("all_equal", 9000),
                                    ("descending", 8192), ("descending", 8193),
                                    ("every_length", 29 * 400), ("random", 100003)])
def test_sort_keys_shapes(kind, n):
    """radix sort vs Python sort on equal runs, all-equal, descending and
    1..29-byte keys, across the single-workgroup / onesweep boundary (8,192)."""
    rng = random.Random(n)
    if kind == "equal_runs":
        pool = [bytes(rng.choice(b"abcdefgh") for _ in range(rng.randint(1, 12))) for _ in range(300)]
        keys = [rng.choice(pool) for _ in range(n)]
    elif kind == "all_equal":
        keys = [b"same"] * n
    elif kind == "descending":
        keys = sorted((b"k%08d" % i for i in range(n)), reverse=True)
    elif kind == "every_length":
        keys = [bytes(rng.choice(b"xyz") for _ in range(1 + i % 29)) for i in range(n)]
    else:
        keys = [bytes(rng.choice(b"aZ09~") for _ in range(rng.randint(1, 29))) for _ in range(n)]
    eng = lc.Engine(lc.make_config("gpu"), 1 << 22, 1 << 18)
    s, perm = eng.sort_keys(keys)
    assert s == sorted(keys)
    assert [keys[i] for i in perm] == s
    assert all(a < b for a, b in zip(perm, perm[1:]) if keys[a] == keys[b])  # stable


def test_sort_keys_random():
    rng = random.Random(2)
    keys = [bytes(rng.choice(b"aZ09\x80\xff~") for _ in range(rng.randint(1, 31))) for _ in range(50000)]
    eng = lc.Engine(lc.make_config("gpu"), 1 << 20, 1 << 16)
    s, perm = eng.sort_keys(keys)
    assert s == sorted(keys)
    assert [keys[i] for i in perm] == s
    # stability: equal keys keep input order
    for a, b in zip(perm, perm[1:]):
        if keys[a] == keys[b]:
            assert a < b


def test_engine_reuse_and_stage_split(hamlet):
    text = oracle.window(hamlet, 0, 1000)
    eng = lc.Engine(lc.make_config("gpu"), len(hamlet) + 1, 5000)
    r1 = eng.run(text).entries()
    r2 = eng.run(oracle.window(hamlet, 1000, 2000)).entries()
    r3 = eng.run(text).entries()
    assert r1 == r3 == oracle.wordcount(text)[0]
    assert r2 == oracle.wordcount(oracle.window(hamlet, 1000, 2000))[0]
    toks = eng.map_stage(text)
    assert toks == sorted(toks) and len(toks) == 7061 or len(toks) == oracle.wordcount(text)[1]
    red = eng.reduce_stage(list(reversed(toks)))
    assert red.entries() == r1


@pytest.mark.parametrize("sort", ["dict", "radix"])
def test_reference_semantics_timers(hamlet, sort):
    """--ref-timers: same output; Map is launch-only, Process includes the map kernel."""
    r = gpu(hamlet, sort=sort, ref_timers=True, graph=0)
    assert r.entries() == oracle.wordcount(hamlet)[0]
    t = r.times()
    assert t["ref_map_ms"] > 0 and t["ref_process_ms"] > 0 and t["ref_reduce_ms"] > 0
    assert t["ref_map_ms"] < t["ref_process_ms"]


@pytest.mark.parametrize("graph", [0, 1])
def test_graph_replay_repeated(hamlet, graph):
    """The captured job replays correctly across runs and input changes (re-capture)."""
    cfg = lc.make_config("gpu", check=True, graph=graph)
    eng = lc._C.GpuEngine(cfg, len(hamlet), 5000)
    for text in (hamlet, hamlet, oracle.window(hamlet, 0, 700), hamlet):
        r = eng.run(text)
        assert r.entries() == oracle.wordcount(text)[0]
        assert r.times()["graph"] == bool(graph)


@pytest.mark.parametrize("kind", ["one_partition_overflow", "many_keys_balanced"])
def test_ordered_partitions_edge_cases(kind):
    """The one-kernel ordered Process/Reduce: a partition (first key byte) with more
    distinct keys than its LDS table falls back to the HBM table; > 32K distinct keys
    spread over partitions are emitted directly."""
    if kind == "one_partition_overflow":
        words = [b"w%06d" % i for i in range(40000)]
    else:
        words = [bytes([97 + i % 26]) + b"%05d" % i for i in range(40000)]
    text = b"".join(b" ".join(words[i:i + 10]) + b"\n" for i in range(0, len(words), 10))
    ent, ntok, _ = oracle.wordcount(text)
    r = gpu(text, graph=0)
    assert r.num_tokens == ntok and r.entries() == ent


@pytest.mark.parametrize("graph", [0, 1])
def test_zero_copy_results_stay_valid(hamlet, graph):
    """Results adopt the host-mapped buffer their job wrote: results kept alive across
    later jobs (different texts, a radix-path fallback, a self-cleaned replay) keep their
    own entries; dropped results give their buffers back for reuse."""
    cfg = lc.make_config("gpu", check=True, graph=graph)
    eng = lc._C.GpuEngine(cfg, len(hamlet) + 1, 1 << 16)
    texts = [hamlet, oracle.window(hamlet, 0, 700), hamlet, oracle.window(hamlet, 2000, 4000)]
    many = b"".join(b"k%06d\n" % i for i in range(40000))  # > 32K distinct: radix emit
    kept = [(t, eng.run(t)) for t in texts + [many]]
    for _ in range(6):  # dropped results: their buffers are reused
        assert eng.run(hamlet).num_unique == 5608
    for t, r in kept:
        assert r.entries() == oracle.wordcount(t)[0]
    kept.clear()
    r = eng.run(hamlet)
    assert r.entries() == oracle.wordcount(hamlet)[0]


@pytest.mark.parametrize("default_map", ["letters", "byte"])
@pytest.mark.parametrize("plan_min_kb", ["0", "256"])
def test_starting_map_and_in_job_plan_match_oracle(hamlet, monkeypatch, default_map, plan_min_kb):
    """An untuned engine (LOCUST_PART_TUNE=0) on the starting partition map -- letters split
    on the second byte, or the first-byte map -- with the in-job plan forced on (every pass
    plans; the first-byte map then splits the hot letters over sibling workgroups) or left
    to its size threshold: every job matches the oracle."""
    monkeypatch.setenv("LOCUST_PART_TUNE", "0")
    monkeypatch.setenv("LOCUST_VPLAN_MIN_KB", plan_min_kb)
    if default_map == "byte":
        monkeypatch.setenv("LOCUST_PART_DEFAULT", "byte")
    for start, end in [(-1, -1), (0, 700), (1000, 3000)]:
        text = oracle.window(hamlet, start, end)
        ent, ntok, _ = oracle.wordcount(text)
        eng = lc._C.GpuEngine(lc.make_config("gpu", reduce_path="lds", check=True), len(text),
                              text.count(b"\n") + 1)
        for _ in range(3):
            r = eng.run(text)
            assert r.num_tokens == ntok and r.entries() == ent


@pytest.mark.parametrize("mode", ["trigger", "always", "off"])
def test_crowded_partition_plans_and_stays_in_lds(monkeypatch, mode):
    """12,000 distinct keys that all fall into one partition of the starting map ('w0...'):
    every 1 KiB tile holds far more than kPlanTrigger tokens of it, so the map raises the
    plan flag, the ordered kernel splits the partition over sibling workgroups and the job
    stays on the LDS path -- with the trigger and with the plan forced in every job
    (LOCUST_PLAN_TRIGGER=0).  Without the plan (LOCUST_VPLAN=0) the one LDS table
    overflows and the job takes the HBM-table fallback (same entries).  (Past ~16 K tokens
    in one partition a sibling's token list overflows too: the fallback again.)  Whole
    Hamlet never raises the flag (27 tokens of one partition per tile at most)."""
    monkeypatch.setenv("LOCUST_PART_TUNE", "0")
    if mode == "always":
        monkeypatch.setenv("LOCUST_PLAN_TRIGGER", "0")
    if mode == "off":
        monkeypatch.setenv("LOCUST_VPLAN", "0")
    words = [b"w%05d" % i for i in range(12000)]
    text = b"\n".join(b" ".join(words[i:i + 10]) for i in range(0, len(words), 10)) + b"\n"
    ent, ntok, _ = oracle.wordcount(text)
    eng = lc._C.GpuEngine(lc.make_config("gpu", reduce_path="lds", check=True), len(text),
                          text.count(b"\n") + 1)
    for _ in range(2):
        r = eng.run(text)
        assert r.num_tokens == ntok and r.entries() == ent
    assert (eng.stats()["fallbacks"] == 0) == (mode != "off"), eng.stats()


@pytest.mark.parametrize("graph", [-1, 0, 1])
def test_compact_output_hamlet(hamlet, graph):
    """The ordered kernel drains compact records (kv.hpp) into host memory: byte-identical
    entries, and fewer bytes across PCIe than 40 per entry.  graph -1
    (auto, lean launches), 0 (event-timed) and 1 (replayed graph) each keep the flag."""
    cfg = lc.make_config("gpu", reduce_path="lds", check=True, graph=graph)
    eng = lc._C.GpuEngine(cfg, len(hamlet), 5000)
    eng.load(hamlet)
    ent = oracle.wordcount(hamlet)[0]
    for _ in range(3):
        r = eng.run_loaded()
        assert r.compact and r.entries() == ent
    assert r.wire_bytes < 0.55 * 40 * len(ent), r.wire_bytes


def test_compact_output_large_ordered():
    """A one-pass synthetic input past kPartBuildMaxTokens: the partials + ordered kernels
    (PartialsSource) write compact records too; long keys (up to 31 bytes) use 4 words."""
    text = lc._C.HostText.generate(lines=120000, seed=3, first_block=0).to_bytes()
    text += b"".join(b"%s\n" % (b"x" * n + b"%d" % n) for n in range(1, 30))
    want = lc._C.cpu_run(lc.make_config("cpu"), text)
    cfg = lc.make_config("gpu", reduce_path="lds", check=True)
    eng = lc._C.GpuEngine(cfg, len(text), text.count(b"\n") + 1)
    eng.load(text)
    for _ in range(2):
        r = eng.run_loaded()
        assert r.compact and r.entries() == want.entries()
        assert r.wire_bytes < 0.6 * 40 * r.num_unique
