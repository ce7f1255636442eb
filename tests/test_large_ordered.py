"""Large single passes (more than kPartBuildMaxTokens tokens) on the two-kernel ordered
build: line-aligned upload pieces mapped as they land (4 KiB tiles), per-slice partials
(dict_partials_kernel), merge + sort + records (dict_ordered_kernel<PartialsSource>).
Checked against the CPU engine (an independent implementation) on Zipfian synthetic text:
the first job of an engine plans its partition map from its own first piece (partplan.hip)
instead of overflowing the first-byte map, the jobs after it run on the map retuned from
the output; graphs replayed with another text of the same size must not reuse the first
text's pieces."""
import random

import pytest

import locust_amd as lc

pytestmark = pytest.mark.gpu


def cpu_entries(text: bytes):
    return lc._C.cpu_run(lc.make_config("cpu"), text).entries()


def gen(lines, seed=3):
    return lc._C.HostText.generate(lines=lines, seed=seed)


@pytest.mark.parametrize("graph", [0, 1])
def test_pinned_pieces_match_cpu(graph):
    h = gen(220_000)  # ~9.7 MB: pieces of 4 MiB, 4 KiB map tiles
    want = cpu_entries(h.to_bytes())
    eng = lc._C.GpuEngine(lc.make_config("gpu", check=True, graph=graph), h.size, h.size)
    for _ in range(4):
        r = eng.run_text(h)
        assert r.num_unique == len(want)
        assert r.entries() == want


@pytest.mark.parametrize("tune", ["1", "0"])
def test_first_job_plans_its_own_map(monkeypatch, tune):
    """A fresh engine's first large pass (no earlier output to tune from) neither overflows
    nor falls back; with the between-job tuning off every pass plans itself."""
    monkeypatch.setenv("LOCUST_PART_TUNE", tune)
    h = gen(300_000, seed=11)  # ~13 MB
    want = cpu_entries(h.to_bytes())
    eng = lc._C.GpuEngine(lc.make_config("gpu", check=True), h.size, h.size)
    for _ in range(3):
        assert eng.run_text(h).entries() == want
    st = eng.stats()
    assert st["fallbacks"] == 0 and not st["devplan_failed"], st
    if tune == "1":  # the map tuned from the first output (built on a host thread) takes over
        assert st["planned_passes"] >= 1 and st["retunes"] >= 1, st
    else:
        assert st["planned_passes"] == 3 and st["retunes"] == 0, st


def test_staged_bytes_and_small_tiles():
    """Pageable input (staged through the engine's pinned buffer, still in pieces) and a
    2 MB pass below the piece threshold (one map launch, 1 KiB tiles)."""
    for lines in (220_000, 45_000):
        text = gen(lines, seed=5).to_bytes()
        want = cpu_entries(text)
        eng = lc._C.GpuEngine(lc.make_config("gpu", check=True), len(text), text.count(b"\n"))
        for _ in range(3):
            assert eng.run(text).entries() == want


def test_same_size_other_text_replays_correctly():
    """Piece boundaries depend on where the newlines are: a replayed graph must belong to
    the same pieces, not just the same byte count."""
    a = gen(220_000, seed=7).to_bytes()
    lines = a.split(b"\n")[:-1]
    random.Random(1).shuffle(lines)
    b = b"\n".join(lines) + b"\n"
    assert len(a) == len(b) and a != b
    wa, wb = cpu_entries(a), cpu_entries(b)
    eng = lc._C.GpuEngine(lc.make_config("gpu", check=True, graph=1), len(a), len(a))
    for t, w in ((a, wa), (b, wb), (a, wa), (b, wb), (a, wa)):
        assert eng.run(t).entries() == w


def test_many_distinct_keys_fall_back():
    """More distinct keys than the partition tables hold whatever the map: the HBM-table
    path takes over every time, with identical output."""
    rng = random.Random(4)
    words = [b"k%07d" % rng.randrange(3_000_000) for _ in range(600_000)]
    text = b"".join(b" ".join(words[i:i + 12]) + b"\n" for i in range(0, len(words), 12))
    want = cpu_entries(text)
    eng = lc._C.GpuEngine(lc.make_config("gpu", check=True), len(text), text.count(b"\n"))
    for _ in range(2):
        assert eng.run(text).entries() == want


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("strategy", ["shuffle", "gather", "auto"])
def test_one_rank_distributed_large_shard(strategy):
    """A large shard on one RCCL rank: the combining piecewise map + partials + ordered
    build feed the exchange (shuffle), the gather, or -- auto -- the local pipeline; every
    job matches the CPU engine, token count included (the counter snapshot the exchange
    header is built from carries the combining map's token count)."""
    text = gen(220_000, seed=9).to_bytes()
    want = cpu_entries(text)
    ntok = sum(c for _k, _v, c in want)
    dcfg = lc.make_dist_config(1, lc.make_config("gpu", combine=True), strategy=strategy)
    dr = lc._C.DistRank(dcfg, 0, "rccl", "127.0.0.1", _free_port(), len(text),
                        text.count(b"\n"), 60.0)
    for _ in range(3):
        res, info = dr.run(text, 0)
        assert info["strategy"] == ("local" if strategy == "auto" else strategy)
        assert res.num_tokens == ntok
        assert res.entries() == want
