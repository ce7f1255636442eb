"""Streaming (inputs larger than one device pass): line-aligned chunks,
double-buffered H2D, one dictionary across chunks.  Single GPU and distributed shards."""
import pytest

import locust_amd as lc
from locust_amd.utils import oracle

pytestmark = pytest.mark.gpu


def engine(chunk, **kw):
    cfg = lc.make_config("gpu", check=True, chunk_bytes=chunk, **kw)
    return lc._C.GpuEngine(cfg, 1 << 30, 1 << 30)


@pytest.mark.parametrize("chunk", [4096, 32 << 10, 100 << 10])
def test_hamlet_streamed_pageable(hamlet, chunk):
    r = engine(chunk).run(hamlet)
    ent, ntok, _ = oracle.wordcount(hamlet)
    assert r.entries() == ent and r.num_tokens == ntok


def test_hamlet_streamed_pinned_and_repeated(hamlet):
    eng = engine(16 << 10)
    h = lc._C.HostText.from_bytes(hamlet)
    ent = oracle.wordcount(hamlet)[0]
    for _ in range(3):  # buffers and events are reused across runs
        assert eng.run_text(h).entries() == ent
    # a whole-input run on the same engine after streaming ones
    assert eng.run(hamlet[:2000]).entries() == oracle.wordcount(hamlet[:2000])[0]


def test_generated_many_distinct_streamed():
    """> 32K distinct keys: the streamed dictionary is ranked by the radix fallback."""
    t = lc._C.gen_text(lines=60000, seed=3)
    ent, ntok, _ = oracle.wordcount(t)
    assert len(ent) > 32768
    r = engine(512 << 10).run_text(lc._C.HostText.from_bytes(t))
    assert r.num_tokens == ntok
    assert r.entries() == ent


def test_line_longer_than_chunk_is_an_error():
    with pytest.raises(lc.LocustError, match="longer than"):
        engine(64).run(b"a " * 100 + b"\n")


@pytest.mark.parametrize("strategy", ["gather", "shuffle"])
@pytest.mark.parametrize("world", [2, 4])
def test_distributed_streamed_shards(hamlet, strategy, world):
    job = lc.make_config("gpu", combine=True, check=True, chunk_bytes=8 << 10)
    cfgs = [lc.make_dist_config(world, job, strategy=strategy) for _ in range(2)]
    ent, ntok, _ = oracle.wordcount(hamlet)
    for res, info in lc._C.run_multi_schedule(hamlet, cfgs):
        assert res.entries() == ent and res.num_tokens == ntok


@pytest.mark.parametrize("sort", ["dict", "radix"])
def test_ten_million_tokens_vs_cpu_engine(sort):
    """SURVEY §4 item 2 sizes up to 10^7: ~10M tokens through the HBM-table dictionary /
    the onesweep radix sort, checked against the C++ CPU engine (same semantics as the
    oracle, fast enough at this size)."""
    text = lc._C.gen_text(lines=1_600_000, seed=11)
    gpu = lc._C.GpuEngine(lc.make_config("gpu", sort=sort, check=True), len(text), 1_700_000)
    r = gpu.run(text)
    c = lc._C.cpu_run(lc.make_config("cpu"), text)
    assert r.num_tokens == c.num_tokens and r.num_tokens > 9_000_000
    assert r.num_unique == c.num_unique
    assert r.format(False) == c.format(False)


@pytest.mark.gpu
def test_device_exchange_first_job_is_ordered(hamlet):
    """Four ranks sharing the GPU, streamed shards: the first device exchange allocates and
    zeroes its buffers; the zeroing must be ordered with the same job's header upload
    (a null-stream memset once landed after it now and then: a rank's header arrived as
    zeros and the token total came out short).  Repeated, as the race was intermittent."""
    ent, ntok, _ = oracle.wordcount(hamlet)
    for _ in range(20):
        job = lc.make_config("gpu", combine=True, chunk_bytes=8 << 10)
        cfgs = [lc.make_dist_config(4, job, strategy="shuffle") for _ in range(2)]
        for res, info in lc._C.run_multi_schedule(hamlet, cfgs):
            assert res.num_tokens == ntok
            assert res.entries() == ent
