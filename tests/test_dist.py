"""Distributed WordCount: splitter/partition/all-to-all/global-offset logic.

CPU: loopback ranks in one process, and real multi-process ranks over the TCP
communicator.  GPU: loopback ranks on the one GPU of the test box (RCCL refuses two ranks
per device), byte-identical to the single-GPU output including global `val` indices."""
import multiprocessing as mp
import os
import socket

import pytest

import locust_amd as lc
from locust_amd.utils import oracle


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("combine", [True, False])
@pytest.mark.parametrize("strategy", ["shuffle", "gather", "auto"])
def test_cpu_loopback(hamlet, world, combine, strategy):
    r = lc.run_multi(hamlet, world, backend="cpu", combine=combine, strategy=strategy)
    ent, ntok, _ = oracle.wordcount(hamlet)
    assert r.entries() == ent
    assert r.num_tokens == ntok


def test_cpu_loopback_more_ranks_than_lines():
    text = b"b a\nc a\n"
    r = lc.run_multi(text, 8, backend="cpu")
    assert r.entries() == oracle.wordcount(text)[0]


def _rank_main(rank, world, port, text, q):
    import locust_amd as lc2
    try:
        dcfg = lc2.make_dist_config(world, lc2.make_config("cpu", combine=True))
        bounds = lc2._C.shard_bounds(text, world)
        off, nbytes, _nl, first = bounds[rank]
        dr = lc2._C.DistRank(dcfg, rank, "tcp", "127.0.0.1", port, 1, 1, 60.0)
        res, info = dr.run(text[off:off + nbytes], first)
        q.put((rank, res.entries() if rank == 0 else None, info["range_tokens"]))
    except Exception as e:  # report instead of hanging the test
        q.put((rank, "ERR " + repr(e), 0))


@pytest.mark.parametrize("world", [2, 3])
def test_cpu_multiprocess_tcp(hamlet, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, hamlet, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    out.sort(key=lambda t: t[0])
    assert not any(isinstance(o[1], str) for o in out), out
    ent, ntok, _ = oracle.wordcount(hamlet)
    assert out[0][1] == ent
    assert sum(o[2] for o in out) == ntok


def test_fault_injection_clean_failure(hamlet, monkeypatch):
    monkeypatch.setenv("LOCUST_FAULT", "1:reduce")
    with pytest.raises(lc.LocustError, match="stage 'reduce' on rank 1"):
        lc.run_multi(hamlet, 3, backend="cpu", strategy="shuffle")


@pytest.mark.parametrize("fault,match", [("2:map", "stage 'map' on rank 2"),
                                         ("0:reduce", "rank 0")])
def test_fault_injection_gather_strategy(hamlet, monkeypatch, fault, match):
    monkeypatch.setenv("LOCUST_FAULT", fault)
    with pytest.raises(lc.LocustError, match=match):
        lc.run_multi(hamlet, 3, backend="cpu", strategy="gather")


def test_auto_strategy_threshold(hamlet):
    """auto picks gather below gather_max_records and the shuffle above; same output."""
    ent = oracle.wordcount(hamlet)[0]
    for bound, want in [(1 << 20, "gather"), (10, "shuffle")]:
        d = lc.make_dist_config(2, lc.make_config("cpu", combine=True), gather_max_records=bound)
        r = lc._C.run_multi(hamlet, d)
        assert r.entries() == ent, want


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("combine,sort,strategy", [(True, "dict", "auto"), (True, "dict", "shuffle"),
                                                   (True, "radix", "shuffle"),
                                                   (False, "radix", "shuffle"),
                                                   (False, "dict", "gather")])
def test_gpu_loopback(hamlet, world, combine, sort, strategy):
    r = lc.run_multi(hamlet, world, backend="gpu", combine=combine, check=True, sort=sort,
                     strategy=strategy)
    ent, ntok, _ = oracle.wordcount(hamlet)
    assert r.num_tokens == ntok
    assert r.entries() == ent


def _schedule(backend, world):
    job = lc.make_config(backend, combine=True, check=backend == "gpu")
    plan = [("auto", 1 << 20, "gather"),   # predicted shuffle, takes gather
            ("auto", 1 << 20, "gather"),   # predicted gather: unsorted records, root merge
            ("auto", 10, "shuffle"),       # predicted gather, mispredict -> late sampling
            ("auto", 10, "shuffle"),
            ("auto", 1 << 20, "gather"),   # predicted shuffle (sorted records) -> gather
            ("gather", 0, "gather"),
            ("shuffle", 0, "shuffle")]
    cfgs = [lc.make_dist_config(world, job, strategy=s, gather_max_records=m) for s, m, _ in plan]
    return cfgs, [w for _, _, w in plan]


@pytest.mark.parametrize("world", [1, 2, 3])
def test_cpu_strategy_schedule(hamlet, world):
    """Long-lived ranks switching strategies between jobs (plan/mispredict paths)."""
    cfgs, want = _schedule("cpu", world)
    ent, ntok, _ = oracle.wordcount(hamlet)
    for (res, info), w in zip(lc._C.run_multi_schedule(hamlet, cfgs), want):
        assert info["strategy"] == w
        assert res.entries() == ent
        assert res.num_tokens == ntok


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_gpu_strategy_schedule(hamlet, world):
    cfgs, want = _schedule("gpu", world)
    ent, ntok, _ = oracle.wordcount(hamlet)
    for (res, info), w, c in zip(lc._C.run_multi_schedule(hamlet, cfgs), want, cfgs):
        # one rank under auto: the local pipeline, no exchange (DistStrategy::kLocal)
        auto1 = world == 1 and c.strategy == lc._C.DistStrategy.auto
        assert info["strategy"] == ("local" if auto1 else w)
        assert res.entries() == ent
        assert res.num_tokens == ntok


def _distinct_text(n_words, per_line=10):
    words = [b"w%06d" % i for i in range(n_words)]
    return b"".join(b" ".join(words[i:i + per_line]) + b"\n" for i in range(0, n_words, per_line))


@pytest.mark.parametrize("strategy", ["gather", "shuffle"])
def test_cpu_many_distinct(strategy):
    text = _distinct_text(20000)
    r = lc.run_multi(text, 3, backend="cpu", strategy=strategy)
    assert r.entries() == oracle.wordcount(text)[0]


@pytest.mark.gpu
@pytest.mark.parametrize("n_words", [30000, 70000])
def test_gpu_gather_merge_overflow(n_words):
    """Root merge past the root's dense dictionary capacity / the rank-sort range falls
    back to the general reduce; repeated jobs cover the unsorted (gather-planned) records."""
    text = _distinct_text(n_words)
    ent = oracle.wordcount(text)[0]
    job = lc.make_config("gpu", combine=True, check=True)
    cfgs = [lc.make_dist_config(4, job, strategy=s) for s in ("gather", "gather", "shuffle")]
    for res, info in lc._C.run_multi_schedule(text, cfgs):
        assert res.entries() == ent


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_gpu_slot_gather_resizes(world):
    """Gather in one all-gather of fixed-size slots: the first job's slots (2,048 records)
    are too small for ~40,000/world distinct keys per rank, so every rank falls back to the
    standard gather together; the next jobs use slots sized from the headers and merge
    straight from the all-gather buffer."""
    text = _distinct_text(40000) + b"w000001 w000002\n"
    ent = oracle.wordcount(text)[0]
    job = lc.make_config("gpu", combine=True, check=True)
    cfgs = [lc.make_dist_config(world, job, strategy="gather") for _ in range(3)]
    for res, info in lc._C.run_multi_schedule(text, cfgs):
        assert info["strategy"] == "gather"
        assert res.entries() == ent


@pytest.mark.gpu
@pytest.mark.parametrize("fault", ["1:map", "0:reduce"])
def test_gpu_slot_gather_fault(hamlet, monkeypatch, fault):
    """A failing rank's slot header carries the failure: every rank raises (no hang)."""
    monkeypatch.setenv("LOCUST_FAULT", fault)
    job = lc.make_config("gpu", combine=True)
    cfgs = [lc.make_dist_config(3, job, strategy="gather") for _ in range(2)]
    with pytest.raises(lc.LocustError, match="rank"):
        lc._C.run_multi_schedule(hamlet, cfgs)


@pytest.mark.gpu
@pytest.mark.parametrize("slot_graph", ["1", "0", "refused", "refused_late"])
def test_gpu_rccl_one_rank_gather_jobs(hamlet, monkeypatch, slot_graph):
    """One RCCL rank (the pool's boxes have one GPU): repeated gather-strategy jobs take
    the slot path -- with LOCUST_SLOT_GRAPH=1 map + all-gather + merge replay as ONE
    captured graph (the collective inside it), with 0 as separate launches -- and every
    job matches the oracle, including the first (slot overflow -> standard path).
    "refused": the capture fails (injected), so the jobs run the same work uncaptured."""
    if slot_graph == "refused":
        monkeypatch.setenv("LOCUST_FAULT", "0:slot_capture")
    if slot_graph == "refused_late":  # refused after the all-gather was recorded
        monkeypatch.setenv("LOCUST_FAULT", "0:slot_capture_late")
    monkeypatch.setenv("LOCUST_SLOT_GRAPH", "0" if slot_graph == "0" else "1")
    nlines = hamlet.count(b"\n") + (0 if hamlet.endswith(b"\n") else 1)
    dcfg = lc.make_dist_config(1, lc.make_config("gpu", combine=True), strategy="gather")
    dr = lc._C.DistRank(dcfg, 0, "rccl", "127.0.0.1", free_port(), len(hamlet), nlines, 60.0)
    ent, ntok, _ = oracle.wordcount(hamlet)
    for _ in range(4):
        res, info = dr.run(hamlet, 0)
        assert res.num_tokens == ntok
        assert res.entries() == ent


@pytest.mark.gpu
def test_gpu_rccl_failure_after_allgather_entered(hamlet, monkeypatch):
    """A failure after this rank issued the slot all-gather fails the job on this rank
    without entering a second all-gather (the collective sequence must stay in
    step); the next job (replayed graph, hook silent) succeeds."""
    monkeypatch.setenv("LOCUST_FAULT", "0:slot_after_allgather")
    monkeypatch.setenv("LOCUST_SLOT_GRAPH", "1")
    nlines = hamlet.count(b"\n") + (0 if hamlet.endswith(b"\n") else 1)
    dcfg = lc.make_dist_config(1, lc.make_config("gpu", combine=True), strategy="gather")
    dr = lc._C.DistRank(dcfg, 0, "rccl", "127.0.0.1", free_port(), len(hamlet), nlines, 60.0)
    ent, ntok, _ = oracle.wordcount(hamlet)
    # A slot-job shape runs once uncaptured (the hook fires: this rank entered the
    # collective) and is captured + replayed after that (the hook stays silent); which
    # jobs are new shapes depends on the slot size and the scratch state, so only the
    # properties are asserted: failures are clean (no hang, no second all-gather), every
    # successful job is right, and jobs after a failure succeed.
    outcomes = []
    for _ in range(6):
        try:
            res, _ = dr.run(hamlet, 0)
            assert res.entries() == ent and res.num_tokens == ntok
            outcomes.append("ok")
        except lc.LocustError as e:
            assert "after the slot all-gather" in str(e)
            outcomes.append("fail")
    assert "fail" in outcomes and "ok" in outcomes[outcomes.index("fail"):], outcomes
    monkeypatch.delenv("LOCUST_FAULT")
    for _ in range(3):
        res, _ = dr.run(hamlet, 0)
        assert res.entries() == ent and res.num_tokens == ntok


# ---- device-resident shuffle (exch.hpp): one host synchronisation per job ----

@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_gpu_device_exchange_loopback(hamlet, world):
    """Shuffle jobs back to back, all on the device: the first is the sized exchange (two
    host syncs: the all-gathered plans give the exact count matrix), the next the one-sync
    exchange with the slots it sized; every rank writes its range into the shared host
    output, and rank 0's result matches the oracle byte for byte, including the global val."""
    job = lc.make_config("gpu", combine=True, check=True)
    cfgs = [lc.make_dist_config(world, job, strategy="shuffle") for _ in range(4)]
    ent, ntok, _ = oracle.wordcount(hamlet)
    out = lc._C.run_multi_schedule(hamlet, cfgs, "loopback" if world > 1 else "auto")
    # (the schedule keeps every result alive: once they hold both output regions, a job
    # grows the output and writes again -- 2 syncs; see the regions test below)
    assert [i["host_syncs"] for _, i in out][:2] == [2, 1]
    for j, (res, info) in enumerate(out):
        assert info["strategy"] == "shuffle"
        assert info["device_exchange"], (j, info)
        assert res.entries() == ent and res.num_tokens == ntok


@pytest.mark.gpu
def test_gpu_device_exchange_many_keys():
    text = _distinct_text(30000) + b"w000001 w000007 w029999\n" * 3
    ent = oracle.wordcount(text)[0]
    job = lc.make_config("gpu", combine=True, check=True)
    cfgs = [lc.make_dist_config(4, job, strategy="shuffle") for _ in range(3)]
    out = lc._C.run_multi_schedule(text, cfgs, "loopback")
    assert [i["device_exchange"] for _, i in out] == [True, True, True]
    assert [i["host_syncs"] for _, i in out][:2] == [2, 1]
    for res, _ in out:
        assert res.entries() == ent


@pytest.mark.gpu
def test_gpu_device_exchange_outgrown_slots(hamlet, monkeypatch):
    """Slots capped below the data (test hook): every rank sees the overflow in the
    all-gathered reports, every rank redoes the job with the sized exchange (1 + 2 host
    syncs), the slots grow and the next job is a one-sync exchange again."""
    monkeypatch.setenv("LOCUST_EXCH_SLOT", "16")
    job = lc.make_config("gpu", combine=True, check=True)
    cfgs = [lc.make_dist_config(3, job, strategy="shuffle") for _ in range(3)]
    ent = oracle.wordcount(hamlet)[0]
    out = lc._C.run_multi_schedule(hamlet, cfgs, "loopback")
    assert [i["host_syncs"] for _, i in out][:2] == [2, 3]
    for res, _ in out:
        assert res.entries() == ent


@pytest.mark.gpu
@pytest.mark.parametrize("fault", ["1:exchange", "0:exchange"])
def test_gpu_device_exchange_fault(hamlet, monkeypatch, fault):
    """A rank failing inside the device exchange: its header carries the failure through
    the collectives, every rank raises (no hang)."""
    monkeypatch.setenv("LOCUST_FAULT", fault)
    job = lc.make_config("gpu", combine=True)
    cfgs = [lc.make_dist_config(3, job, strategy="shuffle") for _ in range(2)]
    with pytest.raises(lc.LocustError, match="stage 'exchange' on rank " + fault[0]):
        lc._C.run_multi_schedule(hamlet, cfgs, "loopback")


@pytest.mark.gpu
def test_gpu_device_exchange_one_rccl_rank(hamlet):
    """One RCCL rank: ncclAllGather / ncclAllToAll through the real communicator."""
    nlines = hamlet.count(b"\n") + (0 if hamlet.endswith(b"\n") else 1)
    dcfg = lc.make_dist_config(1, lc.make_config("gpu", combine=True, check=True),
                               strategy="shuffle")
    dr = lc._C.DistRank(dcfg, 0, "rccl", "127.0.0.1", free_port(), len(hamlet), nlines, 60.0)
    ent, ntok, _ = oracle.wordcount(hamlet)
    used = []
    for _ in range(4):
        res, info = dr.run(hamlet, 0)
        used.append((info["device_exchange"], info["host_syncs"]))
        assert res.entries() == ent and res.num_tokens == ntok
    assert used == [(True, 2), (True, 1), (True, 1), (True, 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_gpu_device_exchange_async_map_redo(hamlet, monkeypatch, world):
    """One rank's asynchronous map reports an LDS overflow in its exchange header
    (LOCUST_FAULT=<rank>:exch_map_redo): every rank sees it, maps again synchronously and
    runs the device exchange again in the same job; the output is exact."""
    monkeypatch.setenv("LOCUST_FAULT", f"{world - 1}:exch_map_redo")
    job = lc.make_config("gpu", combine=True, check=True)
    cfgs = [lc.make_dist_config(world, job, strategy="shuffle") for _ in range(3)]
    ent, ntok, _ = oracle.wordcount(hamlet)
    out = lc._C.run_multi_schedule(hamlet, cfgs, "loopback")
    for j, (res, info) in enumerate(out):
        assert info["device_exchange"], (j, info)
        assert res.entries() == ent and res.num_tokens == ntok


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_gpu_shared_output_regions_held_by_results(hamlet, world):
    """The root lends a shared-output region to each result: results kept alive across
    jobs (three at once, two regions) make the root announce 'no free region' -- every rank
    grows the output and writes its range again -- and every kept result stays intact."""
    job = lc.make_config("gpu", combine=True, check=True)
    nlines = hamlet.count(b"\n") + (0 if hamlet.endswith(b"\n") else 1)
    cfgs = [lc.make_dist_config(world, job, strategy="shuffle") for _ in range(5)]
    ent, ntok, _ = oracle.wordcount(hamlet)
    out = lc._C.run_multi_schedule(hamlet, cfgs, "loopback")
    # every result of the schedule is alive at the end (the list holds them)
    for res, info in out:
        assert info["device_exchange"]
        assert res.entries() == ent and res.num_tokens == ntok
    syncs = [i["host_syncs"] for _, i in out]
    assert syncs[0] == 2 and 2 in syncs[1:] and max(syncs) == 2, syncs
    assert nlines > 0
