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
def test_cpu_loopback(hamlet, world, combine):
    r = lc.run_multi(hamlet, world, backend="cpu", combine=combine)
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
        lc.run_multi(hamlet, 3, backend="cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("combine,sort", [(True, "dict"), (True, "radix"), (False, "radix")])
def test_gpu_loopback(hamlet, world, combine, sort):
    r = lc.run_multi(hamlet, world, backend="gpu", combine=combine, check=True, sort=sort)
    ent, ntok, _ = oracle.wordcount(hamlet)
    assert r.num_tokens == ntok
    assert r.entries() == ent
