"""Several processes sharing one GPU, each running back-to-back whole-Hamlet jobs.

Every look-back chain in the kernels (ordered Process+Reduce, root merge, scans) takes its
tile from a ticket, so a workgroup only waits on workgroups that are already running.
Tiles taken from blockIdx instead let kernels of different processes fill the CUs with
workgroups spinning on predecessors that were never dispatched: the 4-rank TCP rehearsal
on one GPU showed multi-second stalls and a hang.  This runs that situation directly:
four processes x 60 jobs must all finish, correct, well inside the time limit."""
import multiprocessing as mp
import os
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(idx, jobs, start, out):
    try:
        import locust_amd as lc

        text = open(os.path.join(ROOT, "data", "hamlet.txt"), "rb").read()
        nlines = text.count(b"\n") + (0 if text.endswith(b"\n") else 1)
        eng = lc._C.GpuEngine(lc.make_config("gpu"), len(text), nlines)
        eng.load(text)
        eng.run_loaded()  # warm: graphs captured, buffers grown
        start.wait(timeout=60)  # all processes hit the GPU together
        t0 = time.perf_counter()
        worst = 0.0
        res = None
        for _ in range(jobs):
            t = time.perf_counter()
            res = eng.run_loaded()
            worst = max(worst, time.perf_counter() - t)
        out.put((idx, res.num_tokens, res.num_unique, time.perf_counter() - t0, worst))
    except Exception as e:  # report instead of hanging the test
        out.put((idx, "ERR " + repr(e), 0, 0.0, 0.0))


def test_processes_sharing_the_gpu():
    ctx = mp.get_context("spawn")
    nproc, jobs = 4, 60
    start = ctx.Barrier(nproc)
    out = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(i, jobs, start, out)) for i in range(nproc)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in range(nproc):
            results.append(out.get(timeout=90))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert not any(isinstance(r[1], str) for r in results), results
    assert sorted(r[0] for r in results) == list(range(nproc))
    for _, ntok, nuniq, total_s, worst_s in results:
        assert (ntok, nuniq) == (32940, 5608)
        # a job takes well under a millisecond alone; even 4-way sharing and first-call
        # effects stay far below the stalls (seconds) this guards against
        assert worst_s < 0.5, worst_s
        assert total_s < 10.0, total_s
