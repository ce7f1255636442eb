"""One rank of a multi-process RCCL WordCount check (real peers, one GPU per rank).

    python -m locust_amd.parallel.launch --nproc N -- \\
        python -m locust_amd.parallel.rccl_check [--jobs J] [--text FILE]

Every rank maps its own byte-range shard of the text (strong scaling) and runs J jobs per
strategy -- gather (the slot job: map + ncclAllGather + root merge, captured into one
hipGraph from the second job of a shape on), shuffle (sample-sort splitters + grouped
ncclSend/ncclRecv all-to-all-v + rank-order gather) and auto -- on the SAME communicator
and engine, like a long-lived job.  Rank 0 checks every job byte-for-byte against the
independent oracle, including the global `val` indices, and prints
one JSON line; the exit code is non-zero on any mismatch or error.  Used by
tests/test_multi_gpu.py when the box has more than one GPU (the reference being replaced:
/root/reference/Distributor/slave.py:14-32, README.md:92-96).
"""
from __future__ import annotations

import argparse
import json
import os
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=4)
    ap.add_argument("--text", default=None, help="input file (default: data/hamlet.txt)")
    ap.add_argument("--timeout", type=float, default=120.0)
    a = ap.parse_args(argv)
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))

    import locust_amd as lc
    from locust_amd.utils import oracle

    path = a.text or os.path.join(lc.REPO_ROOT, "data", "hamlet.txt")
    with open(path, "rb") as f:
        text = f.read()
    off, nbytes, _nl, first = lc._C.shard_bounds(text, world)[rank]
    shard = text[off:off + nbytes]
    want, ntok, _ = oracle.wordcount(text) if rank == 0 else (None, None, None)
    job = lc.make_config("gpu", device=local, combine=True, check=True)
    report = {"rank": rank, "world": world, "jobs": []}
    ok = True
    sys.stdout.flush()
    saved = os.dup(1)  # RCCL's banner goes to stdout: keep stdout for the JSON line
    os.dup2(2, 1)
    try:
        from locust_amd.parallel import connect_rank

        dr = connect_rank(lc.make_dist_config(world, job), rank, world, "rccl", max(nbytes, 1),
                          max(shard.count(b"\n") + 1, 1), a.timeout)
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    for strategy in ("gather", "shuffle", "auto", "gather"):
        dr.set_strategy(getattr(lc._C.DistStrategy, strategy))
        for j in range(a.jobs):
            res, info = dr.run(shard, first)
            rec = {"strategy": strategy, "took": info["strategy"], "job": j}
            if rank == 0:
                good = res.entries() == want and res.num_tokens == ntok
                rec["match"] = good
                ok &= good
            report["jobs"].append(rec)
    dr.barrier()
    report["ok"] = ok
    print(json.dumps(report), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
