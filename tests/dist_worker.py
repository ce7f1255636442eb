"""One rank of a multi-process distributed job (launched by tests/test_dist_procs.py through
locust_amd.parallel.launch_local): maps its line-aligned shard of a text, runs JOBS jobs
back to back on one DistRank, and writes every job's info -- plus, on rank 0, whether each
result matched the oracle -- to OUT.<rank>.json.

    python tests/dist_worker.py TEXT_FILE OUT COMM STRATEGY JOBS [KEEP]

KEEP=1: rank 0 keeps every result alive until the end (the shared output's regions)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import locust_amd as lc  # noqa: E402
from locust_amd.parallel import connect_rank  # noqa: E402
from locust_amd.utils import oracle  # noqa: E402


def main():
    path, out, comm, strategy, jobs = sys.argv[1:6]
    keep = len(sys.argv) > 6 and sys.argv[6] == "1"
    jobs = int(jobs)
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    text = open(path, "rb").read()
    lines = text.split(b"\n")
    per = (len(lines) + world - 1) // world
    mine = lines[rank * per:(rank + 1) * per]
    shard = b"\n".join(mine) + (b"\n" if (rank + 1) * per < len(lines) else b"")
    backend = "cpu" if comm == "tcp" and os.environ.get("LOCUST_TEST_BACKEND") == "cpu" else "gpu"
    job = lc.make_config(backend, combine=True, check=backend == "gpu")
    dcfg = lc.make_dist_config(world, job, strategy=strategy)
    dr = connect_rank(dcfg, rank, world, comm, max(len(shard), 1), max(len(mine), 1), 120.0)
    want = oracle.wordcount(text)[0] if rank == 0 else None
    infos, ok, held = [], [], []
    for _ in range(jobs):
        res, info = dr.run(shard, rank * per)
        infos.append(info)
        if rank == 0:
            ok.append(res.entries() == want)
            if keep:
                held.append(res)
    if rank == 0 and keep:  # every kept result still intact at the end
        ok.append(all(r.entries() == want for r in held))
    with open(f"{out}.{rank}.json", "w") as f:
        json.dump({"infos": infos, "ok": ok, "comm": dr.comm_name}, f)


if __name__ == "__main__":
    main()
