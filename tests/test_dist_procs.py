"""Multi-process distributed jobs with every rank a process (the torchrun shape), on one
GPU: the "tcpdev" communicator stages the device data plane through TCP, so the device
exchange runs exactly as over RCCL -- each process maps the shared output segment and
registers it, writes its key range at its global offset, stamps its completion, and rank 0
adopts the output.  RCCL itself refuses two ranks on
one device; a real multi-GPU node runs the same path with ncclAllGather / ncclAllToAll /
grouped ncclSend/ncclRecv."""
import glob
import json
import os
import sys

import pytest

import locust_amd as lc
from locust_amd.parallel import launch

WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_worker.py")


def _run(tmp_path, world, comm, strategy, jobs, keep=False, text=None, env_extra=None):
    src = tmp_path / "text.txt"
    src.write_bytes(text if text is not None else open(os.path.join(lc.REPO_ROOT, "data", "hamlet.txt"), "rb").read())
    out = str(tmp_path / "res")
    env = {"PYTHONPATH": lc.REPO_ROOT, **(env_extra or {})}
    rc = launch.launch_local([sys.executable, WORKER, str(src), out, comm, strategy, str(jobs),
                              "1" if keep else "0"], world, timeout=300, extra_env=env)
    assert rc == 0
    recs = [json.load(open(f"{out}.{r}.json")) for r in range(world)]
    assert not glob.glob("/dev/shm/locust-*"), "shared output names left behind"
    return recs


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_device_exchange_across_processes(tmp_path, world):
    recs = _run(tmp_path, world, "tcpdev", "shuffle", 4)
    assert all(recs[0]["ok"]), recs[0]["ok"]
    for r in recs:
        assert r["comm"] == "tcpdev"
        assert [i["device_exchange"] for i in r["infos"]] == [True] * 4
        assert [i["host_syncs"] for i in r["infos"]][:2] == [2, 1]
        # compact records the merge counted as it emitted: 8-40 B per key
        assert all(8 * i["range_unique"] <= i["output_bytes"] <= 40 * i["range_unique"]
                   for i in r["infos"])


@pytest.mark.gpu
def test_gather_first_job_across_processes(tmp_path):
    """auto, first job: the sized exchange in its to-root (gather) form."""
    recs = _run(tmp_path, 2, "tcpdev", "auto", 3)
    assert all(recs[0]["ok"])
    assert recs[0]["infos"][0]["strategy"] == "gather"
    assert recs[0]["infos"][0]["device_exchange"]


@pytest.mark.gpu
def test_held_results_across_processes(tmp_path):
    """Rank 0 keeps every result: the output regions run out, every process grows the
    shared output and writes its range again; all kept results stay intact."""
    recs = _run(tmp_path, 2, "tcpdev", "shuffle", 5, keep=True)
    assert all(recs[0]["ok"]), recs[0]["ok"]
    syncs = [i["host_syncs"] for i in recs[0]["infos"]]
    assert 2 in syncs[1:], syncs


@pytest.mark.gpu
@pytest.mark.parametrize("slow", [0, 1])
def test_held_results_slow_rank_regrow(tmp_path, slow):
    """Grow-and-re-emit with one rank 300 ms late to open the new output generation
    (LOCUST_FAULT=<rank>:slow_regrow): the host barrier after the open keeps the fast ranks
    from unlinking the name first."""
    recs = _run(tmp_path, 2, "tcpdev", "shuffle", 5, keep=True,
                env_extra={"LOCUST_FAULT": f"{slow}:slow_regrow", "LOCUST_OUT_WAIT_S": "20"})
    assert all(recs[0]["ok"]), recs[0]["ok"]
