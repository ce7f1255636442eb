"""Multi-GPU RCCL with real peers: world = min(visible GPUs, 8).

* one process per GPU (`locust_amd.parallel.rccl_check`, launched here before any GPU
  call in this process): gather (slot all-gather, captured into a hipGraph from the second
  job of a shape on), shuffle (grouped ncclSend/ncclRecv all-to-all-v) and auto, every
  job byte-identical to the oracle on rank 0 including the global `val`;
* one process, an RCCL clique (ncclCommInitAll), the same strategies;
* bench.py under torch.distributed.run at N = world.

On a box with one GPU these skip (RCCL refuses two ranks per device; the loopback and
one-rank RCCL tests in test_dist.py cover that box)."""
import json
import os
import socket
import subprocess
import sys

import pytest

import locust_amd as lc
from locust_amd.utils import oracle

pytestmark = pytest.mark.gpu


def _gpus() -> int:
    # counted in a child: this test process must not have initialised HIP when it spawns
    # the rank processes
    out = subprocess.run([sys.executable, "-c", "import locust_amd as l; print(l._C.device_count())"],
                         capture_output=True, text=True, timeout=120)
    try:
        return int(out.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


WORLD = min(_gpus(), 8)
needs_peers = pytest.mark.skipif(WORLD < 2, reason="needs >= 2 GPUs (RCCL: one rank per GPU)")


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@needs_peers
@pytest.mark.parametrize("world", sorted({2, WORLD}))
def test_rccl_multiprocess_strategies(world):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", LOCUST_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-m", "locust_amd.parallel.rccl_check",
                                       "--jobs", "3"], env=env, cwd=lc.REPO_ROOT,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, o.decode(), e.decode()[-2000:]))
    assert all(rc == 0 for rc, _, _ in outs), outs
    rep = json.loads(outs[0][1].strip().splitlines()[-1])
    assert rep["ok"] and all(j["match"] for j in rep["jobs"])
    assert {j["took"] for j in rep["jobs"]} == {"gather", "shuffle"}


@needs_peers
@pytest.mark.parametrize("strategy", ["gather", "shuffle", "auto"])
def test_rccl_clique_single_process(hamlet, strategy):
    cfgs = [lc.make_dist_config(WORLD, lc.make_config("gpu", combine=True, check=True),
                                strategy=strategy) for _ in range(3)]
    ent, ntok, _ = oracle.wordcount(hamlet)
    for res, info in lc._C.run_multi_schedule(hamlet, cfgs, "rccl"):
        assert res.entries() == ent and res.num_tokens == ntok


@needs_peers
def test_bench_torchrun_world():
    port = _port()
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        f"--nproc-per-node={WORLD}", "--master-addr", "127.0.0.1",
                        "--master-port", str(port), "bench.py", "--gpus", str(WORLD),
                        "--steps", "20", "--warmup", "5"],
                       cwd=lc.REPO_ROOT, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == WORLD and line["value"] > 0 and line["unique"] == 5608
