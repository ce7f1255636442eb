"""bench.py's rank plumbing without a GPU: `--gpus N` with no
launcher spawns N child rank processes itself and relays rank 0's one JSON line; a run
that cannot give every rank a GPU of its own fails instead of reporting n_gpus=1.  The CPU
engine + TCP communicator stand in for the GPU + RCCL here; the GPU twin of these tests is
tests/test_bench.py."""
import json
import os
import subprocess
import sys

import pytest

import locust_amd as lc
from locust_amd.utils import oracle

ROOT = lc.REPO_ROOT


def _bench(*args, timeout=240):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("world", [2, 3])
def test_self_spawned_ranks_relay_one_line(hamlet, world):
    p = _bench("--gpus", str(world), "--backend", "cpu", "--comm", "tcp", "--steps", "3",
               "--warmup", "1", "--synth-lines", "12000")
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["config"]["parallelism"].startswith(f"dp{world}+tcp_")
    # weak-scaling headline: every rank maps its own copy, merged on rank 0
    ent, ntok, _ = oracle.wordcount(hamlet)
    assert d["unique"] == len(ent) and d["tokens"] == world * ntok
    # strong-scaling synthetic extra: 1/N of the text per rank, one answer
    s = d["synth1m"]
    assert s["n_gpus"] == world and s["lines"] == 12000
    whole = lc._C.HostText.generate(lines=12000, seed=1, first_block=0).to_bytes()
    want = lc._C.cpu_run(lc.make_config("cpu"), whole)
    assert s["unique"] == want.num_unique and s["tokens"] == want.num_tokens
    assert s["bytes"] == len(whole)


def test_gpus_without_enough_gpus_fails_loudly():
    if lc._C.device_count() >= 2:
        pytest.skip("this box has the GPUs")
    p = _bench("--gpus", "2", "--steps", "2", "--warmup", "1", "--no-extra", timeout=120)
    assert p.returncode != 0
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and json.loads(lines[0])["value"] is None  # a failure line only
    assert "needs GPU" in p.stderr


def test_gpus_must_match_world_size():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4",
                        "--backend", "cpu", "--comm", "tcp", "--no-extra"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 2 and "WORLD_SIZE=1" in p.stderr


def test_failed_rank_fails_the_run():
    # LOCUST_FAULT makes rank 1's map throw: the parent exits non-zero and prints ONE
    # failure line -- no value, the failing rank, every rank's last stage
    env = dict(os.environ, LOCUST_FAULT="1:map")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--backend", "cpu", "--comm", "tcp", "--steps", "2", "--warmup", "1",
                        "--no-extra"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode != 0, (p.returncode, p.stdout)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["status"] == "failed" and d["value"] is None and "rank" in d["reason"]
    assert sorted(d["progress"]) == ["0", "1"]
