"""SCALE readiness: the driver's multi-GPU forms, run the moment a box
has the GPUs, each with a twin that runs today.

| form | real peers (skip below 2 GPUs) | twin |
|---|---|---|
| self-spawned `bench.py --gpus N` (the driver's form, no torchrun) | RCCL ranks | CPU + TCP here; tcpdev on one GPU |
| `bench.py --config synth10g --gpus N` | RCCL ranks, 10 GB | CPU + TCP, 20 MB |
| `./MapReduce <synth file> --gpus N --strategy shuffle --json` | RCCL clique | CPU ranks here; loopback ranks on one GPU |

The reference's only scaling evidence is its 1->5-node chart (/root/reference/README.md:92-96)."""
import json
import os
import subprocess
import sys

import pytest

import locust_amd as lc
from locust_amd.utils import oracle

ROOT = lc.REPO_ROOT
SYNTH1M_UNIQUE = 202645  # 1M lines, seed 1 (the CPU engine's count; tests/test_bench.py)


def _bench(*args, timeout=300):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def _line(p) -> dict:
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def _gpus() -> int:
    # counted in a child: no HIP initialisation in this process before ranks are spawned
    out = subprocess.run([sys.executable, "-c", "import locust_amd as l; print(l._C.device_count())"],
                         capture_output=True, text=True, timeout=120)
    try:
        return int(out.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def _synth10g_want(total: int, world: int):
    """The CPU engine over the concatenation of bench.synth_shard's N shards."""
    sys.path.insert(0, ROOT)
    import bench

    whole = b"".join(bench.synth_shard("synth10g", r, world, nbytes=total).to_bytes()
                     for r in range(world))
    return lc._C.cpu_run(lc.make_config("cpu"), whole)


def _gen(cli, path, lines):
    subprocess.run([cli, "--gen", str(path), "--gen-lines", str(lines), "--seed", "1"],
                   check=True, capture_output=True, timeout=300)


def _cli_ranks(cli, path, gpus, extra, timeout=300):
    j = str(path) + ".json"
    p = subprocess.run([cli, str(path), "--gpus", str(gpus), "--json", j, *extra],
                       capture_output=True, timeout=timeout)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    return p.stdout, json.load(open(j))


def _check_cli(out: bytes, rec: dict, path, gpus: int, device: bool):
    from test_cli_gpu import _parse_gpu_out

    want = lc._C.cpu_run(lc.make_config("cpu"), open(path, "rb").read())
    assert _parse_gpu_out(out) == want.entries()
    assert len(rec["ranks"]) == gpus and rec["unique"] == want.num_unique
    assert sum(r["input_bytes"] for r in rec["ranks"]) == os.path.getsize(path)
    if device:
        assert rec["strategy"] == "shuffle"
        assert all(r["device_exchange"] is True for r in rec["ranks"]), rec["ranks"]


# ---------------------------------------------------------------------------------------
# twins that run here (CPU engine, TCP / in-process loopback)
# ---------------------------------------------------------------------------------------
def test_bench_synth10g_cpu_ranks():
    total = 20_000_000
    d = _line(_bench("--config", "synth10g", "--synth-bytes", str(total), "--gpus", "2",
                     "--backend", "cpu", "--comm", "tcp", "--steps", "2", "--warmup", "1"))
    want = _synth10g_want(total, 2)
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["unique"] == want.num_unique and d["tokens"] == want.num_tokens


@pytest.mark.parametrize("gpus", [2, 3])
def test_cli_cpu_ranks_synth_file(tmp_path, cli, gpus):
    f = tmp_path / "s.txt"
    _gen(cli, f, 60_000)
    out, rec = _cli_ranks(cli, f, gpus, ["--backend", "cpu", "--strategy", "shuffle"])
    _check_cli(out, rec, f, gpus, device=False)


# ---------------------------------------------------------------------------------------
# one-GPU-box twins (ranks share the box's GPU)
# ---------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_bench_self_spawned_tcpdev_one_gpu():
    d = _line(_bench("--gpus", "2", "--comm", "tcpdev", "--steps", "5", "--warmup", "2",
                     "--synth-lines", "100000"))
    assert d["n_gpus"] == 2 and d["synth1m"]["n_gpus"] == 2
    whole = lc._C.HostText.generate(lines=100000, seed=1, first_block=0).to_bytes()
    assert d["synth1m"]["unique"] == lc._C.cpu_run(lc.make_config("cpu"), whole).num_unique


@pytest.mark.gpu
@pytest.mark.parametrize("gpus", [2, 4])
def test_cli_loopback_ranks_synth_file(tmp_path, cli, gpus):
    f = tmp_path / "s.txt"
    _gen(cli, f, 200_000)
    out, rec = _cli_ranks(cli, f, gpus, ["--comm", "loopback", "--strategy", "shuffle"])
    _check_cli(out, rec, f, gpus, device=True)


# ---------------------------------------------------------------------------------------
# real peers: RCCL, one GPU per rank (the driver's SCALE run)
# ---------------------------------------------------------------------------------------
WORLD = min(_gpus(), 8)
needs_peers = pytest.mark.skipif(WORLD < 2, reason="needs >= 2 GPUs (RCCL: one rank per GPU)")


@pytest.mark.gpu
@needs_peers
def test_bench_self_spawned_rccl_world():
    d = _line(_bench("--gpus", str(WORLD), "--steps", "5", "--warmup", "2"))
    assert d["n_gpus"] == WORLD and d["rccl_ranks"] == WORLD
    assert d["synth1m"]["n_gpus"] == WORLD and d["synth1m"]["unique"] == SYNTH1M_UNIQUE
    assert d["unique"] == len(oracle.wordcount(open(os.path.join(ROOT, "data", "hamlet.txt"), "rb").read())[0])


@pytest.mark.gpu
@needs_peers
def test_bench_synth10g_rccl_world():
    d = _line(_bench("--config", "synth10g", "--gpus", str(WORLD), "--steps", "2", "--warmup", "1",
                     timeout=900))
    assert d["n_gpus"] == WORLD and d["rccl_ranks"] == WORLD and d["value"] > 0


@pytest.mark.gpu
@needs_peers
def test_cli_rccl_clique_synth1m_file(tmp_path, cli):
    f = tmp_path / "s1m.txt"
    _gen(cli, f, 1_000_000)
    out, rec = _cli_ranks(cli, f, WORLD, ["--comm", "rccl", "--strategy", "shuffle"])
    _check_cli(out, rec, f, WORLD, device=True)
    assert rec["unique"] == SYNTH1M_UNIQUE
