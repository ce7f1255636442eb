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


def check_scale_diag(d: dict, world: int, comm: str, gpu: bool) -> None:
    """The N > 1 line diagnoses itself: per-rank min/max of every
    stage, bytes per peer, each pair's direct access and transport, per-rank peak RSS."""
    diag = d["scale_diag"]
    for k in ("map", "exchange", "merge", "emit"):
        lo, hi = diag["stages_ms_min_max"][k]
        assert 0 <= lo <= hi, (k, lo, hi)
    ranks = diag["ranks"]
    assert [r["rank"] for r in ranks] == list(range(world))
    for r in ranks:
        assert len(r["sent_to"]) == world and len(r["recv_from"]) == world
        assert r["sent_to"][r["rank"]] == 0 and r["peak_rss_kb"] > 0
        others = {str(q) for q in range(world) if q != r["rank"]}
        if comm == "rccl":  # the pairs RCCL logged a channel for (its ring and p2p setup)
            assert r["transport"] and set(r["transport"]) <= others, r
        else:
            assert set(r["transport"]) == others, r
            assert all(v == [comm] for v in r["transport"].values())
        if gpu:
            assert len(r["peer_access"]) == world and r["device"] is not None
        else:
            assert r["peer_access"] is None
    for p in range(world):  # what p sent to q is what q received from p
        for q in range(world):
            assert ranks[p]["sent_to"][q] == ranks[q]["recv_from"][p]
    assert diag["peak_rss_kb_max"] == max(r["peak_rss_kb"] for r in ranks)
    sy = d["synth1m"]["diag"]
    assert len(sy["sent_to"]) == world and set(sy["stages_ms_min_max"]) == {"map", "exchange",
                                                                             "merge", "emit"}


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


@pytest.mark.parametrize("world", [2, 3])
def test_bench_cpu_tcp_twin_diagnoses_itself(world, tmp_path):
    d = _line(_bench("--gpus", str(world), "--backend", "cpu", "--comm", "tcp", "--steps", "3",
                     "--warmup", "1", "--synth-lines", "20000"))
    check_scale_diag(d, world, "tcp", gpu=False)
    # the report tool turns lines into the scaling table
    f = tmp_path / "scale.json"
    one = dict(d, n_gpus=1, value=d["value"] * 0.9, scale_diag=None)
    one["synth1m"] = dict(d["synth1m"], ms_per_step=d["synth1m"]["ms_per_step"] * 1.5)
    f.write_text(json.dumps({"runs": [{"tail": "noise\n" + json.dumps(one)}, {"parsed": d}]}))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scale_report.py"), str(f)],
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    rows = [ln for ln in out.stdout.splitlines() if ln.startswith("| 1 ") or ln.startswith(f"| {world} ")]
    assert len(rows) == 2, out.stdout
    strong = float(rows[1].split("|")[6])
    assert abs(strong - 1.5 / world) < 0.02, rows


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
    check_scale_diag(d, 2, "tcpdev", gpu=True)
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
    check_scale_diag(d, WORLD, "rccl", gpu=True)
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


# ---------------------------------------------------------------------------------------
# a run that hangs still ends with one line: a rank stuck in a stage
# (LOCUST_FAULT=<rank>:hang_<stage> never returns) -> the watchdog's failure line within
# the budget, with every rank's last stage, native stage and heartbeat
# ---------------------------------------------------------------------------------------
def _hung_line(p, world: int, budget: float, elapsed: float) -> dict:
    assert p.returncode != 0, (p.returncode, p.stdout[-2000:])
    assert elapsed < budget + 60, elapsed
    lines = [ln for ln in p.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]
    d = json.loads(lines[0])
    assert d["status"] == "failed" and d["value"] is None and d["n_gpus"] == world
    assert "budget" in d["reason"] or "watchdog" in d["reason"], d["reason"]
    prog = d["progress"]
    assert sorted(prog) == [str(r) for r in range(world)]
    for r in prog.values():  # every rank was alive (beating) and inside a job stage
        assert r["stage"] is not None and r["heartbeat_age_s"] is not None
    return d


@pytest.mark.parametrize("world", [2, 3])
def test_bench_watchdog_cpu_tcp_twin_hang(world):
    import time

    env = dict(os.environ, LOCUST_FAULT="1:hang_map")
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world),
                        "--backend", "cpu", "--comm", "tcp", "--steps", "3", "--warmup", "1",
                        "--no-extra", "--budget-s", "12"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=150)
    d = _hung_line(p, world, 12, time.time() - t0)
    assert d["progress"]["1"]["native_stage"] == "map"
    # the scaling table shows the failed N with its reason and the ranks' last stages
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scale_report.py"), "-"],
                         input=p.stdout, capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert f"| {world} | failed |" in out.stdout and f"N={world}: failed (" in out.stdout
    assert "r1: " in out.stdout


def test_bench_watchdog_under_torchrun_cpu_twin():
    """The driver's form for N > 1: torch.distributed.run starts the ranks; rank 0's own
    watchdog prints the failure line before the launcher tears the job down."""
    import socket
    import time

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, LOCUST_FAULT="1:hang_map")
    env.pop("LOCUST_PROGRESS_DIR", None)
    t0 = time.time()
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend",
                        "cpu", "--comm", "tcp", "--steps", "3", "--warmup", "1", "--no-extra",
                        "--budget-s", "15"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=240)
    _hung_line(p, 2, 15 + 30, time.time() - t0)


@pytest.mark.gpu
def test_bench_watchdog_tcpdev_one_gpu_hang():
    """The one-GPU twin of the device exchange path (tcpdev: TCP control, device data
    plane): rank 1 hangs in the exchange; the line still comes, inside the budget."""
    import time

    env = dict(os.environ, LOCUST_FAULT="1:hang_exchange")
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--comm",
                        "tcpdev", "--steps", "3", "--warmup", "1", "--no-extra", "--strategy",
                        "shuffle", "--budget-s", "25"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=110)
    _hung_line(p, 2, 25, time.time() - t0)
