"""Hosts files, the worker daemon and the launcher (CPU only; several daemons on one box
-- which the reference's fixed 127.0.0.1:1337 slave could not do)."""
import json
import os
import socket
import subprocess
import sys
import threading

import pytest

import locust_amd as lc
from locust_amd.parallel import daemon, launch, parse_hosts
from locust_amd.parallel.hosts import Host
from locust_amd.parallel.protocol import request
from locust_amd.utils import oracle


def test_parse_hosts():
    hs = parse_hosts("# cluster\n10.0.0.1 1337\n\n10.0.0.2 7001 gpus=4  # half node\n")
    assert hs == [Host("10.0.0.1", 1337), Host("10.0.0.2", 7001, 4)]
    for bad in ["", "10.0.0.1\n", "a b\n", "h 1 cpus=3\n", "h 1\nh 1\n", "h 70000\n"]:
        with pytest.raises(ValueError):
            parse_hosts(bad)


TOKEN = "test-token-0123"


def start_daemon(tmp_path, token=TOKEN):
    got = {}
    ev = threading.Event()

    def ready(port):
        got["port"] = port
        ev.set()

    root = str(tmp_path / f"root{len(os.listdir(tmp_path))}")
    t = threading.Thread(target=daemon.serve, kwargs=dict(port=0, root=root, token=token,
                                                         ready=ready), daemon=True)
    t.start()
    assert ev.wait(10)
    return Host("127.0.0.1", got["port"]), root


SELFTEST = [sys.executable, "-m", "locust_amd.parallel.selftest"]


def test_daemon_auth_allowlist_and_files(tmp_path):
    h, root = start_daemon(tmp_path)
    assert not request(h.addr, h.port, {"op": "hello"})["ok"]  # no token
    assert not request(h.addr, h.port, {"op": "hello", "token": "wrong"})["ok"]
    tok = {"token": TOKEN}
    assert request(h.addr, h.port, {"op": "hello", **tok})["ok"]
    rep = request(h.addr, h.port, {"op": "run", **tok, "argv": SELFTEST + ["--fail-rank", "3",
                                   "--code", "5"], "env": {"RANK": "3", "WORLD_SIZE": "4"}})
    assert rep["rc"] == 5 and not rep["ok"]
    assert json.loads(rep["stdout"])["WORLD_SIZE"] == "4"
    # only the framework's own programs, no interpreter flags, no loader hooks
    for argv in (["/bin/rm", "-rf", "x"], [sys.executable, "-c", "print(1)"],
                 [sys.executable, "-m", "locust_amd.parallel.launch", "--", "/bin/true"],
                 [sys.executable, "/tmp/evil.py"]):
        rep = request(h.addr, h.port, {"op": "run", **tok, "argv": argv})
        assert not rep["ok"] and "framework" in rep["error"], argv
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build",
                       "MapReduce")
    rep = request(h.addr, h.port, {"op": "run", **tok, "argv": [cli, "--gen", "/tmp/x.txt",
                                                                "--gen-lines", "1"]})
    assert not rep["ok"] and "--gen" in rep["error"]
    rep = request(h.addr, h.port, {"op": "run", **tok, "argv": SELFTEST,
                                   "env": {"LD_PRELOAD": "/tmp/x.so"}})
    assert not rep["ok"] and "env" in rep["error"]
    assert request(h.addr, h.port, {"op": "put", **tok, "path": "a/b.bin", "data": "aGVsbG8="})["ok"]
    rep = request(h.addr, h.port, {"op": "get", **tok, "path": "a/b.bin"})
    assert rep["ok"] and rep["data"] == "aGVsbG8=" and rep["eof"]
    assert not request(h.addr, h.port, {"op": "get", **tok, "path": "../../etc/passwd"})["ok"]


def test_daemon_refuses_unauthenticated_text_protocol(tmp_path):
    h, _ = start_daemon(tmp_path)
    with socket.create_connection((h.addr, h.port)) as s:
        s.sendall(b"x ./MapReduce hamlet.txt 0 700 1 1\n")
        assert s.recv(64).startswith(b"NAK")


def test_daemon_creates_private_token(tmp_path):
    tok = daemon.load_or_create_token(str(tmp_path / "r"))
    path = tmp_path / "r" / "token"
    assert path.read_text().strip() == tok and len(tok) >= 32
    assert (path.stat().st_mode & 0o077) == 0
    assert daemon.load_or_create_token(str(tmp_path / "r")) == tok


def test_daemon_refuses_planted_token_and_open_root(tmp_path):
    """a token file someone else could have written (group/world readable, a
    symlink) or a root others can enter is refused instead of trusted."""
    root = tmp_path / "r"
    root.mkdir(mode=0o700)
    tok = root / "token"
    tok.write_text("known-secret\n")
    os.chmod(tok, 0o644)
    with pytest.raises(PermissionError, match="token file"):
        daemon.load_or_create_token(str(root))
    tok.unlink()
    (tmp_path / "elsewhere").write_text("known-secret\n")
    os.chmod(tmp_path / "elsewhere", 0o600)
    os.symlink(tmp_path / "elsewhere", tok)
    with pytest.raises(PermissionError, match="symlink"):
        daemon.load_or_create_token(str(root))
    open_root = tmp_path / "open"
    open_root.mkdir()
    os.chmod(open_root, 0o755)
    with pytest.raises(PermissionError, match="daemon root"):
        daemon.load_or_create_token(str(open_root))
    assert daemon.default_root().endswith("locust") and not daemon.default_root().startswith("/tmp/locust")


def test_launch_local_env_and_failure_propagation(tmp_path):
    out = tmp_path / "ranks"
    out.mkdir()
    code = ("import os; open(os.path.join(%r, os.environ['RANK']), 'w').write("
            "os.environ['WORLD_SIZE'] + ' ' + os.environ['MASTER_PORT'])" % str(out))
    assert launch.launch_local([sys.executable, "-c", code], 3) == 0
    vals = {p.name: p.read_text() for p in out.iterdir()}
    assert sorted(vals) == ["0", "1", "2"] and len(set(vals.values())) == 1
    # rank 1 fails fast, rank 0 would sleep: the launcher stops it and returns rank 1's code
    code = "import os,sys,time; r=int(os.environ['RANK']); time.sleep(30 if r==0 else 0); sys.exit(7 if r==1 else 0)"
    assert launch.launch_local([sys.executable, "-c", code], 2, timeout=60) == 7


def test_launch_remote_ranks(tmp_path):
    h1, _ = start_daemon(tmp_path)
    h2, _ = start_daemon(tmp_path)
    replies = []
    assert launch.launch_remote(SELFTEST, [h1, h2], 2, token=TOKEN, replies=replies) == 0
    got = [json.loads(r["stdout"]) for r in replies]
    assert [(g["RANK"], g["LOCAL_RANK"], g["WORLD_SIZE"]) for g in got] == \
        [("0", "0", "4"), ("1", "1", "4"), ("2", "0", "4"), ("3", "1", "4")]
    assert launch.launch_remote(SELFTEST + ["--fail-rank", "2", "--code", "9"], [h1, h2], 2,
                                token=TOKEN) == 9
    assert launch.launch_remote(SELFTEST, [h1], 1, token="wrong") != 0


@pytest.mark.parametrize("reducers", [1, 2, 3])
def test_stage_split_wordcount_over_daemons(tmp_path, hamlet, cli, capfd, reducers):
    """3 local daemons map line ranges; R key-range reducers on the daemons each merge their
    slice of every spill; the concatenation is the single-stage output byte for byte,
    val included (GPU-format lines)."""
    hosts = [start_daemon(tmp_path)[0] for _ in range(3)]
    f = tmp_path / "h.txt"
    f.write_bytes(hamlet)
    rc = launch.stage_split_wordcount(str(f), hosts, cli, token=TOKEN, backend="cpu",
                                      workdir=str(tmp_path / "spills"), reducers=reducers,
                                      extra=["--output-format", "gpu"])
    assert rc == 0
    out = capfd.readouterr().out
    single = subprocess.run([cli, str(f), "--backend", "cpu", "--output-format", "gpu"],
                            capture_output=True, timeout=120).stdout.decode()
    body = out[out.index("print key:"):out.rindex("\nDone")]
    want = single[single.index("print key:"):single.rindex("\nDone")]
    assert body == want, body[:300]  # (no full diff: the output is 5,608 lines)
    assert out.startswith("Running\n") and out.endswith("\nDone\n")


def test_daemon_confines_result_files(tmp_path, cli):
    h, _root = start_daemon(tmp_path)
    rep = request(h.addr, h.port, {"op": "run", "token": TOKEN, "argv": [
        cli, "x", "0", "0", "0", "2", "--result-file", "/tmp/elsewhere.txt"]})
    assert not rep["ok"] and "--result-file" in rep["error"]


def test_bootstrap_port_from_torchrun_store(tmp_path):
    """Under torch.distributed.run rank 0 binds a free port, keeps the socket listening and
    hands it to the native communicator; the others read the port from the file it
    publishes -- no window in which another process could take the port, no torch import.
    The ranks then meet for real (TCP communicator, CPU engine)."""
    script = tmp_path / "port.py"
    script.write_text(
        "import os, sys\n"
        "import locust_amd as lc\n"
        "from locust_amd.parallel import bootstrap_listener, connect_rank\n"
        "w = int(os.environ['WORLD_SIZE'])\n"
        "dr = connect_rank(lc.make_dist_config(w, lc.make_config('cpu')), int(os.environ['RANK']),"
        " w, 'tcp', 1, 1, 60.0)\n"
        "dr.barrier()\n"
        "from locust_amd import parallel\n"
        "row = ' '.join(map(str, ['PORT', os.environ['RANK'], dr.size, 'torch' in sys.modules,"
        " parallel._port_file is None]))\n"
        "open(sys.argv[1] + '.' + os.environ['RANK'], 'w').write(row)\n")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    master = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k not in ("LOCUST_PORT", "LOCUST_LISTEN_FD")}
    env["PYTHONPATH"] = lc.REPO_ROOT + os.pathsep + env.get("PYTHONPATH", "")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=3", "--master-addr", "127.0.0.1", "--master-port",
                        str(master), str(script), str(tmp_path / "row")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    rows = [(tmp_path / f"row.{r}").read_text().split() for r in range(3)]
    assert sorted(r[1] for r in rows) == ["0", "1", "2"], p.stdout
    assert all(r[2] == "3" and r[3] == "False" and r[4] == "True" for r in rows), p.stdout


def test_bootstrap_stale_port_file_of_previous_attempt(monkeypatch, tmp_path):
    """A restarted torchrun attempt (same run id, MASTER_PORT and agent) never reads the
    port file a failed earlier attempt left behind: the restart count names the file."""
    from locust_amd import parallel

    monkeypatch.setenv("XDG_RUNTIME_DIR", str(tmp_path))
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "job-7")
    monkeypatch.setenv("MASTER_PORT", "31000")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    monkeypatch.delenv("LOCUST_PORT", raising=False)
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    stale = parallel._port_file_path(31000)
    with open(stale, "w") as f:
        f.write("1")  # attempt 0 died after publishing a port nobody listens on any more
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    assert parallel._port_file_path(31000) != stale
    port, fd = parallel.bootstrap_listener(0, 2)
    try:
        assert fd >= 0 and port != 1
        assert parallel.bootstrap_listener(1, 2, timeout=5) == (port, -1)
        # the listener is really bound and listening on that port
        c = socket.create_connection(("127.0.0.1", port), timeout=5)
        c.close()
    finally:
        os.close(fd)
        parallel.release_bootstrap_port()
    assert not os.path.exists(parallel._port_file_path(31000))


def test_bootstrap_port_fixed_rules(monkeypatch):
    from locust_amd.parallel import bootstrap_listener, bootstrap_port

    monkeypatch.delenv("TORCHELASTIC_RUN_ID", raising=False)
    monkeypatch.setenv("MASTER_PORT", "31000")
    monkeypatch.delenv("LOCUST_PORT", raising=False)
    assert bootstrap_port(0, 4) == 31001
    monkeypatch.setenv("LOCUST_PORT", "32000")
    assert bootstrap_port(1, 4) == 32000
    # an inherited listener goes to rank 0 only, and only once
    monkeypatch.setenv("LOCUST_LISTEN_FD", "7")
    assert bootstrap_listener(1, 4) == (32000, -1)
    monkeypatch.setenv("LOCUST_LISTEN_FD", "7")
    assert bootstrap_listener(0, 4) == (32000, 7)
    assert "LOCUST_LISTEN_FD" not in os.environ


def test_launch_local_hands_listener_to_rank0(tmp_path):
    """launch_local binds the bootstrap socket itself and rank 0 inherits it."""
    script = tmp_path / "meet.py"
    script.write_text(
        "import os\n"
        "import locust_amd as lc\n"
        "from locust_amd.parallel import connect_rank\n"
        "w = int(os.environ['WORLD_SIZE'])\n"
        "dr = connect_rank(lc.make_dist_config(w, lc.make_config('cpu')), int(os.environ['RANK']),"
        " w, 'tcp', 1, 1, 60.0)\n"
        "dr.barrier()\n")
    env = {"PYTHONPATH": lc.REPO_ROOT}
    assert launch.launch_local([sys.executable, str(script)], 3, timeout=120, extra_env=env) == 0


def test_stage_split_resumes_from_map_outputs(tmp_path, hamlet, cli, capfd):
    """The spills are the job's checkpoint: a rerun with resume maps only
    the hosts whose stage-1 output is missing, and gives the same output."""
    hosts_roots = [start_daemon(tmp_path) for _ in range(3)]
    hosts = [h for h, _r in hosts_roots]
    f = tmp_path / "h.txt"
    f.write_bytes(hamlet)
    kw = dict(token=TOKEN, backend="cpu", reducers=2, extra=["--output-format", "gpu"])
    mapped = []
    assert launch.stage_split_wordcount(str(f), hosts, cli, workdir=str(tmp_path / "w1"),
                                        mapped=mapped, **kw) == 0
    first = capfd.readouterr().out
    assert mapped == [0, 1, 2]
    os.remove(os.path.join(hosts_roots[1][1], "out.1.kv.idx"))  # host 1 lost its map output
    mapped = []
    assert launch.stage_split_wordcount(str(f), hosts, cli, workdir=str(tmp_path / "w2"),
                                        mapped=mapped, resume=True, **kw) == 0
    assert mapped == [1]
    assert capfd.readouterr().out == first


def test_stage_split_map_failure_propagates(tmp_path, cli, capfd):
    """A failing map stage stops the job with its exit code (the reference's slave ACKed
    whatever happened, slave.py:19-20); no reducer runs."""
    hosts = [start_daemon(tmp_path)[0] for _ in range(2)]
    f = tmp_path / "t.txt"
    f.write_bytes(b"a b\nc\n")
    rc = launch.stage_split_wordcount(str(f), hosts, cli, token=TOKEN, backend="cpu",
                                      workdir=str(tmp_path / "w"), extra=["--emits-per-line", "0"])
    assert rc == 2  # the CLI's error exit
    cap = capfd.readouterr()
    assert "map stage failed" in cap.err and "print key" not in cap.out


def _range_bytes(spills, lo, hi):
    from locust_amd.parallel.spillindex import range_record_bytes, read_binary_spill

    return [range_record_bytes(read_binary_spill(open(p, "rb").read()), lo, hi) for p in spills]


@pytest.mark.parametrize("reducers", [2, 3, 5])
def test_reducers_pull_only_their_range_peer_to_peer(tmp_path, cli, capfd, reducers):
    """no launcher hub.  The launcher fetches only the spills' indexes
    and the result lines; each reducer pulls its key range of every other host's spill
    straight from that host's daemon -- at most 1.2x the bytes of the records in its range
    (plus headers); the output is the single-stage output."""
    from locust_amd.parallel.spillindex import reducer_range

    hosts_roots = [start_daemon(tmp_path) for _ in range(3)]
    hosts = [h for h, _ in hosts_roots]
    f = tmp_path / "g.txt"
    subprocess.run([cli, "--gen", str(f), "--gen-lines", "60000", "--seed", "3"], check=True,
                   capture_output=True, timeout=120)
    traffic = {}
    rc = launch.stage_split_wordcount(str(f), hosts, cli, token=TOKEN, backend="cpu",
                                      workdir=str(tmp_path / "w"), reducers=reducers,
                                      extra=["--output-format", "gpu"], traffic=traffic)
    assert rc == 0
    out = capfd.readouterr().out
    single = subprocess.run([cli, str(f), "--backend", "cpu", "--output-format", "gpu"],
                            capture_output=True, timeout=120).stdout.decode()
    assert out[out.index("print key:"):out.rindex("\nDone")] == \
        single[single.index("print key:"):single.rindex("\nDone")]
    spills = [os.path.join(root, f"out.{k}.kv") for k, (_h, root) in enumerate(hosts_roots)]
    spill_total = sum(os.path.getsize(p) for p in spills)
    idx_total = sum(os.path.getsize(p + ".idx") for p in spills)
    results = len(out.encode())
    # the launcher held the indexes and the results, never a spill
    assert traffic["launcher_fetched"] <= idx_total + results
    assert traffic["launcher_fetched"] < spill_total
    spl = traffic["splitters"]
    for r in range(reducers):
        lo, hi = reducer_range(spl, r)
        want = _range_bytes(spills, lo, hi)
        for k in range(3):
            if k == r % 3:
                assert traffic["pulled"][r][k] == 0  # its own spill: read in place
                continue
            assert traffic["pulled"][r][k] <= 1.2 * want[k] + 32 + 2 * 40 * 16, (r, k)
        remote = sum(want[k] for k in range(3) if k != r % 3)
        assert sum(traffic["pulled"][r]) <= 1.2 * remote + 3 * (32 + 40 * 32), r


def test_python_splitters_match_native(tmp_path, cli):
    from locust_amd.parallel.spillindex import BEYOND, parse_index, plan_splitters

    f = tmp_path / "g.txt"
    subprocess.run([cli, "--gen", str(f), "--gen-lines", "20000", "--seed", "9"], check=True,
                   capture_output=True, timeout=120)
    n = os.path.getsize(f)
    spills = []
    for k in range(4):
        subprocess.run([cli, str(f), "0", "0", str(k), "1", "--byte-range",
                        f"{n * k // 4}:{n * (k + 1) // 4}", "--spill-dir", str(tmp_path),
                        "--spill-format", "binary", "--backend", "cpu"], check=True,
                       capture_output=True, timeout=120)
        spills.append(str(tmp_path / f"out.{k}.kv"))
    idx = [parse_index(open(p + ".idx", "rb").read()) for p in spills]
    for R in (1, 2, 3, 7, 64, 5000):
        py = plan_splitters(idx, R)
        nat = lc._C.reducer_splitters(spills, R)
        import struct

        def words(b):
            b = b.ljust(32, b"\0")
            return tuple(struct.unpack(">4Q", b))
        assert [words(b) for b in nat] == py, R
        assert R < 5000 or py[-1] == BEYOND  # more reducers than keys: empty tail ranges


def test_stage_split_resume_checks_input_and_command(tmp_path, hamlet, cli, capfd):
    """a resume reuses a map output only for the same command on the unchanged
    input -- an input edited in place, or other tokenizer flags, map again."""
    hosts = [start_daemon(tmp_path)[0] for _ in range(2)]
    f = tmp_path / "h.txt"
    f.write_bytes(hamlet)
    kw = dict(token=TOKEN, backend="cpu", reducers=2)
    mapped = []
    assert launch.stage_split_wordcount(str(f), hosts, cli, mapped=mapped,
                                        extra=["--output-format", "gpu"], **kw) == 0
    assert mapped == [0, 1]
    mapped = []
    assert launch.stage_split_wordcount(str(f), hosts, cli, mapped=mapped, resume=True,
                                        extra=["--output-format", "gpu"], **kw) == 0
    assert mapped == []  # unchanged: nothing mapped again
    capfd.readouterr()
    mapped = []
    assert launch.stage_split_wordcount(str(f), hosts, cli, mapped=mapped, resume=True,
                                        extra=["--output-format", "gpu", "--emits-per-line", "5"],
                                        **kw) == 0
    assert mapped == [0, 1]  # other tokenizer flags
    out5 = capfd.readouterr().out
    ent, _n, _ = oracle.wordcount(hamlet, emits=5)
    assert out5[out5.index("print key:"):out5.rindex("\nDone")].encode().rstrip(b"\n") == \
        oracle.format_gpu(ent).rstrip(b"\n")
    f.write_bytes(hamlet.replace(b"Hamlet", b"Omelet"))  # same size, edited in place
    mapped = []
    assert launch.stage_split_wordcount(str(f), hosts, cli, mapped=mapped, resume=True,
                                        extra=["--output-format", "gpu", "--emits-per-line", "5"],
                                        **kw) == 0
    assert mapped == [0, 1]
    out = capfd.readouterr().out
    assert "Omelet" in out and "print key: Hamlet " not in out


def test_stage_split_resume_remaps_a_truncated_spill(tmp_path, hamlet, cli, capfd):
    """a spill shorter than its index's spill_bytes (a map killed while writing,
    a disk that filled) is mapped again on resume, the intact one is reused."""
    hosts_roots = [start_daemon(tmp_path) for _ in range(2)]
    hosts = [h for h, _ in hosts_roots]
    f = tmp_path / "h.txt"
    f.write_bytes(hamlet)
    kw = dict(token=TOKEN, backend="cpu", reducers=2, extra=["--output-format", "gpu"])
    assert launch.stage_split_wordcount(str(f), hosts, cli, **kw) == 0
    first = capfd.readouterr().out
    spill = os.path.join(hosts_roots[0][1], "out.0.kv")
    with open(spill, "r+b") as fh:
        fh.truncate(os.path.getsize(spill) - 40)
    mapped = []
    assert launch.stage_split_wordcount(str(f), hosts, cli, mapped=mapped, resume=True, **kw) == 0
    assert mapped == [0]
    out = capfd.readouterr().out
    assert out[out.index("print key:"):] == first[first.index("print key:"):]


def test_daemon_pull_validates_and_confines(tmp_path):
    """The `pull` op: byte ranges of a peer daemon's file written at their offsets under
    this daemon's root (the rest a hole); bad ranges and paths outside the root refused."""
    (a, _ra), (b, rb) = start_daemon(tmp_path), start_daemon(tmp_path)
    tok = {"token": TOKEN}
    assert request(a.addr, a.port, {"op": "put", **tok, "path": "src.bin",
                                    "data": "MDEyMzQ1Njc4OQ=="})["ok"]  # b"0123456789"
    peer = [a.addr, a.port]
    rep = request(b.addr, b.port, {"op": "pull", **tok, "peer": peer, "src": "src.bin",
                                   "dest": "got.bin", "ranges": [[2, 3], [7, 2]], "size": 10})
    assert rep["ok"] and rep["bytes"] == 5
    assert open(os.path.join(rb, "got.bin"), "rb").read() == b"\x00\x00234\x00\x0078\x00"
    for bad in ({"ranges": [[-1, 4]]}, {"ranges": [[0, 4]], "size": -5}, {"ranges": [["x", 1]]},
                {"ranges": [[0, 4]], "dest": "../escape.bin"}, {"peer": "nowhere"}):
        req = {"op": "pull", **tok, "peer": peer, "src": "src.bin", "dest": "bad.bin", **bad}
        assert not request(b.addr, b.port, req)["ok"], bad
    assert not os.path.exists(os.path.join(os.path.dirname(rb), "escape.bin"))


def test_launcher_cli_wordcount_resume(tmp_path, hamlet, cli, capfd, monkeypatch):
    """`python -m locust_amd.parallel.launch --hosts H --wordcount F [--resume]`: the second
    run with --resume maps nothing again and prints the same output."""
    hosts_roots = [start_daemon(tmp_path) for _ in range(2)]
    hf = tmp_path / "hosts.txt"
    hf.write_text("".join(f"{h.addr} {h.port}\n" for h, _ in hosts_roots))
    tf = tmp_path / "token"
    tf.write_text(TOKEN + "\n")
    f = tmp_path / "h.txt"
    f.write_bytes(hamlet)
    base = ["--hosts", str(hf), "--token-file", str(tf), "--wordcount", str(f), "--backend",
            "cpu", "--cli", cli, "--output-format", "gpu"]
    assert launch.main(base) == 0
    first = capfd.readouterr().out
    ran = []
    real = launch._RemoteRun

    def spy(h, argv, env, token):
        ran.append(argv[5])  # the stage
        return real(h, argv, env, token)

    monkeypatch.setattr(launch, "_RemoteRun", spy)
    assert launch.main(base + ["--resume"]) == 0
    assert ran == ["2", "2"]  # reducers only: both map outputs reused
    assert capfd.readouterr().out == first
    ent, _n, _ = oracle.wordcount(hamlet)
    assert first[first.index("print key:"):first.rindex("\nDone")].encode().rstrip(b"\n") == \
        oracle.format_gpu(ent).rstrip(b"\n")
