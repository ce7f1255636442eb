"""Job launcher: the master the reference documents but never shipped.

The reference's README describes a master that reads a hosts file, sends each worker a
``MapReduce file start end node 1`` command over TCP, moves the intermediate files and
starts the reducers (/root/reference/README.md:18-29).  Three
modes here:

1. Local ranks (single node, one process per GPU -- what ``bench.py`` uses via
   ``torch.distributed.run``; this launcher needs no torch)::

       python -m locust_amd.parallel.launch --nproc 8 -- python bench.py --gpus 8

   Sets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT; the ranks meet over
   the framework's TCP bootstrap and RCCL.  The first failing rank stops the job: the
   others' process groups are terminated and its exit code is the launcher's.

2. Ranks on worker daemons (multi-node)::

       python -m locust_amd.parallel.launch --hosts hosts.txt --nproc-per-host 8 -- CMD...

   Each daemon starts its host's ranks with the same environment; a failed rank makes
   the launcher drop every other connection, and the daemons kill those ranks.

3. The reference's stage-split WordCount over daemons (map -> spill files -> reduce)::

       python -m locust_amd.parallel.launch --hosts hosts.txt --wordcount data/hamlet.txt \\
           [--reducers R]

   Byte ranges (cut at line starts by the CLI) go to the hosts as stage-1 commands
   (combined, indexed binary spills); R key-range reducers (``--reducer r/R``, default
   one per host) pull their key range of every spill straight from the mapper daemons,
   merge it -- summing counts, never expanding them -- and write it with its global val;
   the launcher, which only ever holds the spills' indexes, prints the slices in order.
"""
from __future__ import annotations

import argparse
import base64
import os
import signal
import socket
import subprocess
import sys
import threading
import time

from .hosts import Host, load_hosts
from .protocol import ProtocolError, recv_msg, request, send_msg


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(rank: int, local_rank: int, world: int, master_addr: str, master_port: int) -> dict:
    return {
        "RANK": str(rank),
        "LOCAL_RANK": str(local_rank),
        "WORLD_SIZE": str(world),
        "LOCAL_WORLD_SIZE": "",  # filled per host by the caller
        "MASTER_ADDR": master_addr,
        "MASTER_PORT": str(master_port),
    }


# --------------------------------------------------------------------------------------
# mode 1: local ranks
# --------------------------------------------------------------------------------------
def bound_listener(addr: str, backlog: int) -> socket.socket:
    """A listening socket on a free port of `addr`, for the framework's bootstrap: handed
    to rank 0 (``LOCUST_LISTEN_FD``) so the port is never free between its choice and use."""
    s = socket.socket()
    s.bind((addr, 0))
    s.listen(backlog)
    return s


def spawn_local_ranks(cmd: list[str], nproc: int, master_addr: str = "127.0.0.1",
                      master_port: int | None = None, extra_env: dict | None = None,
                      stdout_of_rank0=None) -> list[subprocess.Popen]:
    """Start `nproc` local rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set;
    the bootstrap socket bound here and inherited by rank 0).  Child processes, never an
    exec: the caller may already have initialised the GPU."""
    port = master_port or _free_port()
    boot = bound_listener(master_addr, nproc)
    procs: list[subprocess.Popen] = []
    try:
        for r in range(nproc):
            env = dict(os.environ)
            env.update(rank_env(r, r, nproc, master_addr, port))
            env["LOCAL_WORLD_SIZE"] = str(nproc)
            env["LOCUST_PORT"] = str(boot.getsockname()[1])
            env.pop("LOCUST_LISTEN_FD", None)
            fds: tuple = ()
            if r == 0:
                env["LOCUST_LISTEN_FD"] = str(boot.fileno())
                fds = (boot.fileno(),)
            env.update(extra_env or {})
            procs.append(subprocess.Popen(cmd, env=env, start_new_session=True, pass_fds=fds,
                                          stdout=stdout_of_rank0 if r == 0 else None))
    except BaseException:
        for p in procs:
            _kill_group(p)
        raise
    finally:
        boot.close()  # rank 0 holds its own copy
    return procs


def launch_local(cmd: list[str], nproc: int, master_addr: str = "127.0.0.1",
                 master_port: int | None = None, timeout: float | None = None,
                 extra_env: dict | None = None) -> int:
    return _supervise(spawn_local_ranks(cmd, nproc, master_addr, master_port, extra_env), timeout)


def _supervise(procs: list[subprocess.Popen], timeout: float | None) -> int:
    deadline = time.time() + timeout if timeout else None
    failed_rc = 0
    while True:
        alive = False
        for p in procs:
            rc = p.poll()
            if rc is None:
                alive = True
            elif rc != 0 and not failed_rc:
                failed_rc = rc if rc > 0 else 128 - rc
        if failed_rc or not alive:
            break
        if deadline and time.time() > deadline:
            failed_rc = 124
            break
        time.sleep(0.05)
    if failed_rc:
        for p in procs:
            if p.poll() is None:
                _kill_group(p)
    for p in procs:
        p.wait()
    return failed_rc


def _kill_group(p: subprocess.Popen) -> None:
    for sig in (signal.SIGTERM, signal.SIGKILL):
        try:
            os.killpg(p.pid, sig)
        except ProcessLookupError:
            return
        try:
            p.wait(timeout=3)
            return
        except subprocess.TimeoutExpired:
            continue


# --------------------------------------------------------------------------------------
# mode 2: ranks on daemons
# --------------------------------------------------------------------------------------
class _RemoteRun(threading.Thread):
    """One rank (or stage) on a daemon; holds the connection for the process lifetime."""

    def __init__(self, host: Host, argv: list[str], env: dict, token: str | None,
                 timeout: float | None = None):
        super().__init__(daemon=True)
        self.host, self.argv, self.env, self.token = host, argv, env, token
        self.timeout = timeout
        self.reply: dict | None = None
        self.sock: socket.socket | None = None

    def run(self) -> None:
        try:
            self.sock = socket.create_connection((self.host.addr, self.host.port), timeout=30)
            self.sock.settimeout(None)
            req = {"op": "run", "argv": self.argv, "env": self.env, "timeout": self.timeout}
            if self.token:
                req["token"] = self.token
            send_msg(self.sock, req)
            self.reply = recv_msg(self.sock)
        except (OSError, ProtocolError) as e:
            self.reply = self.reply or {"ok": False, "rc": 255, "error": f"{self.host}: {e}"}
        finally:
            self.close()

    def close(self) -> None:
        s, self.sock = self.sock, None
        if s is not None:
            try:
                s.close()
            except OSError:
                pass


def _join_all(runs: list[_RemoteRun], what: str) -> int:
    for r in runs:
        r.start()
    failed = None
    while any(r.is_alive() for r in runs):
        for r in runs:
            if not r.is_alive() and r.reply is not None and not r.reply.get("ok"):
                failed = r
                break
        if failed:
            break
        time.sleep(0.05)
    if failed is None:
        failed = next((r for r in runs if not (r.reply or {}).get("ok")), None)
    if failed is not None:
        for r in runs:
            r.close()  # the daemons kill the process groups of dropped connections
        for r in runs:
            r.join(timeout=10)
        rep = failed.reply or {}
        sys.stderr.write(f"locust launch: {what} failed on {failed.host}: rc={rep.get('rc')} "
                         f"{rep.get('error', '')}\n{rep.get('stderr', '')[-4000:]}\n")
        rc = rep.get("rc")
        return rc if isinstance(rc, int) and rc > 0 else 1
    return 0


def launch_remote(cmd: list[str], hosts: list[Host], nproc_per_host: int,
                  master_addr: str | None = None, master_port: int | None = None,
                  token: str | None = None, replies: list | None = None) -> int:
    """Start world = sum over hosts of min(nproc_per_host, gpus=) ranks on the daemons.
    `replies` (optional) receives each rank's daemon reply, in rank order."""
    placement: list[tuple[Host, int]] = []
    for h in hosts:
        for lr in range(min(nproc_per_host, h.gpus or nproc_per_host)):
            placement.append((h, lr))
    world = len(placement)
    addr = master_addr or hosts[0].addr
    port = master_port or _free_port()
    runs = []
    for rank, (h, lr) in enumerate(placement):
        env = rank_env(rank, lr, world, addr, port)
        env["LOCAL_WORLD_SIZE"] = str(sum(1 for hh, _ in placement if hh == h))
        runs.append(_RemoteRun(h, cmd, env, token))
    rc = _join_all(runs, "rank")
    if replies is not None:
        replies.extend(r.reply for r in runs)
    return rc


# --------------------------------------------------------------------------------------
# mode 3: stage-split WordCount over daemons
# --------------------------------------------------------------------------------------
def _fetch(host: Host, path: str, dest: str, token: str | None) -> None:
    off = 0
    with open(dest, "wb") as f:
        while True:
            req = {"op": "get", "path": path, "offset": off, "length": 32 << 20}
            if token:
                req["token"] = token
            rep = request(host.addr, host.port, req, timeout=120)
            if not rep.get("ok"):
                raise RuntimeError(f"fetch {path} from {host}: {rep.get('error')}")
            data = base64.b64decode(rep["data"])
            f.write(data)
            off += len(data)
            if rep.get("eof") or not data:
                break


def _req(host: Host, obj: dict, token: str | None, timeout: float = 120) -> dict:
    if token:
        obj = dict(obj, token=token)
    return request(host.addr, host.port, obj, timeout=timeout)


def _get_small(host: Host, name: str, token: str | None, limit: int = 1 << 20) -> bytes | None:
    """A small file of a daemon's root (a map record, an index), or None."""
    try:
        rep = _req(host, {"op": "get", "path": name, "offset": 0, "length": limit}, token, 60)
    except (OSError, ProtocolError):
        return None
    return base64.b64decode(rep["data"]) if rep.get("ok") else None


def _spill_done(host: Host, k: int, argv: list[str], path: str, token: str | None) -> bool:
    """Host k's stage-1 output from an earlier run can stand in for this one:
    the launcher's record of that run names the same command line (input, byte range,
    backend, tokenizer flags), the map record's input identity (size, mtime, inode) equals
    the input file's on that host now, and the spill is present at the size its index
    describes."""
    import json

    from .spillindex import parse_index

    job, rec, idx = (_get_small(host, n, token) for n in
                     (f"out.{k}.launch.json", f"out.{k}.map.json", f"out.{k}.kv.idx"))
    if job is None or rec is None or idx is None:
        return False
    try:
        j, m, x = json.loads(job), json.loads(rec), parse_index(idx)
        st = _req(host, {"op": "stat", "path": path}, token, 60)
        sp = _req(host, {"op": "get", "path": f"out.{k}.kv", "offset": 0, "length": 0}, token, 60)
    except (ValueError, OSError, ProtocolError):
        return False
    if not (st.get("ok") and sp.get("ok")):
        return False
    return (j.get("argv") == argv and m.get("mode") == "map_stage" and m.get("input") == path
            and m.get("input_size") == st["size"] and m.get("input_mtime_ns") == st["mtime_ns"]
            and m.get("input_inode") == st["inode"] and sp.get("size") == x.spill_bytes
            and m.get("spill_bytes") == x.spill_bytes)


def _put_bytes(host: Host, path: str, data: bytes, token: str | None) -> None:
    rep = _req(host, {"op": "put", "path": path, "data": base64.b64encode(data).decode(),
                      "append": False}, token)
    if not rep.get("ok"):
        raise RuntimeError(f"put {path} to {host}: {rep.get('error')}")


def count_lines(path: str) -> int:
    """Lines of a file (a final line without a newline counts): the native parallel scan
    when the extension is built, else a Python pass."""
    try:
        from .. import _C  # type: ignore[attr-defined]

        return int(_C.find_line_window(path, 0, -1)[2])
    except Exception:  # noqa: BLE001 -- no native module on this host: count here
        n, last = 0, b"\n"
        with open(path, "rb") as f:
            for block in iter(lambda: f.read(1 << 24), b""):
                n += block.count(b"\n")
                last = block[-1:]
        return n + (0 if last == b"\n" else 1)


def stage_split_wordcount(path: str, hosts: list[Host], cli: str, token: str | None = None,
                          backend: str = "gpu", workdir: str | None = None,
                          remote_root: str | None = None, extra: list[str] | None = None,
                          reducers: int | None = None, out=None, resume: bool = False,
                          mapped: list | None = None, traffic: dict | None = None) -> int:
    """The reference's distributed WordCount (README.md:18-29): map on every host, then R
    key-range reducers on the hosts (default R = number of hosts).

    1. Host k runs stage 1 on bytes [k*S/H, (k+1)*S/H) of the S-byte input, both ends moved
       to line starts by the CLI (``--byte-range``): the launcher needs the file's size only,
       and no mapper scans the file's prefix for its window (the reference passes line
       numbers, main.cu:369-374).  Its combined (key, count) spill out.k.kv and index
       out.k.kv.idx land in its daemon root.
    2. Only the indexes come here (a few KiB each).  From them the launcher plans the same
       splitters every reducer computes and, for reducer r and spill k, the byte slice the
       reducer reads: the header, and from the last index sample below its key range to the
       first record past it.
    3. Reducer r (on host r mod H) has its daemon pull those slices straight from the
       mapper daemons (``pull``: a sparse file at the spill's own offsets, plus the index),
       or reads the spill in place when it mapped it itself; then it runs stage 2 with
       ``--reducer r/R`` and writes its result lines, with their global val, to
       ``result.r.txt``.  No spill byte passes through the launcher.
    4. The results are fetched and concatenated in reducer order -- the single-stage
       output byte for byte.  The first failing stage stops the job (its exit code).

    resume: the map outputs are the job's checkpoint -- a host whose spill
    and index from an earlier run of the same command on the unchanged input are still in
    its root is not mapped again (_spill_done).  `mapped` (optional) receives the hosts that
    ran stage 1; `traffic` (optional) gets the bytes each reducer pulled per spill, the
    bytes the launcher fetched, and the splitters."""
    import json
    import tempfile

    from .spillindex import parse_index, plan_splitters, reducer_range, reducer_slices

    out = out or sys.stdout.buffer
    apath = os.path.abspath(path)
    size = os.path.getsize(apath)
    parts = len(hosts)
    reducers = max(1, reducers or parts)
    hello = []
    for h in hosts:
        rep = _req(h, {"op": "hello"}, token)
        if not rep.get("ok"):
            raise RuntimeError(f"{h}: {rep.get('error')}")
        hello.append(rep)
    roots = [remote_root or hello[k]["root"] for k in range(parts)]
    runs, argvs, ran = [], {}, []
    for k, h in enumerate(hosts):
        a, b = size * k // parts, size * (k + 1) // parts
        rng = f"{a}:{b}" if k < parts - 1 else f"{a}:"
        argv = [cli, apath, "0", "0", str(k), "1", "--byte-range", rng, "--spill-dir", roots[k],
                "--spill-format", "binary", "--backend", backend,
                "--json", f"{roots[k]}/out.{k}.map.json"] + list(extra or [])
        argvs[k] = argv
        if resume and _spill_done(h, k, argv, apath, token):
            continue
        _put_bytes(h, f"out.{k}.launch.json", b"", token)  # (void until this map succeeds)
        runs.append(_RemoteRun(h, argv, {}, token))
        ran.append(k)
    if mapped is not None:
        mapped.extend(ran)
    rc = _join_all(runs, "map stage") if runs else 0
    if rc:
        return rc
    for k in ran:
        _put_bytes(hosts[k], f"out.{k}.launch.json", json.dumps({"argv": argvs[k]}).encode(), token)
    tmp = workdir or tempfile.mkdtemp(prefix="locust_results_")
    os.makedirs(tmp, exist_ok=True)
    fetched = 0
    idx = []
    for k, h in enumerate(hosts):
        data = _get_small(hosts[k], f"out.{k}.kv.idx", token, 64 << 20)
        if data is None:
            raise RuntimeError(f"{h}: no spill index out.{k}.kv.idx")
        fetched += len(data)
        idx.append(parse_index(data))
    spl = plan_splitters(idx, reducers)
    pulled = [[0] * parts for _ in range(reducers)]
    # every (reducer, remote spill) pull at once: each is one request to the reducer host's
    # daemon, which fetches from the mapper's daemon (both serve requests on threads)
    pulls, inputs_of = [], []
    for r in range(reducers):
        hk = r % parts
        lo, hi = reducer_range(spl, r)
        inputs = []
        for k in range(parts):
            if k == hk:  # its own map output: read in place
                inputs.append(f"{roots[hk]}/out.{k}.kv")
                continue
            dest = f"spills/r{r}/out.{k}.kv"
            for name, rngs, sz in ((dest, reducer_slices(idx[k], lo, hi), idx[k].spill_bytes),
                                   (dest + ".idx", [(0, -1)], None)):
                pulls.append((r, k, sz, {"op": "pull", "peer": [hosts[k].addr, hosts[k].port],
                                         "src": f"out.{k}.kv" + name[len(dest):], "dest": name,
                                         "size": sz, "ranges": [list(x) for x in rngs]}))
            inputs.append(f"{roots[hk]}/{dest}")
        inputs_of.append(inputs)
    if pulls:
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(max_workers=min(16, len(pulls))) as pool:
            reps = list(pool.map(lambda x: _req(hosts[x[0] % parts], x[3], token, 600), pulls))
        for (r, k, sz, _q), rep in zip(pulls, reps):
            if not rep.get("ok"):
                raise RuntimeError(f"reducer {r} on {hosts[r % parts]}: {rep.get('error')}")
            if sz is not None:
                pulled[r][k] += rep["bytes"]
    runs = []
    for r in range(reducers):
        hk = r % parts
        argv = [cli, apath, "0", "0", str(r), "2", "--inputs", ",".join(inputs_of[r]),
                "--reducer", f"{r}/{reducers}", "--result-file", f"{roots[hk]}/result.{r}.txt",
                "--backend", backend] + list(extra or [])
        runs.append(_RemoteRun(hosts[hk], argv, {}, token))
    rc = _join_all(runs, "reduce stage")
    if rc:
        return rc
    out.write(b"Running\n")
    for r in range(reducers):
        dest = os.path.join(tmp, f"result.{r}.txt")
        _fetch(hosts[r % parts], f"result.{r}.txt", dest, token)
        fetched += os.path.getsize(dest)
        with open(dest, "rb") as f:
            out.write(f.read())
    out.write(b"\nDone\n")
    out.flush()
    if traffic is not None:
        traffic.update({"pulled": pulled, "launcher_fetched": fetched, "splitters": spl,
                        "indexes": idx})
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m locust_amd.parallel.launch",
                                 description="Locust job launcher (local ranks, daemons, "
                                             "stage-split WordCount)")
    ap.add_argument("--nproc", type=int, default=0, help="local ranks (mode 1)")
    ap.add_argument("--hosts", help="hosts file of worker daemons (modes 2 and 3)")
    ap.add_argument("--nproc-per-host", type=int, default=1)
    ap.add_argument("--master-addr", default=None)
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("--token-file", default=None,
                    help="the daemons' shared secret (default: LOCUST_TOKEN)")
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("--wordcount", metavar="FILE", help="stage-split WordCount of FILE (mode 3)")
    ap.add_argument("--backend", default="gpu", choices=["gpu", "cpu"])
    ap.add_argument("--cli", default=None, help="path of the MapReduce binary")
    ap.add_argument("--reducers", type=int, default=0,
                    help="key-range reducers of --wordcount (default: one per host)")
    ap.add_argument("--output-format", choices=["gpu", "cpu"], default=None,
                    help="--wordcount result lines: GPU build's (with val) or CPU build's")
    ap.add_argument("--resume", action="store_true",
                    help="--wordcount: keep the map outputs of an earlier run of the same "
                         "command on the unchanged input (only missing or stale ones map again)")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    token = os.environ.get("LOCUST_TOKEN")
    if a.token_file:
        with open(a.token_file, encoding="utf-8") as f:
            token = f.read().strip()
    if a.wordcount:
        if not a.hosts:
            ap.error("--wordcount needs --hosts")
        from .._native import cli_path

        extra = ["--output-format", a.output_format] if a.output_format else []
        return stage_split_wordcount(a.wordcount, load_hosts(a.hosts), a.cli or cli_path(),
                                     token, a.backend, extra=extra, reducers=a.reducers or None,
                                     resume=a.resume)
    if not cmd:
        ap.error("no command given (put it after --)")
    if a.hosts:
        return launch_remote(cmd, load_hosts(a.hosts), a.nproc_per_host, a.master_addr,
                             a.master_port, token)
    return launch_local(cmd, max(a.nproc, 1), a.master_addr or "127.0.0.1", a.master_port,
                        a.timeout)


if __name__ == "__main__":
    sys.exit(main())
