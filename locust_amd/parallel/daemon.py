"""Worker daemon: runs stages / ranks for a launcher (replaces Distributor/slave.py).

    python -m locust_amd.parallel.daemon [--bind 127.0.0.1] [--port 1337] [--root DIR]
                                         [--token-file F | LOCUST_TOKEN]

What the reference's slave did (/root/reference/Distributor/slave.py:1-38) and what
changes here:

* It bound a hard-coded 127.0.0.1:1337, so one slave per machine -- the address and port
  are flags here, so several daemons can rehearse a cluster on one box.
* It served one connection at a time and replied ``ACK`` after ``subprocess.call``
  returned, whatever the exit code; a bare ``except`` tore the server down.  Here every
  connection has its own thread, the reply carries the exit code and output tails, a
  failed request answers an error instead of killing the server, and a client that
  disconnects mid-run (the launcher aborting a failed job) gets its process group killed.
* It ran any command anyone on the network sent it.  Here every request must carry the
  daemon's shared secret (``LOCUST_TOKEN`` or ``--token-file``; without one the daemon
  creates a random token in ``<root>/token``, mode 0600; a token file or root that another
  uid owns, that is group/world accessible or that is a symlink is refused, and the
  default root is per-user: ``$XDG_RUNTIME_DIR/locust`` or ``~/.cache/locust``, mode
  0700), and it only starts the
  framework's own programs (this repository's ``MapReduce`` binary, ``bench.py``, an
  allow-listed ``locust_amd`` module -- never a program that runs a command line it is
  given), from the repository root, with only rank-layout and ``LOCUST_*`` variables
  settable.  File transfer (spill files) is confined to ``--root``; files
  are opened with ``O_NOFOLLOW`` and the opened file's real path is checked again.

Requests (JSON frames, see protocol.py): ``hello``, ``run`` {argv, env, timeout},
``get`` {path, offset, length}, ``put`` {path, data, append}, ``stat`` {path} (size, mtime,
inode of an input file: a resume checks that the input is unchanged) and ``pull`` {peer,
src, dest, size, ranges}: this daemon fetches byte ranges of a file from a peer daemon
(same token) into a file of its own root, each at its own offset -- a sparse copy of the
spill of the same size, so the spill's index stays valid.  Reducers get their key range of
every spill this way, straight from the mapper hosts (the reference's missing inter-node
transfer), never through the launcher.  The reference's unauthenticated
raw-text form (``"<x> prog args..."``) is recognised and refused.
"""
from __future__ import annotations

import argparse
import base64
import hmac
import os
import signal
import socket
import socketserver
import stat
import subprocess
import sys
import threading
import time

from .protocol import PROTOCOL_VERSION, ProtocolError, recv_exact, recv_msg, send_msg

TAIL = 64 << 10  # bytes of stdout/stderr returned with a run reply


_REPO = os.path.realpath(os.path.join(os.path.dirname(__file__), "..", ".."))


# Programs a daemon may start: nothing that takes a command line to run in turn (so not
# the launcher itself), and no interpreter flags such as -c.
_MODULES = {"locust_amd.parallel.selftest"}
_SCRIPTS = {os.path.join(_REPO, "bench.py")}
# Environment a request may set: the rank layout and the framework's own switches; never
# loader/interpreter hooks (LD_*, PYTHON*).
_ENV_PREFIXES = ("LOCUST_",)
_ENV_KEYS = {"RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
             "MASTER_PORT", "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "OMP_NUM_THREADS"}


def _allowed(argv: list[str]) -> bool:
    """Only the framework's own programs: the repository's MapReduce binary, this Python
    interpreter running an allow-listed locust_amd module, or the benchmark script."""
    exe = os.path.realpath(argv[0])
    if exe == os.path.join(_REPO, "build", "MapReduce"):
        return True
    if exe != os.path.realpath(sys.executable) or len(argv) < 2:
        return False
    if argv[1] == "-m":
        return len(argv) > 2 and argv[2] in _MODULES
    return os.path.isabs(argv[1]) and os.path.realpath(argv[1]) in _SCRIPTS


def _env_allowed(env: dict) -> bool:
    return all(isinstance(k, str) and (k in _ENV_KEYS or k.startswith(_ENV_PREFIXES))
               for k in env)


def default_root() -> str:
    """Per-user daemon root: $XDG_RUNTIME_DIR/locust, else ~/.cache/locust (never a shared
    /tmp path another local user could create first)."""
    base = os.environ.get("XDG_RUNTIME_DIR") or os.path.join(os.path.expanduser("~"), ".cache")
    return os.path.join(base, "locust")


def _check_private(path: str, what: str) -> None:
    """Refuse a token file / root not owned by this uid or accessible by group/others."""
    st = os.lstat(path)
    if stat.S_ISLNK(st.st_mode):
        raise PermissionError(f"{what} {path!r} is a symlink")
    if st.st_uid != os.getuid():
        raise PermissionError(f"{what} {path!r} is owned by uid {st.st_uid}, not {os.getuid()}")
    if st.st_mode & 0o077:
        raise PermissionError(f"{what} {path!r} is group/world accessible "
                              f"(mode {stat.S_IMODE(st.st_mode):o}); chmod go= it")


def ensure_private_dir(root: str) -> str:
    """Create `root` mode 0700 (or verify an existing one is ours and private)."""
    root = os.path.abspath(root)
    os.makedirs(os.path.dirname(root), exist_ok=True)
    try:
        os.mkdir(root, 0o700)
    except FileExistsError:
        pass
    _check_private(root, "daemon root")
    return os.path.realpath(root)


def load_or_create_token(root: str, token_file: str | None = None) -> str:
    """The daemon's shared secret: LOCUST_TOKEN, the token file, or a fresh random token
    written to <root>/token (mode 0600) for the launcher to read.  A token file that is
    not ours or is readable by others is refused (someone else may have planted it)."""
    if os.environ.get("LOCUST_TOKEN"):
        return os.environ["LOCUST_TOKEN"]
    if token_file is None:
        root = ensure_private_dir(root)
    path = token_file or os.path.join(root, "token")
    if os.path.lexists(path):
        _check_private(path, "token file")
        fd = os.open(path, os.O_RDONLY | os.O_NOFOLLOW)
        with os.fdopen(fd, encoding="utf-8") as f:
            tok = f.read().strip()
        if tok:
            return tok
    import secrets

    tok = secrets.token_hex(24)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC | os.O_NOFOLLOW, 0o600)
    with os.fdopen(fd, "w", encoding="utf-8") as f:
        f.write(tok + "\n")
    return tok


class _Server(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True

    def __init__(self, addr, root: str, token: str):
        if not token:
            raise ValueError("the daemon needs a token (LOCUST_TOKEN or a token file)")
        super().__init__(addr, _Handler)
        self.root = ensure_private_dir(root)
        self.token = token


class _Handler(socketserver.BaseRequestHandler):
    server: _Server

    def handle(self) -> None:
        sock: socket.socket = self.request
        try:
            head = recv_exact(sock, 4)
        except ProtocolError:
            return
        if _looks_like_text(head):
            self._handle_text(sock, head)
            return
        try:
            n = int.from_bytes(head, "big")
            body = recv_exact(sock, n)
            import json

            req = json.loads(body.decode())
            reply = self._dispatch(req, sock)
        except Exception as e:  # report, never take the server down
            reply = {"ok": False, "error": f"{type(e).__name__}: {e}"}
        try:
            send_msg(sock, reply)
        except OSError:
            pass

    # ---- the reference's text protocol: unauthenticated, so refused ----
    def _handle_text(self, sock: socket.socket, head: bytes) -> None:
        sock.sendall(b"NAK unauthenticated text commands are not accepted; "
                     b"use python -m locust_amd.parallel.launch")

    # ---- JSON requests ----
    def _dispatch(self, req: dict, sock: socket.socket) -> dict:
        if not hmac.compare_digest(str(req.get("token", "")), self.server.token):
            return {"ok": False, "error": "authentication failed"}
        op = req.get("op")
        if op == "hello":
            return {"ok": True, "version": PROTOCOL_VERSION, "host": socket.gethostname(),
                    "root": self.server.root, "pid": os.getpid()}
        if op == "run":
            argv = req.get("argv")
            if not isinstance(argv, list) or not argv or not all(isinstance(a, str) for a in argv):
                return {"ok": False, "error": "run: argv must be a non-empty list of strings"}
            if not _allowed(argv):
                return {"ok": False, "error": f"run: {argv[0]!r} is not one of the framework's "
                                             "programs"}
            bad = self._writes_outside_root(argv)
            if bad:
                return {"ok": False, "error": f"run: {bad} must name a path inside the daemon "
                                             f"root {self.server.root}"}
            env = req.get("env") or {}
            if not isinstance(env, dict) or not _env_allowed(env):
                return {"ok": False, "error": "run: env may only set the rank layout "
                                             "(RANK, WORLD_SIZE, MASTER_*, ...) and LOCUST_*"}
            # the CLI's per-file caches (partition maps, line indexes) stay inside the root
            env = dict(env)
            env["LOCUST_CACHE_DIR"] = os.path.join(self.server.root, "cache")
            t0 = time.time()
            # always run from the repository root (module imports resolve to this package)
            rc, out, err = _run(argv, env, _REPO, req.get("timeout"), sock)
            return {"ok": rc == 0, "rc": rc, "stdout": out, "stderr": err,
                    "elapsed": time.time() - t0}
        if op == "get":
            path = self._path(req.get("path", ""))
            off, length = int(req.get("offset", 0)), int(req.get("length", 64 << 20))
            # O_NOFOLLOW + a re-check of the opened file: a symlink planted between the
            # realpath check and the open cannot redirect the read out of the root
            with os.fdopen(self._open_checked(path, os.O_RDONLY), "rb") as f:
                f.seek(off)
                data = f.read(length)
                eof = f.tell() >= os.fstat(f.fileno()).st_size
            return {"ok": True, "data": base64.b64encode(data).decode(), "eof": eof,
                    "size": os.path.getsize(path)}
        if op == "put":
            path = self._path(req.get("path", ""))
            os.makedirs(os.path.dirname(path), exist_ok=True)
            flags = os.O_WRONLY | os.O_CREAT | (os.O_APPEND if req.get("append") else os.O_TRUNC)
            with os.fdopen(self._open_checked(path, flags), "ab" if req.get("append") else "wb") as f:
                f.write(base64.b64decode(req.get("data", "")))
            return {"ok": True}
        if op == "stat":
            st = os.stat(str(req.get("path", "")))
            return {"ok": True, "size": st.st_size, "mtime_ns": st.st_mtime_ns,
                    "inode": st.st_ino}
        if op == "pull":
            return self._pull(req)
        return {"ok": False, "error": f"unknown op {op!r}"}

    def _pull(self, req: dict) -> dict:
        """Byte ranges of `src` on a peer daemon into `dest` under this root, each written at
        its own offset; `size` (optional) sets the file's length (the rest stays a hole)."""
        from .protocol import request as _request

        peer = req.get("peer")
        if not (isinstance(peer, list) and len(peer) == 2 and isinstance(peer[0], str)
                and isinstance(peer[1], int)):
            return {"ok": False, "error": "pull: peer must be [address, port]"}
        ranges = req.get("ranges") or [[0, -1]]
        try:
            ranges = [(int(o), int(n)) for o, n in ranges]
            size = None if req.get("size") is None else int(req["size"])
        except (TypeError, ValueError):
            return {"ok": False, "error": "pull: ranges must be [offset, length] integer pairs"}
        if any(o < 0 or n < -1 for o, n in ranges) or (size is not None and size < 0):
            return {"ok": False, "error": "pull: negative offset, length or size"}
        dest = self._path(req.get("dest", ""))
        os.makedirs(os.path.dirname(dest), exist_ok=True)
        fd = self._open_checked(dest, os.O_WRONLY | os.O_CREAT | os.O_TRUNC)
        got = 0
        frame = 32 << 20
        try:
            for off, length in ranges:
                pos = off
                while length < 0 or pos < off + length:
                    want = frame if length < 0 else min(frame, off + length - pos)
                    rep = _request(peer[0], peer[1], {"op": "get", "token": self.server.token,
                                                      "path": str(req.get("src", "")),
                                                      "offset": pos, "length": want},
                                   timeout=120)
                    if not rep.get("ok"):
                        return {"ok": False, "error": f"pull from {peer[0]}:{peer[1]}: "
                                                      f"{rep.get('error')}"}
                    data = base64.b64decode(rep["data"])
                    if data:
                        os.pwrite(fd, data, pos)
                    pos += len(data)
                    got += len(data)
                    if rep.get("eof") or not data:
                        break
            if size is not None:
                os.ftruncate(fd, size)
        finally:
            os.close(fd)
        return {"ok": True, "bytes": got}

    def _writes_outside_root(self, argv: list[str]) -> str | None:
        """The CLI's file-writing flags may only target the daemon root."""
        writing = {"--spill-dir", "--gen", "--json", "--result-file", "--export-kiv"}
        for i, a in enumerate(argv[:-1]):
            if a in writing:
                try:
                    self._path(argv[i + 1])
                except PermissionError:
                    return a
        return None

    def _open_checked(self, path: str, flags: int) -> int:
        fd = os.open(path, flags | os.O_NOFOLLOW, 0o600)
        try:
            real = os.path.realpath(f"/proc/self/fd/{fd}") if os.path.exists("/proc/self/fd") else path
            if real != self.server.root and not real.startswith(self.server.root + os.sep):
                raise PermissionError(f"path {path!r} escapes the daemon root")
        except BaseException:
            os.close(fd)
            raise
        return fd

    def _path(self, rel: str) -> str:
        p = os.path.realpath(os.path.join(self.server.root, rel))
        if p != self.server.root and not p.startswith(self.server.root + os.sep):
            raise PermissionError(f"path {rel!r} escapes the daemon root")
        return p


def _looks_like_text(head: bytes) -> bool:
    # A JSON frame starts with a 4-byte length < 256 MiB, i.e. a 0x00..0x0f first byte;
    # the reference's commands start with printable ASCII.
    return head[0] >= 0x20


def _run(argv, env, cwd, timeout, sock: socket.socket):
    """Run argv in its own process group; kill the group if the client goes away or the
    timeout passes.  Returns (rc, stdout tail, stderr tail)."""
    full_env = dict(os.environ)
    full_env.update({str(k): str(v) for k, v in (env or {}).items()})
    try:
        p = subprocess.Popen(argv, env=full_env, cwd=cwd, stdout=subprocess.PIPE,
                             stderr=subprocess.PIPE, start_new_session=True)
    except OSError as e:
        return 127, "", f"cannot start {argv[0]!r}: {e}"
    out_buf, err_buf = bytearray(), bytearray()

    def pump(stream, buf):
        for chunk in iter(lambda: stream.read(1 << 16), b""):
            buf += chunk
            if len(buf) > 2 * TAIL:
                del buf[:-TAIL]

    threads = [threading.Thread(target=pump, args=(p.stdout, out_buf), daemon=True),
               threading.Thread(target=pump, args=(p.stderr, err_buf), daemon=True)]
    for t in threads:
        t.start()
    deadline = time.time() + float(timeout) if timeout else None
    while p.poll() is None:
        if deadline and time.time() > deadline:
            _kill_group(p)
            break
        if _peer_closed(sock):
            _kill_group(p)
            break
        time.sleep(0.05)
    rc = p.wait()
    for t in threads:
        t.join(timeout=5)
    return rc, out_buf[-TAIL:].decode(errors="replace"), err_buf[-TAIL:].decode(errors="replace")


def _peer_closed(sock: socket.socket) -> bool:
    try:
        sock.setblocking(False)
        try:
            data = sock.recv(1, socket.MSG_PEEK)
            return data == b""
        except (BlockingIOError, InterruptedError):
            return False
        finally:
            sock.setblocking(True)
    except OSError:
        return True


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


def serve(bind: str = "127.0.0.1", port: int = 1337, root: str | None = None,
          token: str | None = None, ready=None) -> None:
    root = root or default_root()
    token = token or load_or_create_token(root)
    with _Server((bind, port), root, token) as srv:
        if ready is not None:
            ready(srv.server_address[1])
        print(f"locust daemon listening on {bind}:{srv.server_address[1]} (root {srv.root})",
              file=sys.stderr, flush=True)
        srv.serve_forever()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--bind", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=1337)
    ap.add_argument("--root", default=None,
                    help="directory for file transfers, mode 0700 (default: "
                         "$XDG_RUNTIME_DIR/locust or ~/.cache/locust)")
    ap.add_argument("--token-file", default=None,
                    help="shared secret file (default: LOCUST_TOKEN, else <root>/token)")
    a = ap.parse_args(argv)
    a.root = a.root or default_root()
    token = load_or_create_token(a.root, a.token_file)
    try:
        serve(a.bind, a.port, a.root, token)
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
