"""Distribution: launcher, worker daemon, hosts files and rank helpers.

Replaces /root/reference/Distributor/slave.py (a TCP command runner bound to
127.0.0.1:1337) and the master the reference's README describes but never shipped.

* :mod:`.launch`  -- local ranks (one process per GPU), ranks on daemons, stage-split jobs
* :mod:`.daemon`  -- the worker agent (JSON frames; the reference's text form still works)
* :mod:`.hosts`   -- ``address port [gpus=N]`` hosts files
* :func:`init_rank` -- a long-lived rank (RCCL or TCP) from the launcher's environment
"""
from __future__ import annotations

import os

from .hosts import Host, load_hosts, parse_hosts
from .launch import launch_local, launch_remote, stage_split_wordcount


_port_file: str | None = None


def bootstrap_port(rank: int | None = None, world: int | None = None,
                   timeout: float = 120.0) -> int:
    """The TCP port rank 0 of the framework's bootstrap listens on (the RCCL unique id and
    the TCP communicator's control messages go through it).

    * ``LOCUST_PORT`` if set (every rank must see the same value);
    * under ``torch.distributed.run`` on one node (``TORCHELASTIC_RUN_ID`` set, world > 1,
      every rank local): rank 0 asks the OS for a free port and publishes it in a file named
      after MASTER_PORT and the launching agent's pid (the ranks' common parent); the other
      ranks read it there -- no guess that MASTER_PORT + 1 happens to be free.  No torch
      import: the engine's HIP/RCCL must stay the only ones in the process;
    * otherwise MASTER_PORT + 1 (this package's launcher keeps that one free)."""
    global _port_file
    if "LOCUST_PORT" in os.environ:
        return int(os.environ["LOCUST_PORT"])
    rank = int(os.environ.get("RANK", "0")) if rank is None else rank
    world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else world
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    master = int(os.environ.get("MASTER_PORT", "29500"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", "0"))
    if world > 1 and "TORCHELASTIC_RUN_ID" in os.environ and local_world == world:
        import socket
        import tempfile
        import time

        # a per-user directory when there is one; in a shared /tmp a reader only trusts a
        # file this user owns and nobody else can write
        base = os.environ.get("XDG_RUNTIME_DIR", "")
        if not (base and os.path.isdir(base) and os.access(base, os.W_OK)):
            base = tempfile.gettempdir()
        path = os.path.join(base, f"locust_port_{master}_{os.getppid()}_{os.getuid()}")
        if rank == 0:
            with socket.socket() as s:  # released just before the communicator binds it
                s.bind((host, 0))
                port = s.getsockname()[1]
            tmp = f"{path}.{os.getpid()}"
            fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
            with os.fdopen(fd, "w") as f:
                f.write(str(port))
            os.replace(tmp, path)  # readers never see a partial file
            _port_file = path
            return port
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            try:
                fd = os.open(path, os.O_RDONLY | os.O_NOFOLLOW)
                with os.fdopen(fd) as f:
                    st = os.fstat(f.fileno())
                    txt = f.read().strip()
                if txt and st.st_uid == os.getuid() and not st.st_mode & 0o022:
                    return int(txt)
            except (FileNotFoundError, OSError):
                pass
            time.sleep(0.005)
        raise TimeoutError(f"rank {rank}: no bootstrap port from rank 0 in {path} "
                           f"after {timeout:.0f} s")
    return master + 1


def release_bootstrap_port() -> None:
    """Rank 0, once every rank has connected: remove the published port file."""
    global _port_file
    if _port_file:
        try:
            os.unlink(_port_file)
        except FileNotFoundError:
            pass
        _port_file = None


def init_rank(cfg, max_bytes: int, max_lines: int, comm: str = "rccl", timeout: float = 300.0):
    """A :class:`locust_amd._locust.DistRank` for this process, from RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT (set by this launcher or by torch.distributed.run).  The
    framework's own bootstrap port comes from :func:`bootstrap_port`."""
    from .. import _C

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if cfg.world != world:
        raise ValueError(f"DistConfig.world={cfg.world} but WORLD_SIZE={world}")
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    dr = _C.DistRank(cfg, rank, comm, host, bootstrap_port(rank, world), max_bytes,
                     max_lines, timeout)
    release_bootstrap_port()  # every rank connected inside the constructor
    return dr


__all__ = ["Host", "load_hosts", "parse_hosts", "launch_local", "launch_remote",
           "stage_split_wordcount", "init_rank", "bootstrap_port", "release_bootstrap_port"]
