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


def _port_file_path(master: int) -> str:
    """Where rank 0 of a torchrun job publishes its bootstrap port.  Named after what every
    rank of ONE attempt shares -- the rendezvous run id, the restart count and MASTER_PORT --
    so a restarted attempt (``--max-restarts``) never reads the previous attempt's port, and
    ranks started through per-rank wrappers (different parent pids) still agree."""
    import tempfile

    # a per-user directory when there is one; in a shared /tmp a reader only trusts a file
    # this user owns and nobody else can write
    base = os.environ.get("XDG_RUNTIME_DIR", "")
    if not (base and os.path.isdir(base) and os.access(base, os.W_OK)):
        base = tempfile.gettempdir()
    run = "".join(c if c.isalnum() or c in "-_" else "_"
                  for c in os.environ.get("TORCHELASTIC_RUN_ID", "none"))[:64]
    restart = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    return os.path.join(base, f"locust_port_{run}_{restart}_{master}_{os.getuid()}")


def bootstrap_listener(rank: int | None = None, world: int | None = None,
                       timeout: float = 120.0) -> tuple[int, int]:
    """``(port, listen_fd)`` of the framework's bootstrap (the RCCL unique id and the TCP
    communicator's control messages go through rank 0's listening socket).  ``listen_fd``
    is a socket already bound to ``port`` and listening, for rank 0 to hand to the native
    communicator (``DistRank(..., listen_fd=)``), or -1 when the communicator binds itself:

    * ``LOCUST_LISTEN_FD`` + ``LOCUST_PORT`` (rank 0 of a launcher that bound the socket
      itself and passed it down: ``bench.py --gpus N``, :func:`launch.launch_local`);
    * ``LOCUST_PORT`` alone: that port (every rank must see the same value);
    * under ``torch.distributed.run`` on one node (``TORCHELASTIC_RUN_ID`` set, world > 1,
      every rank local): rank 0 binds port 0, listens, and publishes the port in a file
      (:func:`_port_file_path`); the other ranks read it there.  The socket never closes
      between the choice of the port and its use, so no other process can take it.  No
      torch import: the engine's HIP/RCCL must stay the only ones in the process;
    * otherwise MASTER_PORT + 1."""
    global _port_file
    rank = int(os.environ.get("RANK", "0")) if rank is None else rank
    world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else world
    if "LOCUST_PORT" in os.environ:
        fd = int(os.environ.get("LOCUST_LISTEN_FD", "-1")) if rank == 0 else -1
        os.environ.pop("LOCUST_LISTEN_FD", None)  # one owner: never handed out twice
        return int(os.environ["LOCUST_PORT"]), fd
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    master = int(os.environ.get("MASTER_PORT", "29500"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", "0"))
    if world > 1 and "TORCHELASTIC_RUN_ID" in os.environ and local_world == world:
        import socket
        import time

        path = _port_file_path(master)
        if rank == 0:
            s = socket.socket()
            try:
                s.bind((host, 0))
                s.listen(world)
                port = s.getsockname()[1]
                tmp = f"{path}.{os.getpid()}"
                fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
                with os.fdopen(fd, "w") as f:
                    f.write(str(port))
                os.replace(tmp, path)  # readers never see a partial file
            except BaseException:
                s.close()
                raise
            _port_file = path
            return port, s.detach()
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            try:
                fd = os.open(path, os.O_RDONLY | os.O_NOFOLLOW)
                with os.fdopen(fd) as f:
                    st = os.fstat(f.fileno())
                    txt = f.read().strip()
                if txt and st.st_uid == os.getuid() and not st.st_mode & 0o022:
                    return int(txt), -1
            except (FileNotFoundError, OSError):
                pass
            time.sleep(0.005)
        raise TimeoutError(f"rank {rank}: no bootstrap port from rank 0 in {path} "
                           f"after {timeout:.0f} s")
    return master + 1, -1


def bootstrap_port(rank: int | None = None, world: int | None = None,
                   timeout: float = 120.0) -> int:
    """The bootstrap port alone (see :func:`bootstrap_listener`; a listening socket it
    created is closed here, so prefer :func:`bootstrap_listener` + ``listen_fd``)."""
    port, fd = bootstrap_listener(rank, world, timeout)
    if fd >= 0:
        os.close(fd)
    return port


def release_bootstrap_port() -> None:
    """Rank 0, once every rank has connected (or the attempt failed): remove the published
    port file."""
    global _port_file
    if _port_file:
        try:
            os.unlink(_port_file)
        except FileNotFoundError:
            pass
        _port_file = None


def connect_rank(cfg, rank: int, world: int, comm: str, max_bytes: int, max_lines: int,
                 timeout: float = 300.0):
    """A :class:`locust_amd._locust.DistRank` (communicator + engine) for this process: the
    bootstrap listener goes to the native communicator, and the port file is removed
    whether or not the ranks meet."""
    from .. import _C

    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port, fd = bootstrap_listener(rank, world)
    try:
        return _C.DistRank(cfg, rank, comm, host, port, max_bytes, max_lines, timeout, fd)
    finally:
        release_bootstrap_port()  # every rank connected inside the constructor (or failed)


def init_rank(cfg, max_bytes: int, max_lines: int, comm: str = "rccl", timeout: float = 300.0):
    """A :class:`locust_amd._locust.DistRank` for this process, from RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT (set by this launcher or by torch.distributed.run)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if cfg.world != world:
        raise ValueError(f"DistConfig.world={cfg.world} but WORLD_SIZE={world}")
    if comm == "rccl":  # on the GPU's NUMA node before the engine allocates anything
        from .numa import bind_to_gpu

        bind_to_gpu(cfg.job.device)
    return connect_rank(cfg, rank, world, comm, max_bytes, max_lines, timeout)


__all__ = ["Host", "load_hosts", "parse_hosts", "launch_local", "launch_remote",
           "stage_split_wordcount", "init_rank", "connect_rank", "bootstrap_listener",
           "bootstrap_port", "release_bootstrap_port"]
