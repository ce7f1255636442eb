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


_PORT_KEY = "locust_amd/bootstrap_port"


def bootstrap_port(rank: int | None = None, world: int | None = None,
                   timeout: float = 120.0) -> int:
    """The TCP port rank 0 of the framework's bootstrap listens on (the RCCL unique id and
    the TCP communicator's control messages go through it).

    * ``LOCUST_PORT`` if set (every rank must see the same value);
    * under ``torch.distributed.run`` (``TORCHELASTIC_RUN_ID`` set, world > 1): rank 0 asks
      the OS for a free port and publishes it in the agent's rendezvous store at
      MASTER_ADDR:MASTER_PORT, the other ranks read it there -- no guess that
      MASTER_PORT + 1 happens to be free on the node;
    * otherwise MASTER_PORT + 1 (this package's launcher keeps that one free)."""
    if "LOCUST_PORT" in os.environ:
        return int(os.environ["LOCUST_PORT"])
    rank = int(os.environ.get("RANK", "0")) if rank is None else rank
    world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else world
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    master = int(os.environ.get("MASTER_PORT", "29500"))
    if world > 1 and "TORCHELASTIC_RUN_ID" in os.environ:
        try:
            return _port_from_store(host, master, rank, timeout)
        except Exception as e:  # noqa: BLE001  (no torch / no store: the fixed rule)
            import sys
            print(f"locust_amd: rendezvous store unavailable ({e}); bootstrap on "
                  f"MASTER_PORT+1", file=sys.stderr)
    return master + 1


def _port_from_store(host: str, master: int, rank: int, timeout: float) -> int:
    import datetime
    import socket

    from torch.distributed import TCPStore

    store = TCPStore(host, master, is_master=False,
                     timeout=datetime.timedelta(seconds=timeout))
    run = os.environ.get("TORCHELASTIC_RUN_ID", "")
    restart = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    key = f"{_PORT_KEY}/{run}/{restart}"
    if rank == 0:
        with socket.socket() as s:  # released just before the communicator binds it
            s.bind((host, 0))
            port = s.getsockname()[1]
        store.set(key, str(port))
        return port
    return int(store.get(key).decode())


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
    return _C.DistRank(cfg, rank, comm, host, bootstrap_port(rank, world), max_bytes,
                       max_lines, timeout)


__all__ = ["Host", "load_hosts", "parse_hosts", "launch_local", "launch_remote",
           "stage_split_wordcount", "init_rank", "bootstrap_port"]
