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


def init_rank(cfg, max_bytes: int, max_lines: int, comm: str = "rccl", timeout: float = 300.0):
    """A :class:`locust_amd._locust.DistRank` for this process, from RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT (set by this launcher or by torch.distributed.run).  The
    framework's own bootstrap listens on MASTER_PORT + 1 (LOCUST_PORT overrides)."""
    from .. import _C

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if cfg.world != world:
        raise ValueError(f"DistConfig.world={cfg.world} but WORLD_SIZE={world}")
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("LOCUST_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 1))
    return _C.DistRank(cfg, rank, comm, host, port, max_bytes, max_lines, timeout)


__all__ = ["Host", "load_hosts", "parse_hosts", "launch_local", "launch_remote",
           "stage_split_wordcount", "init_rank"]
