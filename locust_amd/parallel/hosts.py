"""Hosts file of a distributed job.

The reference documents (but never parses) a hosts file of ``ip_address port`` lines
(/root/reference/README.md:18-22) for a master that does not exist.  Here it is parsed:

    # comment
    10.0.0.1 1337            # one worker daemon, all its GPUs
    10.0.0.2 1337 gpus=4     # at most 4 ranks on this host
    127.0.0.1 7001           # several daemons may share a host (distinct ports)

Blank lines and ``#`` comments are ignored.  ``gpus=N`` caps the ranks placed on a host
(default: the launcher's ``--nproc-per-host``).
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Host:
    addr: str
    port: int
    gpus: int | None = None

    def __str__(self) -> str:
        return f"{self.addr}:{self.port}"


def parse_hosts(text: str) -> list[Host]:
    hosts: list[Host] = []
    for lineno, raw in enumerate(text.splitlines(), 1):
        line = raw.split("#", 1)[0].strip()
        if not line:
            continue
        parts = line.split()
        if len(parts) < 2:
            raise ValueError(f"hosts line {lineno}: expected 'address port', got {raw!r}")
        addr, port_s, *opts = parts
        try:
            port = int(port_s)
        except ValueError:
            raise ValueError(f"hosts line {lineno}: bad port {port_s!r}") from None
        if not 0 < port < 65536:
            raise ValueError(f"hosts line {lineno}: port {port} out of range")
        gpus = None
        for o in opts:
            key, _, val = o.partition("=")
            if key != "gpus" or not val.isdigit() or int(val) < 1:
                raise ValueError(f"hosts line {lineno}: unknown option {o!r}")
            gpus = int(val)
        hosts.append(Host(addr, port, gpus))
    if not hosts:
        raise ValueError("hosts file lists no hosts")
    if len(set((h.addr, h.port) for h in hosts)) != len(hosts):
        raise ValueError("hosts file lists a daemon twice")
    return hosts


def load_hosts(path: str) -> list[Host]:
    with open(path, encoding="utf-8") as f:
        return parse_hosts(f.read())
