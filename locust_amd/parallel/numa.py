"""NUMA placement of GPU ranks.

On a two-socket MI355X node half of the GPUs hang off each socket's PCIe root; a rank
whose CPU threads and pinned host buffers sit on the far socket pulls its text across the
socket link at a fraction of the ~55 GB/s its own x16 link gives.  So every rank process is
bound to the CPUs of its GPU's NUMA node *before any GPU call* (the HIP runtime's own
threads then start there too, and the pinned shard the engine allocates is first touched
there).  The GPU -> node mapping comes from sysfs only, no HIP call:

* ``/sys/class/kfd/kfd/topology/nodes/<n>/properties``: GPU nodes (``simd_count`` > 0) in
  the order HIP numbers devices, with ``domain`` and ``location_id`` (the PCI address);
* ``/sys/bus/pci/devices/<domain:bus:dev.fn>/numa_node`` and
  ``/sys/devices/system/node/node<k>/cpulist``.

``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES`` (indices)
select and reorder the devices as the runtime does.  Every function takes ``sys_root`` so
the tests can run on a fake tree.  The in-process clique's threads are placed by the C++
twin of this module (``csrc/engine/numa.cpp``).
"""
from __future__ import annotations

import os
import sys


def parse_cpulist(text: str) -> list[int]:
    """``0-3,8,10-11`` -> [0, 1, 2, 3, 8, 10, 11]."""
    out: list[int] = []
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _read(path: str) -> str | None:
    try:
        with open(path, encoding="ascii") as f:
            return f.read()
    except OSError:
        return None


def kfd_gpu_bdfs(sys_root: str = "/sys") -> list[str]:
    """PCI addresses of the GPUs in KFD topology order (the runtime's device order)."""
    base = os.path.join(sys_root, "class/kfd/kfd/topology/nodes")
    try:
        nodes = sorted((int(n) for n in os.listdir(base) if n.isdigit()))
    except OSError:
        return []
    out = []
    for n in nodes:
        txt = _read(os.path.join(base, str(n), "properties"))
        if not txt:
            continue
        props = {}
        for line in txt.splitlines():
            kv = line.split()
            if len(kv) == 2 and kv[1].lstrip("-").isdigit():
                props[kv[0]] = int(kv[1])
        if props.get("simd_count", 0) <= 0:
            continue  # a CPU node
        loc, dom = props.get("location_id", 0), props.get("domain", 0)
        out.append(f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}")
    return out


def visible_order(n: int, env: dict | None = None) -> list[int]:
    """Physical indices of the visible devices, in the order the runtime numbers them."""
    env = os.environ if env is None else env
    order = list(range(n))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is None or v == "":
            continue
        try:
            idx = [int(x) for x in v.split(",") if x.strip() != ""]
        except ValueError:
            continue  # UUIDs: leave the order alone
        order = [order[i] for i in idx if 0 <= i < len(order)]
    return order


def gpu_numa_node(device: int, sys_root: str = "/sys", env: dict | None = None) -> int:
    """NUMA node of visible HIP device `device` (-1: unknown)."""
    bdfs = kfd_gpu_bdfs(sys_root)
    order = visible_order(len(bdfs), env)
    if not 0 <= device < len(order):
        return -1
    txt = _read(os.path.join(sys_root, "bus/pci/devices", bdfs[order[device]], "numa_node"))
    try:
        return int(txt.strip()) if txt is not None else -1
    except ValueError:
        return -1


def node_cpus(node: int, sys_root: str = "/sys") -> list[int]:
    if node < 0:
        return []
    txt = _read(os.path.join(sys_root, f"devices/system/node/node{node}/cpulist"))
    return parse_cpulist(txt) if txt else []


def bind_to_gpu(device: int, sys_root: str = "/sys", env: dict | None = None,
                log: bool | None = None) -> dict:
    """Bind this process to the CPUs of `device`'s NUMA node (those it may use at all).
    Returns the placement; a no-op (node -1) where sysfs says nothing.  Call it before the
    first GPU call.  LOCUST_NUMA=0 switches it off; LOCUST_LOG=info|debug logs it."""
    env_ = os.environ if env is None else env
    place = {"device": device, "node": -1, "cpus": 0, "bound": False}
    if env_.get("LOCUST_NUMA", "1") == "0":
        return place
    node = gpu_numa_node(device, sys_root, env)
    place["node"] = node
    cpus = node_cpus(node, sys_root)
    try:
        allowed = os.sched_getaffinity(0)
    except (AttributeError, OSError):
        allowed = set(cpus)
    mine = sorted(set(cpus) & allowed)
    if mine:
        try:
            os.sched_setaffinity(0, mine)
            place["bound"] = True
        except OSError:
            pass
    place["cpus"] = len(mine)
    if log is None:
        log = env_.get("LOCUST_LOG", "") in ("info", "debug")
    if log:
        print(f"[locust INFO] rank on GPU {device}: NUMA node {node}, "
              f"{'bound to ' + str(len(mine)) + ' CPUs' if place['bound'] else 'not bound'}",
              file=sys.stderr, flush=True)
    return place
