"""NUMA placement from sysfs, on a fake tree: two sockets, four GPUs
(two per socket) interleaved with the CPU nodes of the KFD topology; visible-device
reordering; the process binding; the C++ twin the in-process clique threads use."""
import os

import pytest

import locust_amd as lc
from locust_amd.parallel import numa

# KFD node -> (simd_count, domain, location_id); GPU i at bus 0x10 * (i + 1)
GPUS = [(0, 0x10, 0), (0, 0x20, 0), (0, 0x90, 1), (0, 0xa0, 1)]  # (domain, bus, numa node)


def fake_sys(root):
    kfd = root / "class/kfd/kfd/topology/nodes"
    n = 0
    for sock in (0, 1):  # a CPU node per socket, then its two GPUs
        (kfd / str(n)).mkdir(parents=True)
        (kfd / str(n) / "properties").write_text("cpu_cores_count 4\nsimd_count 0\n")
        n += 1
        for dom, bus, node in GPUS:
            if node != sock:
                continue
            (kfd / str(n)).mkdir(parents=True)
            (kfd / str(n) / "properties").write_text(
                f"cpu_cores_count 0\nsimd_count 1024\ndomain {dom}\nlocation_id {bus << 8}\n")
            n += 1
    for dom, bus, node in GPUS:
        d = root / f"bus/pci/devices/{dom:04x}:{bus:02x}:00.0"
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{node}\n")
    for node, cpus in ((0, "0-3"), (1, "4-5,6-7")):
        d = root / f"devices/system/node/node{node}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpus + "\n")
    return str(root)


def test_topology_order_and_nodes(tmp_path):
    sysr = fake_sys(tmp_path)
    assert numa.kfd_gpu_bdfs(sysr) == ["0000:10:00.0", "0000:20:00.0", "0000:90:00.0",
                                       "0000:a0:00.0"]
    assert [numa.gpu_numa_node(d, sysr, env={}) for d in range(4)] == [0, 0, 1, 1]
    assert numa.gpu_numa_node(4, sysr, env={}) == -1
    # visible devices renumber: HIP device 0 is physical GPU 3
    env = {"HIP_VISIBLE_DEVICES": "3,0"}
    assert numa.visible_order(4, env) == [3, 0]
    assert [numa.gpu_numa_node(d, sysr, env=env) for d in range(2)] == [1, 0]
    assert numa.node_cpus(1, sysr) == [4, 5, 6, 7]
    assert numa.parse_cpulist("0-2, 5,7-8") == [0, 1, 2, 5, 7, 8]
    assert numa.kfd_gpu_bdfs(str(tmp_path / "nowhere")) == []


def test_bind_process(tmp_path, capfd):
    sysr = fake_sys(tmp_path)
    before = os.sched_getaffinity(0)
    try:
        p = numa.bind_to_gpu(2, sysr, env={"LOCUST_LOG": "info"})
        assert p["node"] == 1
        want = {4, 5, 6, 7} & before
        if want:
            assert p["bound"] and os.sched_getaffinity(0) == want
        assert "NUMA node 1" in capfd.readouterr().err
        off = numa.bind_to_gpu(2, sysr, env={"LOCUST_NUMA": "0"})
        assert off["node"] == -1 and not off["bound"]
    finally:
        os.sched_setaffinity(0, before)


def test_cpp_placement(tmp_path):
    sysr = fake_sys(tmp_path)
    assert lc._C.gpu_placement("0000:A0:00.0", sysr) == ("0000:a0:00.0", 1, [4, 5, 6, 7])
    assert lc._C.gpu_placement("0000:10:00.0", sysr) == ("0000:10:00.0", 0, [0, 1, 2, 3])
    assert lc._C.gpu_placement("0000:ff:00.0", sysr)[1] == -1
    assert lc._C.parse_cpulist("1-3,9") == [1, 2, 3, 9]
    assert lc._C.parse_cpulist("x") == []
