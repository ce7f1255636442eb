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


# ---- page placement of the shared distributed output ----
def test_rank_slices_plan():
    # 4 ranks on two sockets (0, 0, 1, 1): per region, the first half of the pages on node 0
    # (ranks 0-1, merged), the second half on node 1; the header page with rank 0
    hdr, region = 4096, 1_000_000 * 40
    plan = lc._C.plan_rank_slices(hdr, region, 2, [0, 0, 1, 1])
    assert plan[0] == (0, 4096 + ((region // 2 + 4095) // 4096) * 4096, 0)
    pos = 0
    for off, n, node in plan:  # contiguous, page-aligned, alternating nodes
        assert off == pos and off % 4096 == 0 and n % 4096 == 0 and n > 0
        pos += n
    assert pos == ((hdr + 2 * region + 4095) // 4096) * 4096
    assert [node for _o, _n, node in plan] == [0, 1, 0, 1]
    # the seam of region 0 lies at its middle, rounded up to a page
    assert plan[1][0] == ((hdr + region // 2 + 4095) // 4096) * 4096
    # unknown nodes leave their slices to the default policy; one node: nothing to place
    assert [s[2] for s in lc._C.plan_rank_slices(hdr, region, 1, [0, -1, 1, 1])] == [0, 1]
    assert lc._C.spans_numa_nodes([0, 1]) and not lc._C.spans_numa_nodes([0, 0, -1])
    # eight ranks, one node each: slice p of every region on node p
    p8 = lc._C.plan_rank_slices(hdr, 8 * 4096 * 10, 3, list(range(8)))
    assert [s[2] for s in p8] == [0] + list(range(1, 8)) + list(range(8)) * 2


def test_shm_segment_placed_before_reserve():
    """The plan is applied to the mapping before posix_fallocate reserves the pages (shmem
    keeps it as the object's policy): every page lands on its slice's node.  This box has
    node 0 only, so the plan binds everything there and a slice naming an absent node is
    logged and skipped, not fatal.  (A child process: the log level is read once.)"""
    import subprocess
    import sys

    code = ("import locust_amd as lc\n"
            "print(lc._C.shm_placement_probe(64 * 4096, [(0, 32 * 4096, 0), (32 * 4096, 32 * 4096, 0)]))\n"
            "print(len(lc._C.shm_placement_probe(8 * 4096, [(0, 8 * 4096, 1000)])))\n")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, LOCUST_LOG="info"))
    assert p.returncode == 0, p.stderr
    out = p.stdout.splitlines()
    assert out[0] == str([0] * 64) and out[1] == "8"
    assert "preferred on NUMA node 0" in p.stderr
    assert "to NUMA node 1000 failed" in p.stderr


def test_rank_slices_from_fake_sysfs(tmp_path):
    """The shared output's placement end to end on the fake two-socket tree: each rank's
    node comes from its GPU's PCI address (placement_for_bdf, what GpuShardEngine::numa_node
    reads), and the plan puts every rank's slice of every region on that node."""
    sysr = fake_sys(tmp_path)
    bdfs = [f"{dom:04x}:{bus:02x}:00.0" for dom, bus, _node in GPUS]
    nodes = [lc._C.gpu_placement(b, sysr)[1] for b in bdfs]
    assert nodes == [0, 0, 1, 1]
    region = 4 * 4096 * 64
    plan = lc._C.plan_rank_slices(4096, region, 3, nodes)
    for k in range(3):  # per region: ranks 0-1 (node 0), then ranks 2-3 (node 1)
        base = 4096 + k * region
        for r, node in enumerate(nodes):
            lo = base + region * r // 4
            hit = [n for off, ln, n in plan if off <= lo < off + ln]
            assert hit == [node], (k, r, plan)
