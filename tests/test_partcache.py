"""The one-shot CLI's per-file partition-map cache (io.hpp): the map a run tuned is kept
under a key of the input file's identity and the tokenizer settings, so the next
`./MapReduce <file>` starts tuned.  A load-balancing hint only: the output never depends
on it (the GPU test runs the CLI twice and compares)."""
import os
import time

import pytest

import locust_amd as lc


def test_cache_key_follows_the_file_and_settings(tmp_path, monkeypatch):
    monkeypatch.setenv("LOCUST_CACHE_DIR", str(tmp_path / "c"))
    monkeypatch.delenv("LOCUST_PART_CACHE", raising=False)
    f = tmp_path / "a.txt"
    f.write_bytes(b"a b c\n")
    cfg = lc.make_config("gpu")
    p1 = lc._C.partmap_cache_path(str(f), cfg)
    assert p1.startswith(str(tmp_path / "c") + "/partmap-") and p1.endswith(".bin")
    assert lc._C.partmap_cache_path(str(f), cfg) == p1  # stable
    assert lc._C.partmap_cache_path(str(f), lc.make_config("gpu", emits_per_line=5)) != p1
    time.sleep(0.01)
    f.write_bytes(b"a b c d\n")  # new size and mtime: a new key
    assert lc._C.partmap_cache_path(str(f), cfg) != p1
    assert lc._C.partmap_cache_path(str(tmp_path / "missing.txt"), cfg) == ""
    monkeypatch.setenv("LOCUST_PART_CACHE", "0")
    assert lc._C.partmap_cache_path(str(f), cfg) == ""


def test_cache_round_trip_and_damage(tmp_path):
    p = str(tmp_path / "d" / "e" / "partmap-1.bin")  # directories made on save
    lo = [0] + [i << 40 for i in range(1, 256)] + [(1 << 64) - 1]
    lc._C.save_partmap_cache(p, lo)
    assert lc._C.load_partmap_cache(p) == lo
    assert not [x for x in os.listdir(os.path.dirname(p)) if x.endswith(".tmp")]
    assert lc._C.load_partmap_cache(str(tmp_path / "none.bin")) is None
    with open(p, "r+b") as f:  # truncated / wrong magic: refused
        f.truncate(100)
    assert lc._C.load_partmap_cache(p) is None
    with open(p, "wb") as f:
        f.write(b"XXXXXXXX" + bytes(4 + 257 * 8))
    assert lc._C.load_partmap_cache(p) is None
    lc._C.save_partmap_cache(p, lo[:10])  # wrong length: not written
    assert lc._C.load_partmap_cache(p) is None


@pytest.mark.gpu
def test_engine_refuses_a_malformed_map():
    text = open(os.path.join(lc.REPO_ROOT, "data", "hamlet.txt"), "rb").read()
    from locust_amd.utils import oracle

    eng = lc._C.GpuEngine(lc.make_config("gpu"), len(text), 5000)
    eng.load(text)
    assert not eng.set_partition_map([0, 5, 3] + [7] * 254)  # not ascending
    assert not eng.set_partition_map([1] * 257)               # lo[0] != 0
    # any ascending map is correct, however unbalanced: everything in partition 255
    assert eng.set_partition_map([0] * 256 + [(1 << 64) - 1])
    assert eng.run_loaded().entries() == oracle.wordcount(text)[0]
