"""Per-rank file shards: every rank of `MapReduce <file> --gpus N`
reads only its own line-aligned byte range of the file -- the reference's per-node line
ranges (/root/reference/MapReduce/src/main.cu:40-64, 369-374) as byte ranges -- straight
into its own pinned buffer, or streamed through a pinned ring past one device pass.  No
rank holds the whole file."""
import json
import os
import subprocess

import pytest

import locust_amd as lc
from locust_amd.utils import oracle


def _cuts_ok(data: bytes, shards):
    pos = 0
    for off, n in shards:
        assert off == pos
        if off and n:
            assert data[off - 1:off] == b"\n"  # a range starts at a line start
        pos += n
    assert pos == len(data)


@pytest.mark.parametrize("parts", [1, 2, 3, 7, 8, 64])
def test_file_shards_line_aligned(tmp_path, hamlet, parts):
    f = tmp_path / "h.txt"
    f.write_bytes(hamlet)
    sh = lc._C.file_shards(str(f), parts)
    assert len(sh) == parts
    _cuts_ok(hamlet, sh)
    # the same cuts as the in-memory shard_text
    assert [(o, n) for o, n, _l, _f in lc._C.shard_bounds(hamlet, parts)] == sh


@pytest.mark.parametrize("text", [b"", b"a", b"a b\n", b"x\n" * 3, b"long line " * 20000 + b"\nend",
                                  b"no newline at all " * 9000], ids=range(6))
def test_file_shards_edge_cases(tmp_path, text):
    f = tmp_path / "t.txt"
    f.write_bytes(text)
    for parts in (1, 2, 5, 16):
        _cuts_ok(text, lc._C.file_shards(str(f), parts))


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("tail", [True, False])
def test_cpu_ranks_read_own_ranges(tmp_path, hamlet, world, tail):
    text = hamlet if tail else hamlet.rstrip(b"\n")  # a final line without its newline
    f = tmp_path / "h.txt"
    f.write_bytes(text)
    dcfg = lc.make_dist_config(world, lc.make_config("cpu", combine=True))
    res, infos = lc._C.run_multi_file(str(f), dcfg, "loopback")
    assert res.entries() == oracle.wordcount(text)[0]
    assert res.num_lines == text.count(b"\n") + (0 if text.endswith(b"\n") else 1)
    assert [i["input_bytes"] for i in infos] == [n for _o, n in lc._C.file_shards(str(f), world)]
    assert all(i["peer_p2p"] == -1 for i in infos)  # CPU ranks: no GPU peers


def test_cli_cpu_ranks_file(cli, hamlet):
    p = subprocess.run([cli, "data/hamlet.txt", "--backend", "cpu", "--gpus", "3"],
                       capture_output=True, timeout=120)
    assert p.returncode == 0, p.stderr.decode()
    got = b"".join(l + b"\n" for l in p.stdout.split(b"\n") if l.startswith(b"print key:"))
    assert got == oracle.format_gpu(oracle.wordcount(hamlet)[0])


def _cpu_want(path):
    return lc._C.cpu_run(lc.make_config("cpu"), open(path, "rb").read())


@pytest.mark.gpu
@pytest.mark.parametrize("gpus,chunk_mb", [(1, 64), (2, 64), (4, 64), (2, 0), (3, 0)])
def test_gpu_ranks_file_shards(tmp_path, cli, gpus, chunk_mb):
    """A 320 MB generated file at --gpus 1/2/4 (loopback ranks on the test box's GPU): with
    --chunk-mb 64 every rank streams its 80-160 MB range through its pinned ring; without,
    every range fits one pass and is read straight into the rank's pinned buffer.  Output
    identical to the CPU engine; --json reports each rank's bytes."""
    from test_cli_gpu import _parse_gpu_out

    f = tmp_path / "big.txt"
    subprocess.run([cli, "--gen", str(f), "--gen-bytes", str(320 << 20), "--seed", "5"],
                   check=True, capture_output=True, timeout=120)
    j = tmp_path / "r.json"
    args = [cli, str(f), "--gpus", str(gpus), "--comm", "loopback", "--json", str(j)]
    if chunk_mb:
        args += ["--chunk-mb", str(chunk_mb)]
    p = subprocess.run(args, capture_output=True, timeout=180)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    want = _cpu_want(f)
    lines = p.stdout.split(b"\n")
    assert lines[0] == b"Running" and lines[1] == b"Length: %d" % want.num_lines
    assert _parse_gpu_out(p.stdout) == want.entries()
    rec = json.loads(j.read_text())
    assert sum(r["input_bytes"] for r in rec["ranks"]) == os.path.getsize(f)
    assert all(r["input_streamed"] == bool(chunk_mb) for r in rec["ranks"]), rec["ranks"]
    # streamed ranks hold their rings, never their ranges; one-pass ranks hold their own
    # range once each (the process baseline -- HIP runtime, code objects -- is ~0.5-1 GiB)
    size_kb = os.path.getsize(f) >> 10
    bound = (1 << 21) if chunk_mb else (1 << 21) + size_kb
    print(f"--gpus {gpus} chunk {chunk_mb} MB: peak RSS {rec['peak_rss_kb']} kB")
    assert rec["peak_rss_kb"] < bound
