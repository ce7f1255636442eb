"""`./MapReduce` on the GPU: the reference's minimum slice end to end --
positional CLI, stdout protocol (main.cu:358-532: `Running`, `Using custom start and end
locations`, `Length:`, `GPU mapping|stream compaction and sorting|reduce ... nanoseconds`,
`print key: %s \\t val: %d \\t count: %d`, `Done`), both reduce paths, the stage split on
the GPU and the in-process multi-rank mode (`--gpus N`: an RCCL clique when the node has
N GPUs, loopback ranks otherwise)."""
import os
import re
import subprocess

import pytest

from locust_amd.utils import oracle

pytestmark = pytest.mark.gpu


def run(cli, *args):
    p = subprocess.run([cli, *map(str, args)], capture_output=True, timeout=120)
    assert p.returncode == 0, p.stderr.decode()
    return p


def result_lines(out: bytes) -> bytes:
    return b"".join(l + b"\n" for l in out.split(b"\n") if l.startswith(b"print key:"))


def check_protocol(out: bytes, text: bytes, window=None):
    lines = out.split(b"\n")
    assert lines[0] == b"Running"
    i = 1
    if window:
        assert lines[i] == b"Using custom start and end locations: (%d, %d)" % window
        i += 1
    nlines = len(oracle.split_lines(text))
    assert lines[i] == b"Length: %d" % nlines
    stages = [l for l in lines if l.startswith(b"GPU ")]
    assert [re.sub(rb"\d+", b"N", l) for l in stages] == [
        b"GPU mapping N nanoseconds ", b"GPU stream compaction and sorting N nanoseconds ",
        b"GPU reduce N nanoseconds "]
    entries = oracle.wordcount(text)[0]
    assert result_lines(out) == oracle.format_gpu(entries)
    assert out.endswith(b"\nDone\n")


@pytest.mark.parametrize("extra", [[], ["--sort", "radix", "--reduce-path", "lds"],
                                   ["--sort", "radix", "--reduce-path", "global"],
                                   ["--map-path", "compat"]],
                         ids=["default", "radix-lds", "radix-global", "compat"])
def test_window_0_700(cli, hamlet, extra):
    p = run(cli, "data/hamlet.txt", 0, 700, *extra)
    check_protocol(p.stdout, oracle.window(hamlet, 0, 700), window=(0, 700))
    d = {k: c for k, _v, c in oracle.wordcount(oracle.window(hamlet, 0, 700))[0]}
    assert d[b"the"] == 143 and len(d) == 1566


@pytest.mark.parametrize("extra", [[], ["--reduce-path", "global", "--sort", "radix"]],
                         ids=["default", "radix-global"])
def test_whole_file(cli, hamlet, extra):
    p = run(cli, "data/hamlet.txt", *extra)
    check_protocol(p.stdout, hamlet)
    assert p.stdout.count(b"print key:") == 5608


def test_ref_compat_and_ref_timers(cli, hamlet):
    p = run(cli, "data/hamlet.txt", "--ref-compat", "--ref-timers")
    text = oracle.window(hamlet, ref_compat=True)
    check_protocol(p.stdout, text)
    assert b"print key: THE \t val: " in p.stdout and p.stdout.count(b"print key:") == 5607


def test_stage_split_gpu(cli, hamlet, tmp_path):
    for node, (s, e) in enumerate([(0, 1500), (1500, 3000), (3000, 4463)]):
        p = run(cli, "data/hamlet.txt", s, e, node, 1, "--spill-dir", tmp_path)
        assert b"MODE_MULTI: Finished map" in p.stdout
    files = ",".join(f"{tmp_path}/out.{k}.txt" for k in range(3))
    p = run(cli, "data/hamlet.txt", 0, 0, 0, 2, "--inputs", files)
    assert result_lines(p.stdout) == oracle.format_gpu(oracle.wordcount(hamlet)[0])


def test_stage_split_gpu_binary(cli, hamlet, tmp_path):
    for node, (s, e) in enumerate([(0, 2200), (2200, 4463)]):
        run(cli, "data/hamlet.txt", s, e, node, 1, "--spill-dir", tmp_path,
            "--spill-format", "binary")
    files = ",".join(f"{tmp_path}/out.{k}.kv" for k in range(2))
    p = run(cli, "data/hamlet.txt", 0, 0, 0, 2, "--inputs", files)
    assert result_lines(p.stdout) == oracle.format_gpu(oracle.wordcount(hamlet)[0])


@pytest.mark.parametrize("gpus,comm", [(1, "auto"), (1, "rccl"), (2, "auto"), (3, "loopback")])
def test_multi_rank_gpu_cli(cli, hamlet, gpus, comm):
    """--comm rccl: an ncclCommInitAll clique (one rank per GPU); auto (the default until a
    run with real RCCL peers is on record) and loopback: ranks as threads, collectives as
    device copies -- more ranks than GPUs share a device.  Output byte-identical to one GPU
    incl. `val`."""
    p = subprocess.run([cli, "data/hamlet.txt", "--gpus", str(gpus), "--comm", comm],
                       capture_output=True, timeout=120, env={**__import__("os").environ,
                                                              "LOCUST_LOG": "info"})
    assert p.returncode == 0, p.stderr.decode()
    assert result_lines(p.stdout) == oracle.format_gpu(oracle.wordcount(hamlet)[0])
    want = b"RCCL clique" if comm == "rccl" else b"over loopback"
    assert want in p.stderr


def _parse_gpu_out(out: bytes):
    ent = []
    for l in out.split(b"\n"):
        if l.startswith(b"print key: "):
            k, v, c = re.match(rb"print key: (.*) \t val: (\d+) \t count: (\d+)$", l).groups()
            ent.append((k, int(v), int(c)))
    return ent


@pytest.mark.parametrize("mb,chunk_mb", [(320, 64), (200, 0)])
def test_file_read_direct_and_streamed(tmp_path, cli, mb, chunk_mb):
    """Generated files: 320 MB streamed through two pinned 64 MiB
    chunks read by parallel preads (host memory bounded: max RSS far below the file), and
    200 MB -- under the default 256 MiB pass -- read whole straight into the engine's
    pinned buffer; the output is the CPU engine's, protocol lines included."""
    import json

    import locust_amd as lc

    f = tmp_path / "big.txt"
    run(cli, "--gen", f, "--gen-bytes", mb << 20, "--seed", 5)
    j = tmp_path / "r.json"
    args = [f, "--json", j] + (["--chunk-mb", chunk_mb] if chunk_mb else [])
    p = run(cli, *args)
    text = f.read_bytes()
    want = lc._C.cpu_run(lc.make_config("cpu"), text)
    lines = p.stdout.split(b"\n")
    assert lines[0] == b"Running" and lines[1] == b"Length: %d" % want.num_lines
    assert _parse_gpu_out(p.stdout) == want.entries()
    rec = json.loads(j.read_text())
    assert rec["tokens"] == want.num_tokens and rec["unique"] == want.num_unique
    if chunk_mb:
        assert rec["chunks"] >= mb // chunk_mb
        # host memory bounded by the engine's buffers, not the file: peak RSS of this run is
        # bimodal between processes -- 0.93-0.94 or 1.13-1.19 GB, +186 MB of anonymous memory
        # outside the engine's pinned buffers, with either pinning path
        # (profiles/r6/rss/cli_320mb_chunk64_rss_by_pin_path.txt)
        assert rec["max_rss_kb"] < (5 << 20) // 4  # < 1.25 GiB


@pytest.mark.parametrize("gpus", [2, 4, 8])
def test_multi_rank_cli_first_job_on_device(tmp_path, cli, gpus):
    """the CLI runs ONE job per process, so its shuffle is always a
    first job.  It runs on the device -- the all-gathered plans size an exact all-to-all-v,
    every rank writes its key range into the shared host output -- with at most two host
    synchronisations per rank; the output is the CPU engine's, byte for byte."""
    import json

    import locust_amd as lc

    f = tmp_path / "synth.txt"
    run(cli, "--gen", f, "--gen-lines", 1_000_000, "--seed", 1)
    j = tmp_path / "r.json"
    p = run(cli, f, "--gpus", gpus, "--comm", "loopback", "--json", j)
    want = lc._C.cpu_run(lc.make_config("cpu"), f.read_bytes())
    assert _parse_gpu_out(p.stdout) == want.entries()
    rec = json.loads(j.read_text())
    assert rec["strategy"] == "shuffle" and len(rec["ranks"]) == gpus
    for rk in rec["ranks"]:
        assert rk["device_exchange"] is True and 1 <= rk["host_syncs"] <= 2, rk
        # compact records (kv.hpp): 8-40 B per key, counted by the merge as it emits
        assert 8 * rk["range_unique"] <= rk["output_bytes"] <= 40 * rk["range_unique"], rk
    assert sum(rk["range_unique"] for rk in rec["ranks"]) == want.num_unique
    assert sum(rk["output_bytes"] for rk in rec["ranks"]) == _compact_bytes(want.entries())
    # page-locked host memory per rank (its engine) and in all (plus the shared output)
    assert all(rk["pinned_bytes"] > 0 for rk in rec["ranks"])
    assert rec["pinned_bytes"] > sum(rk["pinned_bytes"] for rk in rec["ranks"])


def _compact_bytes(entries) -> int:
    """Bytes of the compact result records (kv.hpp compact_words) of (key, val, count)."""
    total = 0
    for key, _v, c in entries:
        kb = len(key)
        total += 8 * (1 + ((kb + 3) >> 3 if kb > 4 else 0) if c < (1 << 24) else 1 + ((kb + 7) >> 3))
    return total


@pytest.mark.gpu
def test_single_gpu_cli_never_loads_rccl(cli):
    """RCCL is dlopen'ed on first use (csrc/comm/rccl_comm.hip): a single-GPU job maps
    neither librccl nor its code objects.  LD_DEBUG=files lists every
    library the dynamic loader opens, including dlopen'ed ones."""
    env = dict(os.environ, LD_DEBUG="files")
    p = subprocess.run([cli, "data/hamlet.txt"], capture_output=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    assert b"Done" in p.stdout or b"print key" in p.stdout
    assert b"libamdhip64" in p.stderr  # LD_DEBUG did report the loads
    assert b"librccl" not in p.stderr
