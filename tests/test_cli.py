"""`./MapReduce` CLI: reference positional arguments and byte-compatible stdout."""
import os
import subprocess

from locust_amd.utils import oracle


def run(cli, *args, check=True):
    p = subprocess.run([cli, *map(str, args)], capture_output=True)
    if check:
        assert p.returncode == 0, p.stderr.decode()
    return p


def result_lines(out: bytes) -> bytes:
    return b"".join(l + b"\n" for l in out.split(b"\n") if l.startswith(b"print key:"))


def test_usage(cli):
    p = run(cli, check=False)
    assert p.returncode == 255
    assert p.stdout == (b"Running\nMissing or invalid arguments.\n"
                        b"mapreduce <filename> [line_start] [line_end] [node_num] [stage]\n")


def test_cpu_window_output(cli, hamlet):
    p = run(cli, "data/hamlet.txt", 0, 700, "--backend", "cpu")
    lines = p.stdout.split(b"\n")
    assert lines[0] == b"Running"
    assert lines[1] == b"Using custom start and end locations: (0, 700)"
    assert lines[2].startswith(b"CPU mapping ") and lines[2].endswith(b" nanoseconds ")
    entries = oracle.wordcount(oracle.window(hamlet, 0, 700))[0]
    assert result_lines(p.stdout) == oracle.format_cpu(entries)
    assert p.stdout.endswith(b"\nDone\n")


def test_stage_split_cpu(cli, hamlet, tmp_path):
    for node, (s, e) in enumerate([(0, 2000), (2000, 4463)]):
        p = run(cli, "data/hamlet.txt", s, e, node, 1, "--backend", "cpu", "--spill-dir", tmp_path)
        assert b"MODE_MULTI: Finished map" in p.stdout
    files = f"{tmp_path}/out.0.txt,{tmp_path}/out.1.txt"
    p = run(cli, "data/hamlet.txt", 0, 0, 0, 2, "--backend", "cpu", "--inputs", files)
    entries = oracle.wordcount(hamlet)[0]
    assert result_lines(p.stdout) == oracle.format_cpu(entries)


def test_spill_text_format(cli, tmp_path):
    (tmp_path / "in.txt").write_bytes(b"b a b\n")
    run(cli, tmp_path / "in.txt", 0, 1, 3, 1, "--backend", "cpu", "--spill-dir", tmp_path)
    # the reference writer's format "%s \t%d\n" (main.cu:121), combined: one line per key
    assert (tmp_path / "out.3.txt").read_bytes() == b"a \t1\nb \t2\n"
    # --ref-compat: the reference's own spill, one line per token, sorted (the CPU build
    # loads the whole file and drops its last line, B1)
    (tmp_path / "in.txt").write_bytes(b"b a b\nlast\n")
    run(cli, tmp_path / "in.txt", 0, 1, 4, 1, "--backend", "cpu", "--spill-dir", tmp_path,
        "--ref-compat")
    assert (tmp_path / "out.4.txt").read_bytes() == b"a \t1\nb \t1\nb \t1\n"


def test_multi_rank_cpu_cli(cli, hamlet):
    # --gpus N is the multi-GPU mode: GPU-format lines (val) whatever engine the ranks run
    # (docs/PARITY.md C18); --output-format picks either format in any mode
    p = run(cli, "data/hamlet.txt", "--backend", "cpu", "--gpus", 4)
    entries = oracle.wordcount(hamlet)[0]
    assert result_lines(p.stdout) == oracle.format_gpu(entries)
    p = run(cli, "data/hamlet.txt", "--backend", "cpu", "--gpus", 2, "--output-format", "cpu")
    assert result_lines(p.stdout) == oracle.format_cpu(entries)
    p = run(cli, "data/hamlet.txt", "--backend", "cpu", "--output-format", "gpu")
    assert result_lines(p.stdout) == oracle.format_gpu(entries)
    assert run(cli, "x", "--output-format", "tsv", check=False).returncode == 2


def test_json_in_every_mode(tmp_path, cli):
    """--json writes one record in every CLI mode (VERDICT r2 missing #3): the full job,
    the map and reduce stages, and --gpus N with every rank's stage times and the bytes
    each of its links carried."""
    import json
    import subprocess

    hamlet = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "hamlet.txt")
    def run(*args):
        j = tmp_path / "r.json"
        p = subprocess.run([cli, hamlet, *args, "--backend", "cpu", "--quiet", "--json", str(j)],
                           capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, p.stderr
        return json.loads(j.read_text())
    full = run()
    assert full["mode"] == "full" and full["unique"] == 5608 and full["tokens"] == 32940
    m = run("0", "700", "0", "1", "--spill-dir", str(tmp_path))
    assert m["mode"] == "map_stage" and m["tokens"] == 4896 and m["spill_records"] == 1566
    assert m["combined"] is True and m["lines"] == 700
    r = run("0", "0", "0", "2", "--spill-dir", str(tmp_path))
    assert r["mode"] == "reduce_stage" and r["unique"] == 1566 and r["input_records"] == 1566
    assert r["tokens"] == 4896 and r["indexed_files"] == 1
    d = run("--gpus", "3")
    assert d["mode"] == "multi_gpu" and d["unique"] == 5608 and len(d["ranks"]) == 3
    assert d["comm"] == "loopback" and d["pinned_bytes"] == 0  # CPU ranks pin nothing
    for k, rk in enumerate(d["ranks"]):
        assert rk["rank"] == k and len(rk["sent_to"]) == 3 and rk["sent_to"][k] == 0
        assert rk["sent_bytes"] == sum(rk["sent_to"]) and rk["recv_bytes"] == sum(rk["recv_from"])
    # what rank p sent to q is what q received from p
    for p_ in range(3):
        for q in range(3):
            assert d["ranks"][p_]["sent_to"][q] == d["ranks"][q]["recv_from"][p_]


def test_library_does_not_link_rccl():
    """RCCL is dlopen'ed on first use (csrc/comm/rccl_comm.hip): neither liblocust.so nor
    the CLI lists it among the libraries the dynamic loader maps at start (DT_NEEDED)."""
    import shutil
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    readelf = shutil.which("readelf") or "/opt/rocm/lib/llvm/bin/llvm-readelf"
    for f in ("locust_amd/_lib/liblocust.so", "build/MapReduce"):
        out = subprocess.run([readelf, "-d", os.path.join(root, f)], capture_output=True,
                             text=True, timeout=60).stdout
        needed = [ln for ln in out.splitlines() if "NEEDED" in ln]
        assert needed, out
        assert not any("rccl" in ln for ln in needed), needed
