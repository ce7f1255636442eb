"""The reference's stage split (map -> spill files -> reduce; /root/reference/MapReduce/src/
main.cu:421-446), count-carrying: stage 1 spills one (key, count) record per distinct key
with a sparse index, stage 2 merges the spills as sorted runs (never expanding a count into
tokens), and R key-range reducers each write their slice with its global val
(README.md:24-29, the GIF's reducers)."""
import json
import os
import random
import subprocess
import time

import pytest

import locust_amd as lc
from locust_amd.utils import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(cli, *args, check=True, **kw):
    p = subprocess.run([cli, *map(str, args)], capture_output=True, timeout=300, **kw)
    if check:
        assert p.returncode == 0, p.stderr.decode()[-3000:]
    return p


def result_lines(out: bytes) -> bytes:
    return b"".join(l + b"\n" for l in out.split(b"\n") if l.startswith(b"print key:"))


# ------------------------------------------------------------------------------------
# line windows (stage 1 reads its window straight from the file)
# ------------------------------------------------------------------------------------
@pytest.mark.parametrize("tail", [b"\n", b""])
def test_line_window_matches_loader(tmp_path, tail):
    rng = random.Random(5)
    lines = [b"w" * rng.randrange(0, 40) + b" x" for _ in range(3000)]
    text = b"\n".join(lines) + tail
    f = tmp_path / "t.txt"
    f.write_bytes(text)
    nl = text.count(b"\n") + (0 if text.endswith(b"\n") else 1)
    cases = [(0, 0), (0, 1), (0, nl), (0, nl + 5), (1, 2), (nl - 1, nl), (nl, nl + 1),
             (nl + 3, nl + 9), (17, 17), (5, -1), (0, -1), (nl - 1, -1)]
    cases += [tuple(sorted(rng.sample(range(nl + 2), 2))) for _ in range(20)]
    for s, e in cases:
        b, end, n = lc._C.find_line_window(str(f), s, e)
        want = oracle.window(text, s, e if e >= 0 else nl + 1)  # lines, each with its '\n'
        got = text[b:end]
        assert got + (b"\n" if got and not got.endswith(b"\n") else b"") == want, (s, e)
        assert n == want.count(b"\n"), (s, e)


# ------------------------------------------------------------------------------------
# stage 1: combined spill + index
# ------------------------------------------------------------------------------------
@pytest.mark.parametrize("fmt", ["text", "binary", "kiv"])
def test_combined_spill_and_index(cli, hamlet, tmp_path, fmt):
    run(cli, "data/hamlet.txt", 0, 700, 0, 1, "--backend", "cpu", "--spill-dir", tmp_path,
        "--spill-format", fmt, cwd=ROOT)
    ext = {"text": "txt", "binary": "kv", "kiv": "kiv"}[fmt]
    spill = str(tmp_path / f"out.0.{ext}")
    recs = lc._C.read_spill(spill)
    ent, ntok, _ = oracle.wordcount(oracle.window(hamlet, 0, 700))
    assert recs == [(k, c) for k, _v, c in ent]  # one record per distinct key, key order
    idx = lc._C.spill_index(spill)
    assert idx["sorted"] and idx["distinct"] and idx["records"] == len(ent)
    assert idx["total_count"] == ntok and idx["spill_bytes"] == os.path.getsize(spill)
    # every sample: the key of its record and the exact count before it
    cum = [0]
    for _k, c in recs:
        cum.append(cum[-1] + c)
    for key, rec, _off, before in idx["samples"]:
        assert recs[rec][0] == key and cum[rec] == before
    # a spill rewritten after its index: the stale index is ignored
    with open(spill, "ab") as f:
        f.write(b"zzz \t1\n" if fmt == "text" else b"")
    if fmt == "text":
        assert lc._C.spill_index(spill) is None


def test_synth_spill_is_combined(cli, tmp_path):
    """Stage 1 of a synthetic file: the spill holds the distinct keys, not the tokens
    (round 4's token spill of synth1m was 252 MB for a 43 MB input)."""
    f = tmp_path / "s.txt"
    run(cli, "--gen", f, "--gen-lines", 100_000, "--seed", 1)
    j = tmp_path / "m.json"
    run(cli, f, 0, 100_000, 0, 1, "--backend", "cpu", "--spill-dir", tmp_path, "--spill-format",
        "binary", "--json", j)
    m = json.load(open(j))
    assert m["spill_records"] == m["unique"] and m["tokens"] > 5 * m["unique"]
    assert m["spill_bytes"] == 32 + 40 * m["unique"]


# ------------------------------------------------------------------------------------
# stage 2: merge of sorted runs, key-range reducers
# ------------------------------------------------------------------------------------
def _map_windows(cli, tmp_path, windows, backend="cpu", fmts=("text", "binary", "kiv"),
                 extra=()):
    files = []
    for k, (s, e) in enumerate(windows):
        fmt = fmts[k % len(fmts)]
        run(cli, "data/hamlet.txt", s, e, k, 1, "--backend", backend, "--spill-dir", tmp_path,
            "--spill-format", fmt, *extra, cwd=ROOT)
        files.append(str(tmp_path / f"out.{k}.{ {'text': 'txt', 'binary': 'kv', 'kiv': 'kiv'}[fmt] }"))
    return files


@pytest.mark.parametrize("reducers", [1, 2, 3, 5, 8])
def test_range_reducers_concatenate_to_single_stage(cli, hamlet, tmp_path, reducers):
    files = _map_windows(cli, tmp_path, [(0, 1500), (1500, 3000), (3000, 4463)])
    ent = oracle.wordcount(hamlet)[0]
    got = []
    for r in range(reducers):
        res, st = lc._C.reduce_spills(lc.make_config("cpu"), files, r, reducers)
        part = res.entries()
        assert st["indexed_files"] == 3 and st["loaded_files"] == 0
        if part:  # (key, val, count): val is global
            assert part[0][1] == sum(c for k, _v, c in ent if k < part[0][0])
        got += part
    assert got == ent


def test_range_reducers_cli_gpu_format(cli, hamlet, tmp_path):
    """--reducer r/R through the CLI, result lines to --result-file; the concatenation is
    the single-stage output including val (GPU-format lines carry val)."""
    files = _map_windows(cli, tmp_path, [(0, 2000), (2000, 4463)])
    out = b""
    for r in range(3):
        rf = tmp_path / f"res.{r}.txt"
        p = run(cli, "data/hamlet.txt", 0, 0, r, 2, "--backend", "cpu", "--inputs",
                ",".join(files), "--reducer", f"{r}/3", "--result-file", rf, cwd=ROOT)
        assert b"print key:" not in p.stdout and p.stdout.endswith(b"\nDone\n")
        out += rf.read_bytes()
    assert out == oracle.format_cpu(oracle.wordcount(hamlet)[0])
    kiv = b""
    for r in range(3):
        k = tmp_path / f"res.{r}.kiv"
        run(cli, "data/hamlet.txt", 0, 0, r, 2, "--backend", "cpu", "--inputs", ",".join(files),
            "--reducer", f"{r}/3", "--quiet", "--export-kiv", k, cwd=ROOT)
        kiv += b"".join(bytes(x[0]) + b"%d,%d;" % (x[1], x[2]) for x in lc._C.read_kiv(str(k)))
    want = b"".join(k + b"%d,%d;" % (v, c) for k, v, c in oracle.wordcount(hamlet)[0])
    assert kiv == want


def test_reduce_never_expands_counts(cli, tmp_path):
    """A 15-byte spill holding one key with count 300,000,000 (round 4: 69.5 s, 18.3 GB
    RSS, because stage 2 rebuilt one token per unit of count)."""
    f = tmp_path / "big.txt"
    f.write_bytes(b"the \t300000000\n")
    j = tmp_path / "r.json"
    t0 = time.perf_counter()
    p = run(cli, "x", 0, 0, 0, 2, "--backend", "cpu", "--inputs", f, "--json", j)
    dt = time.perf_counter() - t0
    assert result_lines(p.stdout) == b"print key: the \t value: 300000000\n"
    rec = json.load(open(j))
    assert rec["tokens"] == 300_000_000 and rec["input_records"] == 1
    assert dt < 2.0, dt  # ~15 ms measured (process start to exit)
    assert rec["peak_rss_kb"] < 100_000, rec  # ~12 MB measured


def test_unsorted_reference_spills(cli, hamlet, tmp_path):
    """Reference-format spills (one "key \\t1" line per token) that are NOT sorted, e.g. two
    mappers' files concatenated (the reference's reducer needs one pre-sorted file, B7)."""
    a, b = oracle.window(hamlet, 0, 2000), oracle.window(hamlet, 2000, 4463)
    lines = []
    for part in (a, b):
        for k, _v, c in oracle.wordcount(part)[0]:
            lines += [k + b" \t1\n"] * c
    random.Random(1).shuffle(lines)
    f = tmp_path / "mixed.txt"
    f.write_bytes(b"".join(lines))
    p = run(cli, "x", 0, 0, 0, 2, "--backend", "cpu", "--inputs", f)
    assert result_lines(p.stdout) == oracle.format_cpu(oracle.wordcount(hamlet)[0])
    res, st = lc._C.reduce_spills(lc.make_config("cpu"), [str(f)], 1, 2)
    assert st["loaded_files"] == 1
    lo = res.entries()
    assert lo and lo[0][1] == sum(c for k, _v, c in oracle.wordcount(hamlet)[0] if k < lo[0][0])


def test_ref_compat_token_spill_round_trip(cli, hamlet, tmp_path):
    """--ref-compat stage 1 writes the reference's per-token spill (sorted, not combined,
    indexed as such); stage 2 combines adjacent records while reading.  (The CPU build
    loads the whole file without its last line, B1: 32,938 tokens.)"""
    run(cli, "data/hamlet.txt", 0, 700, 0, 1, "--backend", "cpu", "--spill-dir", tmp_path,
        "--ref-compat", cwd=ROOT)
    spill = str(tmp_path / "out.0.txt")
    idx = lc._C.spill_index(spill)
    assert idx["sorted"] and not idx["distinct"] and idx["records"] == 32938
    for reducers in (1, 2):
        got = []
        for r in range(reducers):
            got += lc._C.reduce_spills(lc.make_config("cpu"), [spill], r, reducers)[0].entries()
        assert got == oracle.wordcount(oracle.window(hamlet, ref_compat=True))[0]


def test_stage2_finds_the_spill_format(cli, hamlet, tmp_path):
    run(cli, "data/hamlet.txt", 0, 700, 4, 1, "--backend", "cpu", "--spill-dir", tmp_path,
        "--spill-format", "binary", cwd=ROOT)
    # no --spill-format and no --inputs: out.4.txt is absent, out.4.kv is found
    p = run(cli, "data/hamlet.txt", 0, 0, 4, 2, "--backend", "cpu", "--spill-dir", tmp_path,
            cwd=ROOT)
    assert result_lines(p.stdout) == oracle.format_cpu(oracle.wordcount(oracle.window(hamlet, 0, 700))[0])


def test_many_spills_host_merge(hamlet, tmp_path):
    lines = hamlet.split(b"\n")
    files = []
    for k in range(70):  # more runs than one device merge launch takes
        part = b"\n".join(lines[k::70]) + b"\n"
        files.append(str(tmp_path / f"s{k}.kv"))
        lc._C.write_spill(files[-1], [(key, c) for key, _v, c in oracle.wordcount(part)[0]], "binary")
    res, st = lc._C.reduce_spills(lc.make_config("cpu"), files)
    assert st["loaded_files"] == 70
    whole = oracle.wordcount(b"\n".join(lines) + b"\n")[0]
    assert res.entries() == whole


def test_splitters_order_independent(cli, tmp_path):
    files = _map_windows(cli, tmp_path, [(0, 1000), (1000, 2500), (2500, 4463)])
    a = lc._C.reducer_splitters(files, 4)
    b = lc._C.reducer_splitters(files[::-1], 4)
    assert a == b and len(a) == 3 and a == sorted(a)


def test_help(cli):
    p = run(cli, "--help")
    assert p.stdout.startswith(b"usage: MapReduce <file>") and b"--reducer r/R" in p.stdout


# ------------------------------------------------------------------------------------
# GPU: stage 1 on the device (windows read in place, streamed past one pass), stage 2
# merged on the device
# ------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_gpu_stage_split_hamlet(cli, hamlet, tmp_path):
    files = _map_windows(cli, tmp_path, [(0, 1500), (1500, 3000), (3000, 4463)], backend="gpu")
    for k, f in enumerate(files):
        idx = lc._C.spill_index(f)
        assert idx is not None and idx["sorted"] and idx["distinct"], f
    ent = oracle.wordcount(hamlet)[0]
    p = run(cli, "data/hamlet.txt", 0, 0, 0, 2, "--inputs", ",".join(files), cwd=ROOT)
    assert result_lines(p.stdout) == oracle.format_gpu(ent)
    got = []
    for r in range(3):
        got += lc._C.reduce_spills(lc.make_config("gpu"), files, r, 3)[0].entries()
    assert got == ent


@pytest.mark.gpu
def test_gpu_stage1_streams_large_window(cli, tmp_path):
    """A window larger than one device pass (--chunk-mb 4) streams through the engine's
    pinned ring from the file; same spill as the CPU engine's."""
    f = tmp_path / "s.txt"
    run(cli, "--gen", f, "--gen-lines", 400_000, "--seed", 3)
    j = tmp_path / "m.json"
    run(cli, f, 50_000, 350_000, 0, 1, "--spill-dir", tmp_path, "--spill-format", "binary",
        "--chunk-mb", 4, "--json", j)
    m = json.load(open(j))
    assert m["streamed"] is True and m["lines"] == 300_000
    run(cli, f, 50_000, 350_000, 1, 1, "--backend", "cpu", "--spill-dir", tmp_path,
        "--spill-format", "binary")
    assert lc._C.read_spill(str(tmp_path / "out.0.kv")) == lc._C.read_spill(str(tmp_path / "out.1.kv"))


def test_python_stage_api(hamlet, tmp_path):
    """locust_amd.map_stage / reduce_stage: the stage split from Python."""
    f = tmp_path / "h.txt"
    f.write_bytes(hamlet)
    spills = []
    for k, (s, e) in enumerate([(0, 2000), (2000, 4463)]):
        spills.append(str(tmp_path / f"s{k}.kv"))
        m = lc.map_stage(str(f), spills[-1], s, e, backend="cpu")
        assert m["lines"] == e - s and m["spill_records"] == m["unique"]
    got = []
    for r in range(2):
        res, st = lc.reduce_stage(spills, r, 2, backend="cpu")
        got += res.entries()
    assert got == oracle.wordcount(hamlet)[0]
