"""`./MapReduce` on odd files, every execution mode, against the pure-Python oracle: empty
and newline-only files, no final newline, delimiter-only text, embedded NULs, CRLF, one
long line, every byte value, over-long keys -- through the single engine, the radix path
(both reduce paths), the thread-per-line map, loopback ranks (both strategies), the
streamed engine and the stage split (byte windows + a reduce).  The
same files run through the CPU backend in the CPU suite (the sweep's own check)."""
import os
import subprocess

import pytest

from locust_amd.utils import oracle

FILES = {
    "empty": b"",
    "newlines": b"\n\n\n",
    "no_final_newline": b"alpha beta\ngamma alpha",
    "delims_only": b" ,.-;:'()\"\t\n" * 50,
    "nuls": b"ab\0cd ef\nx\0\0y z\n\0\nlast line\0tail",
    "crlf": b"a b\r\nc d\r\na\r\n",
    "long_line": b" ".join(b"w%d" % (i % 97) for i in range(60000)),
    "all_bytes": bytes(range(256)) * 40 + b"\n",
    "long_keys": b"x" * 100 + b" " + b"y" * 29 + b" " + b"z" * 30 + b"\n" + b"x" * 100 + b"\n",
    "many_tokens": b"a b c d e f g h i j k l m n o p q r s t u v w x y z\n" * 500,
}


def _entries(out: bytes):
    ent = []
    for l in out.split(b"\n"):
        if l.startswith(b"print key: "):
            head, rest = l[len(b"print key: "):].rsplit(b" \t val: ", 1)
            v, c = rest.split(b" \t count: ")
            ent.append((head, int(v), int(c)))
    return ent


def _run(cli, *args):
    # --output-format gpu: result lines with val whichever backend ran
    p = subprocess.run([cli, *map(str, args), "--output-format", "gpu"], capture_output=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr.decode(errors="replace")[-2000:]
    return p.stdout


def _modes(backend):
    yield "single", []
    if backend == "gpu":
        yield "radix", ["--sort", "radix"]
        yield "radix_global", ["--sort", "radix", "--reduce-path", "global"]
        yield "compat_map", ["--map-path", "compat"]
        yield "loopback3", ["--gpus", 3, "--comm", "loopback"]
        yield "loopback2_gather", ["--gpus", 2, "--comm", "loopback", "--strategy", "gather"]
        yield "loopback2_shuffle", ["--gpus", 2, "--comm", "loopback", "--strategy", "shuffle"]
        yield "streamed", ["--chunk-mb", 1]


def _sweep(cli, tmp_path, backend):
    for name, text in FILES.items():
        f = tmp_path / f"{name}.txt"
        f.write_bytes(text)
        want = oracle.wordcount(text)[0]
        for mode, extra in _modes(backend):
            out = _run(cli, f, "--backend", backend, *extra)
            assert _entries(out) == want, (name, mode)
        # the stage split: two byte windows, each moved to a line start, then one reduce
        half = len(text) // 2
        spills = tmp_path / f"{name}_spills"
        spills.mkdir()
        for node, rng in enumerate((f"0:{half}", f"{half}:")):
            _run(cli, f, 0, 0, node, 1, "--byte-range", rng, "--spill-dir", spills,
                 "--spill-format", "binary", "--backend", backend)
        inputs = ",".join(str(spills / f"out.{k}.kv") for k in range(2))
        out = _run(cli, f, 0, 0, 0, 2, "--inputs", inputs, "--backend", backend)
        assert _entries(out) == want, (name, "stage split")


def test_odd_files_cpu_backend(cli, tmp_path):
    _sweep(cli, tmp_path, "cpu")


@pytest.mark.gpu
def test_odd_files_every_gpu_mode(cli, tmp_path):
    _sweep(cli, tmp_path, "gpu")
