"""Randomised differential tests: seeded random byte texts -- delimiters, digits, letters,
'\\r', embedded NULs, bytes >= 0x80, over-long tokens, lines past the 20-emit cap, empty
lines -- through every engine path, against the independent Python oracle.  The CPU
engine is checked here on every run; the GPU paths (lean dictionary job, radix path,
reference-layout map, stage-split and graph modes) on the GPU box."""
import random

import pytest

import locust_amd as lc
from locust_amd.utils import oracle

LETTERS = b"abcdefghijklmnopqrstuvwxyzABCDEFGH0123456789"
DELIMS = b" ,.-;:'()\"\t"
ODD = b"\r\x00\x80\xc3\xa9\xff\x7f"


def random_text(rng: random.Random, size: int, fresh: float = 0.4) -> bytes:
    """fresh: share of words drawn at random (the rest from a 300-word vocabulary)."""
    out = bytearray()
    while len(out) < size:
        r = rng.random()
        if r < 0.06:
            out += b"\n"
        elif r < 0.30:
            out += bytes([rng.choice(DELIMS)]) * rng.randint(1, 3)
        elif r < 0.33:
            out += bytes([rng.choice(ODD)])
        elif r < 0.35:  # an over-long token (truncated at the key width)
            out += bytes(rng.choice(LETTERS) for _ in range(rng.randint(30, 80)))
        elif r < 0.37:  # a long line: more than 20 tokens
            out += b" ".join(bytes([rng.choice(LETTERS)]) * rng.randint(1, 3)
                             for _ in range(rng.randint(21, 60)))
        else:  # a word from a small vocabulary (repeats) or a random one
            if rng.random() >= fresh:
                out += b"w%d" % rng.randint(0, 300)
            else:
                out += bytes(rng.choice(LETTERS) for _ in range(rng.randint(1, 12)))
    return bytes(out[:size])


SIZES = [1, 2, 17, 300, 4095, 4096, 4097, 65536, 200_000]


def cases(n_seeds):
    for seed in range(n_seeds):
        rng = random.Random(1000 + seed)
        for size in SIZES:
            yield seed, size, random_text(rng, size)


@pytest.mark.parametrize("seed", range(4))
def test_cpu_engine_matches_oracle(seed):
    rng = random.Random(1000 + seed)
    for size in SIZES[:-1]:
        text = random_text(rng, size)
        ent, ntok, _ = oracle.wordcount(text)
        r = lc.wordcount_text(text, backend="cpu")
        assert r.num_tokens == ntok, (seed, size)
        assert r.entries() == ent, (seed, size)


GPU_PATHS = [
    dict(),                                           # lean dictionary job
    dict(graph=0),                                    # stage events
    dict(graph=1),                                    # graph replay
    dict(sort="radix"),                               # the reference's algorithm
    dict(sort="radix", reduce_path="global"),
    dict(map_path="compat", sort="dict"),             # the reference's map layout
]


@pytest.mark.gpu
@pytest.mark.parametrize("opts", GPU_PATHS, ids=lambda o: "-".join(f"{k}={v}" for k, v in o.items()) or "default")
def test_gpu_paths_match_oracle(opts):
    for seed, size, text in cases(3):
        ent, ntok, _ = oracle.wordcount(text)
        r = lc.wordcount_text(text, backend="gpu", check=True, **opts)
        assert r.num_tokens == ntok, (seed, size, opts)
        assert r.entries() == ent, (seed, size, opts)


@pytest.mark.gpu
def test_gpu_engine_reused_across_random_texts():
    """One engine, many different texts back to back (buffer pool, self-cleaning scratch,
    partition-map retunes between unrelated inputs)."""
    rng = random.Random(77)
    eng = lc._C.GpuEngine(lc.make_config("gpu", check=True), 300_000, 300_000)
    for _ in range(30):
        text = random_text(rng, rng.choice([100, 5000, 60_000, 250_000]))
        assert eng.run(text).entries() == oracle.wordcount(text)[0]


@pytest.mark.gpu
def test_gpu_large_random_pass_matches_cpu_engine():
    """A ~12 MB random text with a bounded vocabulary: upload pieces, per-piece partials and
    the two-kernel ordered build (first job on the default partition map, then retuned),
    against the CPU engine (itself checked against the oracle above)."""
    rng = random.Random(5)
    parts, size = [], 0
    while size < 12 << 20:
        chunk = random_text(rng, 256 << 10, fresh=0.002)
        chunk = chunk[: chunk.rfind(b"\n") + 1] or b"x\n"
        parts.append(chunk)
        size += len(chunk)
    text = b"".join(parts)
    want = lc._C.cpu_run(lc.make_config("cpu"), text).entries()
    eng = lc._C.GpuEngine(lc.make_config("gpu", check=True), len(text), text.count(b"\n") + 1)
    for _ in range(3):
        assert eng.run(text).entries() == want
    # the same through the distributed shuffle on one RCCL rank (asynchronous map)
    dcfg = lc.make_dist_config(1, lc.make_config("gpu", combine=True), strategy="shuffle")
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dr = lc._C.DistRank(dcfg, 0, "rccl", "127.0.0.1", port, len(text), text.count(b"\n") + 1,
                        60.0)
    for _ in range(3):
        res, _info = dr.run(text, 0)
        assert res.entries() == want
