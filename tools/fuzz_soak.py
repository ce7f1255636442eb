"""A longer randomized soak of the GPU paths than the test suite's (tests/test_fuzz.py runs
3 seeds per path): `--seeds` random byte texts per size (delimiter runs, NUL, CR, 0xFF,
lines up to 2,000 B, with and without a final newline) through every GPU path, fresh
engines and one reused engine, each result compared entry by entry with the pure-Python
oracle; then ~2 MB texts streamed through small chunks against the CPU engine, and
multi-rank jobs (loopback ranks on the GPU, both strategies) against the oracle.  Prints
one line per path and exits non-zero on the first mismatch.

    python tools/fuzz_soak.py [--seeds 30] [--out FILE]
"""
import argparse
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import locust_amd as lc  # noqa: E402
from locust_amd.utils import oracle  # noqa: E402
from test_fuzz import GPU_PATHS, SIZES, random_text  # noqa: E402

EXTRA_PATHS = [dict(zero_copy_text=1), dict(zero_copy_text=0)]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=30)
    ap.add_argument("--out")
    a = ap.parse_args()
    lines = []

    def say(s):
        lines.append(s)
        print(s, flush=True)

    texts = []
    for seed in range(a.seeds):
        rng = random.Random(5000 + seed)
        for size in SIZES:
            texts.append((seed, size, random_text(rng, size)))
    want = [oracle.wordcount(t) for _, _, t in texts]
    for opts in GPU_PATHS + EXTRA_PATHS:
        t0 = time.time()
        for (seed, size, text), (ent, ntok, _) in zip(texts, want):
            r = lc.wordcount_text(text, backend="gpu", check=True, **opts)
            if r.num_tokens != ntok or r.entries() != ent:
                say(f"MISMATCH path={opts} seed={seed} size={size}")
                return 1
        say(f"path {opts or 'default'}: {len(texts)} texts match the oracle ({time.time() - t0:.1f} s)")
    eng = lc._C.GpuEngine(lc.make_config("gpu", check=True), 300_000, 300_000)
    n = 0
    for (seed, size, text), (ent, _n, _) in zip(texts, want):
        if size > 300_000:
            continue
        if eng.run(text).entries() != ent:
            say(f"MISMATCH reused engine seed={seed} size={size}")
            return 1
        n += 1
    say(f"one reused engine: {n} texts back to back match the oracle")
    # streamed passes: ~2 MB random texts through engines with small chunks (line-aligned
    # chunk cuts, map windows, one dictionary across chunks), pageable and pinned input,
    # against the CPU engine (itself matched to the oracle by tests/test_fuzz.py)
    t0 = time.time()
    m = 0
    for seed in range(max(1, a.seeds // 10)):
        rng = random.Random(9000 + seed)
        parts, size = [], 0
        while size < 2 << 20:
            piece = random_text(rng, rng.choice([4096, 60_000, 200_000]))
            piece = piece[: piece.rfind(b"\n") + 1] or b"x\n"
            parts.append(piece)
            size += len(piece)
        text = b"".join(parts)
        ref = lc._C.cpu_run(lc.make_config("cpu"), text).entries()
        for chunk in (4 << 10, 64 << 10, 1 << 20):
            if max(len(x) for x in text.split(b"\n")) + 1 >= chunk:
                continue  # a line longer than the chunk is refused by design
            eng = lc._C.GpuEngine(lc.make_config("gpu", check=True, chunk_bytes=chunk), 1 << 30, 1 << 30)
            if eng.run(text).entries() != ref:
                say(f"MISMATCH streamed pageable seed={seed} chunk={chunk}")
                return 1
            if eng.run_text(lc._C.HostText.from_bytes(text)).entries() != ref:
                say(f"MISMATCH streamed pinned seed={seed} chunk={chunk}")
                return 1
            m += 2
    say(f"streamed: {m} runs of ~2 MB texts (chunks 4 KiB / 64 KiB / 1 MiB) match the CPU engine "
        f"({time.time() - t0:.1f} s)")
    # multi-rank jobs in this process (loopback ranks sharing the GPU: the exchange logic of
    # an N-GPU run), both strategies, several world sizes, against the oracle
    t0 = time.time()
    k = 0
    for i, ((seed, size, text), (ent, _n, _)) in enumerate(zip(texts, want)):
        if i % 9 not in (4, 7, 8) or i >= 9 * max(1, a.seeds // 5):
            continue  # a few sizes (4 KiB .. 200 KB) of every fifth seed
        for world in (2, 3, 8):
            for strategy in ("gather", "shuffle"):
                r = lc.run_multi(text, world, strategy=strategy)
                if r.entries() != ent:
                    say(f"MISMATCH multi-rank world={world} {strategy} seed={seed} size={size}")
                    return 1
                k += 1
    say(f"multi-rank (loopback, 2/3/8 ranks, gather and shuffle): {k} jobs match the oracle "
        f"({time.time() - t0:.1f} s)")
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
