"""Chunk-size sweep of the streaming path on the synthetic 1M-line input (43 MB): whole
job ms per chunk size, engines interleaved in one process.

    python tools/chunk_ab.py [--mb 256 32 16 8 4] [--steps 20] [--rounds 3]
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import locust_amd as lc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, nargs="+", default=[256, 32, 16, 8, 4])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--lines", type=int, default=1_000_000)
    a = ap.parse_args()
    text = lc._C.HostText.generate(lines=a.lines, seed=1, first_block=0)
    engines = {}
    for mb in a.mb:
        cfg = lc.make_config("gpu", reduce_path="lds", chunk_bytes=mb << 20)
        e = lc._C.GpuEngine(cfg, max(text.size, 1), max(text.size, 1))
        for _ in range(3):
            r = e.run_text(text)
        engines[mb] = e
    ms = {mb: [] for mb in engines}
    for _ in range(a.rounds):
        for mb, e in engines.items():
            t0 = time.perf_counter()
            for _ in range(a.steps):
                r = e.run_text(text)
            ms[mb].append((time.perf_counter() - t0) * 1e3 / a.steps)
    for mb in engines:
        print(f"chunk {mb:4d} MiB: {statistics.mean(ms[mb]):.3f} ms/job (min round {min(ms[mb]):.3f})"
              f"  unique={r.num_unique}")


if __name__ == "__main__":
    main()
