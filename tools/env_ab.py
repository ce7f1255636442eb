"""A/B of an environment switch read at engine construction (e.g. LOCUST_OUT_NONCOHERENT)
on the single-GPU headline job, engines interleaved in one process.

    python tools/env_ab.py VAR value_a value_b [--steps 400] [--rounds 5] [--check]
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import locust_amd as lc  # noqa: E402
from locust_amd.utils import oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("var")
    ap.add_argument("values", nargs="+")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--config", default="hamlet4500")
    a = ap.parse_args()
    text = bench.load_text(a.config)
    nlines = text.count(b"\n") + (0 if text.endswith(b"\n") else 1)
    want = oracle.wordcount(text)[0]
    engines = {}
    for v in a.values:
        os.environ[a.var] = v
        e = lc._C.GpuEngine(lc.make_config("gpu", reduce_path="lds"), len(text), nlines)
        e.load(text)
        for _ in range(50):
            r = e.run_loaded()
        assert r.entries() == want, f"{a.var}={v}: wrong result"
        engines[v] = e
    loop = {v: [] for v in engines}
    for _ in range(a.rounds):
        for v, e in engines.items():
            t0 = time.perf_counter()
            for _ in range(a.steps):
                r = e.run_loaded()
            loop[v].append((time.perf_counter() - t0) * 1e3 / a.steps)
            assert r.entries() == want
    for v in engines:
        print(f"{a.var}={v}: ms/job {statistics.mean(loop[v]):.4f} (min round {min(loop[v]):.4f})")


if __name__ == "__main__":
    main()
