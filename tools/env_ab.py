"""A/B of environment switches on the single-GPU headline job, engines interleaved in one
process (box-to-box noise cancels).  A variant is a comma-separated list of VAR=value
settings, applied while its engine is constructed AND while its jobs run (switches read
per job, e.g. LOCUST_PART_TUNE, and at construction, e.g. LOCUST_VPLAN, both take).

    python tools/env_ab.py "LOCUST_VPLAN=1" "LOCUST_VPLAN=0,LOCUST_PART_TUNE=0" \\
        [--steps 400] [--rounds 5] [--config hamlet4500|hamlet700|synth1m]
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


def settings(variant: str) -> dict:
    out = {}
    for kv in filter(None, variant.split(",")):
        k, _, v = kv.partition("=")
        out[k.strip()] = v.strip()
    return out


class Env:
    def __init__(self, kv: dict):
        self.kv, self.old = kv, {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = os.environ.get(k)
            os.environ[k] = v

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--config", default="hamlet4500")
    a = ap.parse_args()
    synth = a.config in bench.SYNTH
    if synth:
        text = bench.synth_shard(a.config, 0, 1)
        want_u = None
    else:
        text = bench.load_text(a.config)
        want = oracle.wordcount(text)[0]
    engines, firsts = {}, {}
    for v in a.variants:
        with Env(settings(v)):
            if synth:
                cfg = lc.make_config("gpu", reduce_path="lds", chunk_bytes=bench.CHUNK_BYTES)
                e = lc._C.GpuEngine(cfg, text.size, text.size)
                run = (lambda e: lambda: e.run_text(text))(e)
            else:
                e = lc._C.GpuEngine(lc.make_config("gpu", reduce_path="lds"), len(text),
                                    bench._nlines(text))
                e.load(text)
                run = e.run_loaded
            t0 = time.perf_counter()
            r = run()
            firsts[v] = (time.perf_counter() - t0) * 1e3
            for _ in range(30 if synth else 50):
                r = run()
            if synth:
                want_u = want_u or r.num_unique
                assert r.num_unique == want_u, f"{v}: wrong result"
            else:
                assert r.entries() == want, f"{v}: wrong result"
            engines[v] = run
    loop = {v: [] for v in engines}
    for _ in range(a.rounds):
        for v, run in engines.items():
            with Env(settings(v)):
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    r = run()
                loop[v].append((time.perf_counter() - t0) * 1e3 / a.steps)
    for v in engines:
        print(f"{v or '(default)'}: first job {firsts[v]:.4f} ms, ms/job "
              f"{statistics.mean(loop[v]):.4f} (min round {min(loop[v]):.4f})", flush=True)


if __name__ == "__main__":
    main()
