"""Where a fresh engine's first job goes: two engines in one process (the second one's
first job pays no process-level first-launch costs), constructor and first/second job
wall times, plus the job's own host timers.

    python tools/cold_probe.py [--config synth1m|hamlet4500] [--engines 2]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import locust_amd as lc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="synth1m")
    ap.add_argument("--engines", type=int, default=2)
    a = ap.parse_args()
    synth = a.config in bench.SYNTH
    text = bench.synth_shard(a.config, 0, 1) if synth else bench.load_text(a.config)
    for k in range(a.engines):
        t0 = time.perf_counter()
        if synth:
            cfg = lc.make_config("gpu", reduce_path="lds", chunk_bytes=bench.CHUNK_BYTES)
            e = lc._C.GpuEngine(cfg, text.size, text.size)
            run = lambda: e.run_text(text)  # noqa: E731
        else:
            e = lc._C.GpuEngine(lc.make_config("gpu", reduce_path="lds"), len(text),
                                bench._nlines(text))
            e.load(text)
            run = e.run_loaded
        t1 = time.perf_counter()
        walls = []
        for _ in range(3):
            s = time.perf_counter()
            r = run()
            walls.append((time.perf_counter() - s) * 1e3)
        tm = {k2: round(v, 3) for k2, v in r.times().items() if isinstance(v, float)}
        print(f"engine {k}: ctor {(t1 - t0) * 1e3:.2f} ms, jobs "
              + " / ".join(f"{w:.3f}" for w in walls) + f" ms; unique {r.num_unique}; "
              f"last job times {tm}", flush=True)


if __name__ == "__main__":
    main()
