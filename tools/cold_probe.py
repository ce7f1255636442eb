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
    ap.add_argument("--jobs", type=int, default=3)
    a = ap.parse_args()
    synth = a.config in bench.SYNTH
    text = bench.synth_shard(a.config, 0, 1) if synth else bench.load_text(a.config)
    r = None
    for k in range(a.engines):
        r = None  # the previous engine's last result: released outside the timed jobs
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
        walls, splits = [], []
        for _ in range(a.jobs):
            s = time.perf_counter()
            r = run()
            walls.append((time.perf_counter() - s) * 1e3)
            t = r.times()
            splits.append("/".join(f"{t[x]:.3f}" for x in ("host_launch_ms", "host_wait_ms",
                                                            "host_copy_ms")))
        print(f"engine {k}: ctor {(t1 - t0) * 1e3:.2f} ms, jobs "
              + " / ".join(f"{w:.3f}" for w in walls) + f" ms; unique {r.num_unique}; "
              "launch/wait/copy per job: " + "  ".join(splits), flush=True)


if __name__ == "__main__":
    main()
