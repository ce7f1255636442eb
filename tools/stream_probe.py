"""Streamed in-memory jobs (the synth10g config), engine after engine in one process:
per-job wall time of each engine, to tell a slow engine from a slow process.

Usage: python tools/stream_probe.py [--gb 10] [--engines 3] [--jobs 3]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=10.0)
    ap.add_argument("--engines", type=int, default=3)
    ap.add_argument("--jobs", type=int, default=3)
    ap.add_argument("--graph0", action="store_true", help="last engine with stage events")
    ap.add_argument("--keep", action="store_true", help="keep every engine alive")
    ap.add_argument("--between", default="", choices=["", "hostfree", "engine"],
                    help="after engine 0's jobs: free a pinned buffer / make and drop a small "
                         "engine, then run engine 0's jobs again")
    a = ap.parse_args()
    import locust_amd as lc

    t = time.perf_counter()
    text = lc._C.HostText.generate(bytes=int(a.gb * 1e9), seed=1, first_block=0)
    print(f"generated {text.size} B in {time.perf_counter() - t:.1f} s", flush=True)
    kept = []
    for e in range(a.engines):
        graph = 0 if (a.graph0 and e == a.engines - 1) else -1
        cfg = lc.make_config("gpu", reduce_path="lds", chunk_bytes=256 << 20, graph=graph)
        t = time.perf_counter()
        eng = lc._C.GpuEngine(cfg, text.size, text.size)
        ctor = (time.perf_counter() - t) * 1e3
        ms = []
        for _ in range(a.jobs):
            t = time.perf_counter()
            r = eng.run_text(text)
            ms.append((time.perf_counter() - t) * 1e3)
        tm = r.times()
        print(f"engine {e} graph={graph}: ctor {ctor:.1f} ms, jobs "
              + " / ".join(f"{m:.1f}" for m in ms)
              + f" ms; unique {r.num_unique}; map {tm['map_ms']:.1f} wall {tm['wall_ms']:.1f}",
              flush=True)
        if a.between and e == 0:
            if a.between == "hostfree":
                tmp = lc._C.HostText.generate(bytes=64 << 20, seed=2, first_block=0)
            else:
                tmp = lc._C.GpuEngine(cfg, 64 << 20, 64 << 20)
            del tmp
            ms = []
            for _ in range(a.jobs):
                t = time.perf_counter()
                r = eng.run_text(text)
                ms.append((time.perf_counter() - t) * 1e3)
            print(f"engine 0 after {a.between}: jobs " + " / ".join(f"{m:.1f}" for m in ms), flush=True)
        if a.keep:
            kept.append(eng)
        del r, eng
    return 0


if __name__ == "__main__":
    sys.exit(main())
