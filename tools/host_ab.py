"""A/B of the single-GPU headline job's host-side variants (graph replay on/off), the
two interleaved in one process so box-to-box noise cancels.

    python tools/host_ab.py [--steps 400] [--rounds 5] [--config hamlet4500|hamlet700]
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import locust_amd as lc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--config", default="hamlet4500")
    a = ap.parse_args()
    text = bench.load_text(a.config)
    nlines = text.count(b"\n") + (0 if text.endswith(b"\n") else 1)
    engines = {}
    for g in (1, 0):
        cfg = lc.make_config("gpu", reduce_path="lds", graph=g)
        e = lc._C.GpuEngine(cfg, len(text), nlines)
        e.load(text)
        for _ in range(50):
            e.run_loaded()
        engines[g] = e
    res = {g: [] for g in engines}
    walls = {g: [] for g in engines}
    gpus = {g: [] for g in engines}
    split = {g: {"host_launch_ms": [], "host_wait_ms": [], "host_copy_ms": []} for g in engines}
    for _ in range(a.rounds):
        for g, e in engines.items():
            t0 = time.perf_counter()
            for _ in range(a.steps):
                r = e.run_loaded()
                t = r.times()
                walls[g].append(t["wall_ms"])
                gpus[g].append(t["gpu_ms"])
                for k in split[g]:
                    split[g][k].append(t[k])
            res[g].append((time.perf_counter() - t0) * 1e3 / a.steps)
    for g in engines:
        print(f"graph={g}: python loop ms/job mean-of-rounds {statistics.mean(res[g]):.4f} "
              f"min-round {min(res[g]):.4f} | C++ wall median {statistics.median(walls[g]):.4f} "
              f"| gpu(event) median {statistics.median(gpus[g]):.4f} | " +
              " ".join(f"{k[5:]} {statistics.median(v):.4f}" for k, v in split[g].items()))


if __name__ == "__main__":
    main()
