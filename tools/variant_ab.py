"""A/B of kernel variants (LOCUST_ORD_VARIANT values) on the single-GPU headline job, the
engines interleaved in one process so box-to-box noise cancels.

    python tools/variant_ab.py 0 1 [--steps 400] [--rounds 5] [--config hamlet4500]
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
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--config", default="hamlet4500")
    a = ap.parse_args()
    text = bench.load_text(a.config)
    nlines = text.count(b"\n") + (0 if text.endswith(b"\n") else 1)
    engines = {}
    for v in a.variants:
        os.environ["LOCUST_ORD_VARIANT"] = v  # read when the engine's graph is captured
        e = lc._C.GpuEngine(lc.make_config("gpu", reduce_path="lds"), len(text), nlines)
        e.load(text)
        for _ in range(50):
            e.run_loaded()
        engines[v] = e
    loop = {v: [] for v in engines}
    gpu = {v: [] for v in engines}
    for _ in range(a.rounds):
        for v, e in engines.items():
            t0 = time.perf_counter()
            for _ in range(a.steps):
                gpu[v].append(e.run_loaded().times()["gpu_ms"])
            loop[v].append((time.perf_counter() - t0) * 1e3 / a.steps)
    for v in engines:
        print(f"variant {v}: ms/job {statistics.mean(loop[v]):.4f} (min round {min(loop[v]):.4f}) "
              f"gpu(event) median {statistics.median(gpu[v]):.4f}")


if __name__ == "__main__":
    main()
