"""How good is the in-job plan on synth1m?  A fresh engine's first job with the ordered
kernel's per-partition trace (LOCUST_ORD_TRACE=1 must be set): distinct keys per partition
under the planned map, against the LDS table size (kPartSlots = 2048).
    LOCUST_ORD_TRACE=1 python tools/plan_quality.py [--lines N] > out 2> trace"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import locust_amd as lc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lines", type=int, default=None)
ap.add_argument("--engines", type=int, default=2)
a = ap.parse_args()
text = bench.synth_shard("synth1m", 0, 1, a.lines)
for k in range(a.engines):
    cfg = lc.make_config("gpu", reduce_path="lds", chunk_bytes=bench.chunk_bytes_for(text.size))
    e = lc._C.GpuEngine(cfg, text.size, text.size)
    print(f"=== engine {k}", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    r = e.run_text(text)
    t1 = time.perf_counter()
    print(f"engine {k}: first job {1e3 * (t1 - t0):.3f} ms, unique {r.num_unique}, stats {e.stats()}",
          flush=True)
    del r
