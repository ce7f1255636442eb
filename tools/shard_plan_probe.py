"""First jobs of fresh engines on 1/N shards of synth1m: did the in-job partition plan
hold (no fallback), how long did each job take?
    python tools/shard_plan_probe.py N [SHARDS] [JOBS]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import locust_amd as lc  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
shards = int(sys.argv[2]) if len(sys.argv) > 2 else n
jobs = int(sys.argv[3]) if len(sys.argv) > 3 else 2
for r in range(shards):
    text = bench.synth_shard("synth1m", r, n)
    cfg = lc.make_config("gpu", reduce_path="lds", chunk_bytes=bench.chunk_bytes_for(text.size))
    e = lc._C.GpuEngine(cfg, text.size, text.size)
    ts = []
    for _ in range(jobs):
        t0 = time.perf_counter()
        res = e.run_text(text)
        ts.append(1e3 * (time.perf_counter() - t0))
        tm = {k: round(v, 3) for k, v in res.times().items() if isinstance(v, float) and v}
        print(f"  job: {ts[-1]:.3f} ms (engine wall {tm.get('wall_ms', 0):.3f}) stats {e.stats()} "
              f"times {tm}", file=sys.stderr, flush=True)
    print(f"shard {r}/{n}: {text.size} B, unique {res.num_unique}, jobs "
          + " / ".join(f"{t:.3f}" for t in ts) + f" ms, stats {e.stats()}", flush=True)
