"""Per-step wall times of the synth1m job (run_text on pinned host text), to separate
outliers from the steady state.   PYTHONPATH=. python tools/steps.py [lines] [steps]"""
import statistics
import sys
import time

import locust_amd as lc

lines = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
graph = int(sys.argv[3]) if len(sys.argv) > 3 else -1
h = lc._C.HostText.generate(lines=lines, seed=1)
cfg = lc.make_config("gpu", reduce_path="lds", chunk_bytes=256 << 20, graph=graph)
eng = lc._C.GpuEngine(cfg, h.size, h.size)
for _ in range(3):
    r = eng.run_text(h)
ts = []
for i in range(steps):
    t0 = time.perf_counter()
    r = eng.run_text(h)
    ts.append((time.perf_counter() - t0) * 1e3)
    if ts[-1] > 2.0:
        print("slow step", i, {k: round(v, 3) for k, v in r.times().items()})
print("steps:", " ".join(f"{t:.3f}" for t in ts))
print(f"mean {statistics.mean(ts):.3f} median {statistics.median(ts):.3f} min {min(ts):.3f} "
      f"max {max(ts):.3f}  unique {r.num_unique}")
