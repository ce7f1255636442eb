"""Per-job wall times of the synth10g job (streamed run_text on pinned host text) in the
regimes bench.py mixes: results dropped at once (the cold probe) vs the previous result
held while the next job runs (the timed loop), and with the between-job retune off.
    PYTHONPATH=. python tools/s10g_probe.py [GB] [jobs]"""
import os
import sys
import time

import locust_amd as lc

gb = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
jobs = int(sys.argv[2]) if len(sys.argv) > 2 else 5
t = time.perf_counter()
h = lc._C.HostText.generate(bytes=int(gb * 1e9), seed=1, first_block=0)
print(f"generated {h.size} B in {time.perf_counter() - t:.1f} s", flush=True)


def run(tag, hold, env=None):
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        cfg = lc.make_config("gpu", reduce_path="lds", chunk_bytes=256 << 20)
        eng = lc._C.GpuEngine(cfg, h.size, h.size)
        ts, keep = [], None
        for _ in range(jobs):
            t0 = time.perf_counter()
            r = eng.run_text(h)
            ts.append((time.perf_counter() - t0) * 1e3)
            keep = r if hold else None
            del r
        st = eng.stats()
        print(f"{tag:28s} " + " ".join(f"{x:7.1f}" for x in ts) + f"   stats {st}", flush=True)
        del keep
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


run("drop results", False)
run("hold previous result", True)
run("hold, PART_TUNE=0", True, {"LOCUST_PART_TUNE": "0"})
run("drop, PART_TUNE=0", False, {"LOCUST_PART_TUNE": "0"})
