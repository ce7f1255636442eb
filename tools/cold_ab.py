"""Cold first jobs on a large vocabulary (synth1m): fresh engines, alternating
LOCUST_ORD_VARIANT values (32 = partials keep walking after their LDS table overflowed,
the old behaviour; 0 = every wave stops at the first overflow).  Prints first/second/third
job wall times and checks the first job's output against the third's.
Usage: python tools/cold_ab.py [lines] [variants...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import locust_amd as lc  # noqa: E402

lines = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
# each variant: V or V:dma (LOCUST_OUT_COPY=dma: the fallback's result copied by
# hipMemcpyAsync instead of a kernel writing the mapped buffer)
variants = sys.argv[2:] or ["32", "0", "32", "0"]
text = lc._C.HostText.generate(lines=lines, seed=1, first_block=0)
for v in variants:
    os.environ["LOCUST_ORD_VARIANT"] = v.split(":")[0]
    os.environ["LOCUST_OUT_COPY"] = "dma" if v.endswith(":dma") else "kernel"
    cfg = lc.make_config("gpu", reduce_path="lds", chunk_bytes=256 << 20)
    eng = lc._C.GpuEngine(cfg, text.size, text.size)
    t = [time.perf_counter()]
    res = []
    for _ in range(3):  # results are kept, so jobs 2-3 also allocate their output buffers
        res.append(eng.run_text(text))
        t.append(time.perf_counter())
    same = res[0].entries() == res[2].entries() and res[0].num_tokens == res[2].num_tokens
    print(f"variant {v:>6}: first {1e3 * (t[1] - t[0]):8.3f} ms  second {1e3 * (t[2] - t[1]):7.3f} ms"
          f"  third {1e3 * (t[3] - t[2]):7.3f} ms  unique {res[2].num_unique}  first==third {same}",
          flush=True)
    del eng, res
