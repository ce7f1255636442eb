"""Distinct-key count vs the HBM-table path's sort (weighted all-pairs rank up to
kRankSortMax, radix above): streamed inputs with U distinct keys.  Run under rocprofv3
--kernel-trace --stats to see rank_sort_kernel / radix_pass_kernel times."""
import sys

import locust_amd as lc

for u in (2000, 8000, 16000, 30000, 60000):
    words = [b"k%06d" % (i % u) for i in range(4 * u)]
    text = b"".join(b" ".join(words[i:i + 10]) + b"\n" for i in range(0, len(words), 10))
    eng = lc._C.GpuEngine(lc.make_config("gpu", chunk_bytes=64 << 10), 64 << 10, 64 << 10)
    for _ in range(5):
        r = eng.run(text)
    t = r.times()
    print(f"U={u} unique={r.num_unique} wall={t['wall_ms']:.3f} ms process={t['process_ms']:.3f} "
          f"reduce={t['reduce_ms']:.3f}", flush=True)
