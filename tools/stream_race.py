"""Repeat the streamed-shard shuffle schedule (test_stream) to catch an intermittent
mismatch; prints the failing job index and the per-job token counts."""
import sys

import locust_amd as lc
from locust_amd.utils import oracle

hamlet = open("data/hamlet.txt", "rb").read()
world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
strategy = sys.argv[3] if len(sys.argv) > 3 else "shuffle"
chunk = int(sys.argv[4]) if len(sys.argv) > 4 else 8 << 10
ent, ntok, _ = oracle.wordcount(hamlet)
bad = 0
for rep in range(reps):
    job = lc.make_config("gpu", combine=True, check=True, chunk_bytes=chunk)
    cfgs = [lc.make_dist_config(world, job, strategy=strategy) for _ in range(2)]
    for j, (res, info) in enumerate(lc._C.run_multi_schedule(hamlet, cfgs)):
        if res.num_tokens != ntok or res.entries() != ent:
            bad += 1
            print(f"rep {rep} job {j}: tokens {res.num_tokens} unique {res.num_unique} info {info}")
            got = res.entries()
            wrong = [(i, g, w) for i, (g, w) in enumerate(zip(got, ent)) if g != w]
            print(f"  {len(wrong)} wrong entries; first/last index {wrong[0][0]} / {wrong[-1][0]}")
            for i, g, w in wrong[:4]:
                print(f"  [{i}] got {g} want {w}")
            kc = sum(1 for _i, g, w in wrong if g[0] == w[0] and g[2] != w[2])
            print(f"  same key, other count: {kc}; val-only differences: "
                  f"{sum(1 for _i, g, w in wrong if g[0] == w[0] and g[2] == w[2])}")
print(f"{bad} bad jobs of {2 * reps}")
