"""Root merge alone (no other kernels in flight): P sorted runs shaped like the gather
strategy's slots -- every run the combined output of one rank's Hamlet copy, or of a 1/P
chunk with --chunk -- merged JOBS times through Engine.merge_runs, for kernel profiles of
merge_split/merge_segment (or merge_rank/merge_emit under LOCUST_MERGE_SEARCH=1).

    python tools/merge_prof.py [runs] [jobs] [--chunk]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import locust_amd as lc  # noqa: E402
from locust_amd.utils import oracle  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
nruns = int(args[0]) if args else 8
jobs = int(args[1]) if len(args) > 1 else 20
text = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         "data", "hamlet.txt"), "rb").read()
if "--chunk" in sys.argv:
    step = len(text) // nruns
    parts = [text[i * step:(i + 1) * step if i + 1 < nruns else len(text)]
             for i in range(nruns)]
else:
    parts = [text] * nruns
runs = []
for p in parts:
    entries, _, _ = oracle.wordcount(p)
    runs.append([(k, c) for k, _, c in entries])
eng = lc.Engine(lc.make_config("gpu"), 1 << 20, 1 << 16)
for _ in range(jobs):
    res = eng.merge_runs(runs)
print("runs", nruns, "records", sum(len(r) for r in runs), "unique", res.num_unique)
