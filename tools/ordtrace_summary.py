"""Summarise an ordered-kernel phase trace (LOCUST_ORD_TRACE=1 stderr) and a bench line.

    python tools/ordtrace_summary.py <dir with trace.txt [bench.json]> [top]"""
import json
import os
import re
import statistics
import sys

d = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 6
rows = []
for line in open(os.path.join(d, "trace.txt")):
    if line.startswith("ord"):
        rows.append({k: int(v) for k, v in re.findall(r"(\w+)=\s*(\d+)", line)})


def tot(r):
    return r["build"] + r["publish"] + r["sort"] + r["wait"] + r["write"]


rows.sort(key=lambda r: -tot(r))
for r in rows[:top]:
    print(tot(r), {k: v for k, v in r.items() if k != "p" or True})
if rows:
    print(len(rows), "partitions; median total", statistics.median(tot(r) for r in rows),
          "median build", statistics.median(r["build"] for r in rows))
b = os.path.join(d, "bench.json")
if os.path.exists(b):
    j = json.loads(open(b).read().strip().splitlines()[-1])
    print("bench", j["value"], j["stages_ms_median"])
