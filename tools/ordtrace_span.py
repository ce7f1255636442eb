"""Critical path of the ordered dictionary kernel from LOCUST_ORD_TRACE=1 stderr (the last
job's block): span, slowest partitions, medians of the phases.

    python tools/ordtrace_span.py TRACE.txt [top]"""
import re
import statistics
import sys

text = open(sys.argv[1]).read()
top = int(sys.argv[2]) if len(sys.argv) > 2 else 5
blocks = text.split("ord span")
last = "ord span" + blocks[-1]
rows = [{k: float(v) for k, v in re.findall(r"(\w+)=\s*([\d.]+)", line)}
        for line in last.splitlines()[1:] if line.startswith("ord p=")]
print(last.splitlines()[0])
rows.sort(key=lambda r: -r["out"])
keys = ("p", "m", "build", "clear", "list", "gather", "publish", "sort", "wait", "write", "in",
        "out")
for r in rows[:top]:
    print({k: r[k] for k in keys})
for k in ("out", "build", "clear", "list", "gather", "publish", "sort", "wait", "write"):
    print(f"median {k}", statistics.median(r[k] for r in rows))
