"""Per-job kernel timeline from rocprofv3 --kernel-trace CSV: kernel durations and the idle
gaps between consecutive kernels (launch / dependency latency inside a job).

    python tools/ktimeline.py run_kernel_trace.csv [last_n_kernels]"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"][:48], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
prev_end = None
for name, s, e in ks[-n:]:
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    print(f"{name:48s} dur={(e - s) / 1e3:8.2f} us  gap_before={gap:8.2f} us")
    prev_end = e
# steady-state medians per kernel name and of the gap before it
by = {}
prev_end = None
for name, s, e in ks[len(ks) // 2:]:
    d = by.setdefault(name, {"dur": [], "gap": []})
    d["dur"].append((e - s) / 1e3)
    if prev_end is not None:
        d["gap"].append((s - prev_end) / 1e3)
    prev_end = e
print("-- medians over the second half of the trace")
for name, d in by.items():
    print(f"{name:48s} calls={len(d['dur']):4d} dur={statistics.median(d['dur']):8.2f} us "
          f"gap_before={statistics.median(d['gap']) if d['gap'] else 0:8.2f} us")
