"""Per-job kernel offsets from a rocprofv3 kernel trace: jobs end at the ordered kernel.
    python tools/kjobs.py run_kernel_trace.csv [jobs]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
jobs, cur = [], []
for r in rows:
    cur.append(r)
    if "dict_ordered" in r["Kernel_Name"]:
        jobs.append(cur)
        cur = []
for j in jobs[-(int(sys.argv[2]) if len(sys.argv) > 2 else 2):]:
    t0 = int(j[0]["Start_Timestamp"])
    print("job span %.1f us" % ((int(j[-1]["End_Timestamp"]) - t0) / 1e3))
    for r in j:
        name = r["Kernel_Name"].replace("void ", "").replace("locust::(anonymous namespace)::", "")
        print("  %-28s q=%s start=%8.1f end=%8.1f" % (name[:28], r["Queue_Id"],
              (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3))
