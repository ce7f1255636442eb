"""Summarise a rocprofv3 kernel_stats.csv: name, calls, avg/min us, share."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    name = r["Name"].replace("locust::(anonymous namespace)::", "").split("(")[0]
    print(f"{name[:48]:48s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:8.2f} "
          f"min_us={float(r['MinNs'])/1e3:8.2f} pct={float(r['Percentage']):5.1f}")
