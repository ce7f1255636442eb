"""Summarise rocprofv3 kernel timings: name, calls, avg/min us, share.

    python tools/kstats.py <kernel_stats.csv | results.db | directory holding either>

A .db is rocprofv3's default rocpd (SQLite) output: per-dispatch start/end are aggregated
here the way --stats would."""
import collections
import csv
import glob
import os
import sqlite3
import sys


def short(name):
    return name.replace("locust::(anonymous namespace)::", "").split("(")[0]


def from_csv(path):
    for r in csv.DictReader(open(path)):
        yield short(r["Name"]), int(r["Calls"]), float(r["AverageNs"]), float(r["MinNs"]), \
            float(r["Percentage"])


def from_db(path):
    c = sqlite3.connect(path)
    names = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    kd = next(n for n in names if n.startswith("rocpd_kernel_dispatch"))
    ks = next(n for n in names if n.startswith("rocpd_info_kernel_symbol"))
    per = collections.defaultdict(list)
    for name, ns in c.execute(f"select s.display_name, d.end - d.start from {kd} d "
                              f"join {ks} s on d.kernel_id = s.id"):
        per[short(name)].append(ns)
    total = sum(sum(v) for v in per.values()) or 1
    for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        yield name, len(v), sum(v) / len(v), min(v), 100.0 * sum(v) / total


def main(arg):
    path = arg
    if os.path.isdir(arg):
        hits = (glob.glob(os.path.join(arg, "**", "*kernel_stats.csv"), recursive=True) or
                glob.glob(os.path.join(arg, "**", "*.db"), recursive=True))
        if not hits:
            sys.exit(f"no kernel_stats.csv or .db under {arg}")
        path = hits[0]
    rows = from_db(path) if path.endswith(".db") else from_csv(path)
    for name, calls, avg, mn, pct in rows:
        print(f"{name[:48]:48s} calls={calls:>5} avg_us={avg / 1e3:8.2f} "
              f"min_us={mn / 1e3:8.2f} pct={pct:5.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
