"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel, the mean of each
counter over its dispatches, plus derived ratios (VALU instructions per wave, wait share,
LDS bank-conflict share, bytes per dispatch).

    python tools/pmc_summary.py OUT.txt DIR [DIR ...]
"""
import collections
import csv
import glob
import os
import sys


def short(name: str) -> str:
    return name.replace("locust::(anonymous namespace)::", "").split("(")[0][:44]


def main() -> int:
    out_path, dirs = sys.argv[1], sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    lines = []
    for k in sorted(acc):
        c = {n: sum(v) / len(v) for n, v in acc[k].items()}
        parts = [f"{n}={c[n]:.4g}" for n in sorted(c)]
        derived = []
        if c.get("SQ_WAVES"):
            if "SQ_INSTS_VALU" in c:
                derived.append(f"valu/wave={c['SQ_INSTS_VALU'] / c['SQ_WAVES']:.1f}")
            if "SQ_INSTS_LDS" in c:
                derived.append(f"lds/wave={c['SQ_INSTS_LDS'] / c['SQ_WAVES']:.1f}")
        if c.get("SQ_WAVE_CYCLES"):
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if n in c:
                    derived.append(f"{n[3:].lower()}_share={c[n] / c['SQ_WAVE_CYCLES']:.2f}")
        if c.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in c:
            derived.append(f"lds_conflict_share={c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:.3f}")
        lines.append(f"{k}\n    " + " ".join(parts) + ("\n    derived: " + " ".join(derived) if derived else ""))
    text = "\n".join(lines) + "\n"
    open(out_path, "w").write(text)
    print(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
