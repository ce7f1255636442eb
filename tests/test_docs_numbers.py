"""The README quotes the driver's own measurement: its
headline cells match the latest BENCH_r*.json the driver wrote (within 5 %), so the docs
never advertise a better number than the round-end run measured."""
import glob
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def latest_bench() -> dict:
    files = sorted(glob.glob(os.path.join(ROOT, "BENCH_r*.json")),
                   key=lambda p: int(re.search(r"BENCH_r(\d+)", p).group(1)))
    assert files, "no driver bench record"
    d = json.load(open(files[-1]))
    tail = d.get("run", {}).get("stdout_tail", "")
    line = next(ln for ln in tail.splitlines() if ln.startswith("{"))
    return json.loads(line) | {"_file": os.path.basename(files[-1])}


def readme_cell(row_start: str) -> float:
    text = open(os.path.join(ROOT, "README.md")).read()
    row = next(ln for ln in text.splitlines() if ln.startswith(row_start))
    cells = [c.strip() for c in row.strip("|").split("|")]
    return float(re.search(r"[0-9]+\.[0-9]+", cells[2]).group(0))


def test_readme_headline_is_the_drivers_number():
    b = latest_bench()
    cases = [("| Hamlet whole file", b["value"]),
             ("| same, untuned", b["untuned"]["ms_per_step"]),
             ("| Hamlet 0-700 lines", b["hamlet700"]["ms_per_step"]),
             ("| A fresh engine's first job", b["cold_start"]["hamlet4500"]["first_job_ms"])]
    for row, want in cases:
        got = readme_cell(row)
        assert abs(got - want) <= 0.05 * want, (row, got, want, b["_file"])
