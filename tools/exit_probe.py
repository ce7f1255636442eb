"""Break a GPU process's start and exit down by how much of the GPU it touched (VERDICT r5
next #8: `./MapReduce`'s ~65 ms after its output is not ours to cut unless it is).

Runs build/exit_probe (tools/exit_probe.hip) in each mode, `--runs` fresh processes each,
and prints medians of: spawn -> main() (loader + static init), main() -> the stamp before
_exit (the mode's HIP work), and stamp -> reaped by this process (the exit: the kernel
driver releasing the process's queues and memory).

    python tools/exit_probe.py [--runs 7] [--out FILE]
"""
import argparse
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "build", "exit_probe")
MODES = ["none", "count", "context", "stream", "streams2", "memory"]


def one(mode: str) -> tuple:
    t0 = time.monotonic_ns()
    p = subprocess.run([PROBE, mode], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=60)
    t1 = time.monotonic_ns()
    if p.returncode:
        sys.exit(f"exit_probe {mode} failed ({p.returncode}): {p.stderr.decode()[-500:]}")
    t_main, t_exit = (int(x) for x in p.stdout.split())
    return (t_main - t0) * 1e-6, (t_exit - t_main) * 1e-6, (t1 - t_exit) * 1e-6


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=7)
    ap.add_argument("--out")
    a = ap.parse_args()
    lines = [f"build/exit_probe: median of {a.runs} fresh processes per mode (ms)",
             f"{'mode':10s} {'spawn->main':>12s} {'HIP work':>10s} {'exit':>8s}"]
    for mode in MODES:
        rows = [one(mode) for _ in range(a.runs)]
        med = [statistics.median(r[i] for r in rows) for i in range(3)]
        lines.append(f"{mode:10s} {med[0]:12.2f} {med[1]:10.2f} {med[2]:8.2f}")
        print(lines[-1], flush=True)
    text = "\n".join(lines) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
