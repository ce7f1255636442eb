"""Cold one-shot CLI breakdown: `./MapReduce data/hamlet.txt` in fresh
processes, process start to exit, split with the CLI's own --json "startup" stamps:

  pre_main      process start -> main() (dynamic loader, libraries' static init), split
                at liblocust's static init (LOCUST_T0 passes the spawn time)
  runtime_init  the first HIP call (HIP runtime + KFD/device open)
  engine        GpuWordCount construction (code objects, device arena, pinned buffers)
  read          the file into the engine's pinned input buffer
  first_job     the first job (warmups included when --warmup > 0)
  later_jobs    the remaining jobs (--iters > 1)
  output        formatting and writing the result lines
  exit          JSON line -> process exit (teardown; LOCUST_FAST_EXIT=0 keeps the full one)

    python tools/cli_cold.py [--runs 5] [--iters 3] [--file data/hamlet.txt] [--out F]

Also reports whether librccl was mapped (LD_DEBUG=files in a separate run).
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "build", "MapReduce")
KEYS = ["runtime_init_ms", "engine_ms", "read_ms", "first_job_ms", "later_jobs_ms", "output_ms"]


def one(file: str, iters: int) -> dict:
    with tempfile.TemporaryDirectory() as d:
        j = os.path.join(d, "r.json")
        env = dict(os.environ, LOCUST_T0=str(time.monotonic_ns()))
        t0 = time.perf_counter()
        p = subprocess.run([CLI, file, "--json", j, "--iters", str(iters)], env=env,
                           stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=120)
        wall = (time.perf_counter() - t0) * 1e3
        if p.returncode:
            sys.exit(f"MapReduce failed: {p.stderr.decode()[-2000:]}")
        rec = json.load(open(j))
    st = rec["startup"]
    row = {k: st[k] for k in KEYS}
    row["process_ms"] = wall
    # the caller's clock also covers fork/exec and exit: what main() did not see
    row["pre_main_and_exit_ms"] = wall - st["main_to_json_ms"]
    # the split (LOCUST_T0): spawn -> this library's static init (fork/exec, loader, the
    # HIP runtime's static init), -> main (the rest of static init), JSON -> exit (teardown)
    row["spawn_to_library_ms"] = st.get("spawn_to_library_ms", float("nan"))
    row["library_to_main_ms"] = st.get("library_to_main_ms", float("nan"))
    row["exit_ms"] = row["pre_main_and_exit_ms"] - row["spawn_to_library_ms"] - row["library_to_main_ms"]
    row["wall_ms_median"] = rec["wall_ms_median"]
    return row


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--file", default=os.path.join(ROOT, "data", "hamlet.txt"))
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    one(a.file, 1)  # page the binaries and the file in
    rows = [one(a.file, a.iters) for _ in range(a.runs)]
    med = {k: statistics.median(r[k] for r in rows) for k in rows[0]}
    env = dict(os.environ, LD_DEBUG="files")
    p = subprocess.run([CLI, a.file], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                       timeout=120, env=env)
    libs = sorted({ln.split("file=")[1].split()[0] for ln in p.stderr.decode().splitlines()
                   if "file=" in ln and "[0];" in ln and "needed by" not in ln} |
                  {ln.split("file=")[1].split()[0] for ln in p.stderr.decode().splitlines()
                   if "file=" in ln and "needed by" in ln})
    steady = med["later_jobs_ms"] / max(a.iters - 1, 1)
    lines = [f"./MapReduce {os.path.relpath(a.file, ROOT)} --iters {a.iters}: median of {a.runs} fresh processes"]
    for k in (["process_ms", "pre_main_and_exit_ms", "spawn_to_library_ms", "library_to_main_ms",
               "exit_ms"] + KEYS + ["wall_ms_median"]):
        lines.append(f"  {k:22s} {med[k]:9.3f} ms")
    lines.append(f"  steady job (later_jobs / {max(a.iters - 1, 1)}) {steady:.3f} ms; first job's own "
                 f"overhead {med['first_job_ms'] - steady:.3f} ms")
    lines.append(f"  librccl mapped: {any('librccl' in x for x in libs)}; libraries opened: {len(libs)}")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n" + json.dumps({"median": med, "runs": rows, "libs": libs}) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
