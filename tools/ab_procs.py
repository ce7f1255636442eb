"""Separate-process A/B of environment variants on one bench config (the in-process
env_ab.py shares HW queues and caches between the variants' engines): every round starts
one fresh process per variant, in alternating order, each timing `--steps` jobs after
`--warmup` on a fresh engine (bench._time_single); prints per-variant medians over rounds.

    python tools/ab_procs.py "LOCUST_PART_TUNE=0" "LOCUST_PART_TUNE=0,LOCUST_PART_DEFAULT=byte" \\
        [--config hamlet4500|hamlet700|synth1m|file:PATH] [--rounds 5] [--steps 300] [--warmup 30]

A variant's ROOT=<dir> runs it from another built tree (e.g. a previous commit exported
with `git archive` and built with make): code changes without a switch of their own.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, time
sys.path.insert(0, sys.argv[1])
import bench
cfg, steps, warmup, rep = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
if cfg.startswith("file:"):
    text = open(cfg[5:], "rb").read() * rep
else:
    text = bench.synth_shard(cfg, 0, 1) if cfg in bench.SYNTH else bench.load_text(cfg) * rep
first = bench.cold_first_run(text)["first_job_ms"]
ms, _st, res = bench._time_single(text, steps, warmup, "dict", -1)
print(json.dumps({"ms": ms, "first": first, "unique": res.num_unique}))
"""


def env_of(variant: str) -> dict:
    env = dict(os.environ)
    for kv in filter(None, variant.split(",")):
        k, _, v = kv.partition("=")
        if k.strip() != "ROOT":
            env[k.strip()] = v.strip()
    return env


def root_of(variant: str) -> str:
    for kv in filter(None, variant.split(",")):
        k, _, v = kv.partition("=")
        if k.strip() == "ROOT":
            return os.path.abspath(os.path.join(ROOT, v.strip()))
    return ROOT


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--config", default="hamlet4500")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--repeat", type=int, default=1, help="text configs: the text N times over")
    a = ap.parse_args()
    got = {v: [] for v in a.variants}
    firsts = {v: [] for v in a.variants}
    for r in range(a.rounds):
        order = a.variants if r % 2 == 0 else a.variants[::-1]
        for v in order:
            p = subprocess.run([sys.executable, "-c", CHILD, root_of(v), a.config, str(a.steps),
                                str(a.warmup), str(a.repeat)], env=env_of(v), capture_output=True, text=True,
                               timeout=300)
            if p.returncode:
                print(p.stderr[-2000:], file=sys.stderr)
                return 1
            d = json.loads(p.stdout.strip().splitlines()[-1])
            got[v].append(d["ms"])
            firsts[v].append(d["first"])
    for v in a.variants:
        print(f"{v or '(default)'}: ms/job median {statistics.median(got[v]):.4f} "
              f"(rounds {' '.join(f'{x:.4f}' for x in got[v])}); first job median "
              f"{statistics.median(firsts[v]):.4f} ms", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
