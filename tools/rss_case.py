"""Peak host RSS of a streamed CLI run under different output handling (captured pipe,
--quiet, /dev/null), with the CLI's own LOCUST_LOG=info rss lines.
    python tools/rss_case.py OUTDIR"""
import os
import subprocess
import sys

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
cli = "./build/MapReduce"
f = "/tmp/locust_rss_case.txt"
subprocess.run([cli, "--gen", f, "--gen-bytes", str(320 << 20), "--seed", "5"], check=True,
               capture_output=True, timeout=120)
env = {**os.environ, "LOCUST_LOG": "info"}
with open(os.path.join(out, "rss_case.txt"), "w") as log:
    for name, extra in [("captured", []), ("quiet", ["--quiet"])]:
        p = subprocess.run([cli, f, "--chunk-mb", "64"] + extra, capture_output=True, env=env,
                           timeout=300)
        rss = [l for l in p.stderr.decode().splitlines() if "rss" in l]
        print(name, p.returncode, len(p.stdout), *rss, sep="\n  ", file=log, flush=True)
    with open(os.devnull, "wb") as dn:
        p = subprocess.run([cli, f, "--chunk-mb", "64"], stdout=dn, stderr=subprocess.PIPE,
                           env=env, timeout=300)
    rss = [l for l in p.stderr.decode().splitlines() if "rss" in l]
    print("devnull", p.returncode, *rss, sep="\n  ", file=log, flush=True)
os.remove(f)
