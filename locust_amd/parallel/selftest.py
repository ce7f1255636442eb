"""Rank self-test: prints this rank's layout as JSON (for launcher/daemon tests and for
checking a cluster's hosts file before a real job).

    python -m locust_amd.parallel.selftest [--fail-rank R --code C]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys

KEYS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--fail-rank", type=int, default=-1)
    ap.add_argument("--code", type=int, default=1)
    a = ap.parse_args(argv)
    info = {k: os.environ.get(k) for k in KEYS}
    info["host"] = socket.gethostname()
    print(json.dumps(info), flush=True)
    return a.code if int(os.environ.get("RANK", "-1")) == a.fail_rank else 0


if __name__ == "__main__":
    sys.exit(main())
