"""Every LOCUST_* switch the native code reads runs in a test:
one process per setting (tests/switch_worker.py) runs its workload -- one-GPU jobs, a
streamed job or loopback ranks -- and checks every result against the oracle.  Switches
whose meaning is diagnostics-only (traces, logging) must not change the output either."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "switch_worker.py")

# (environment, workload).  Each switch appears at least once with a non-default value.
CASES = [
    ({"LOCUST_CHECK": "1"}, "single"),
    ({"LOCUST_MAP_PATH": "compat"}, "single"),
    ({"LOCUST_SORT": "radix", "LOCUST_REDUCE_PATH": "global"}, "single"),
    ({"LOCUST_SORT": "radix", "LOCUST_PSORT": "0"}, "single"),
    ({"LOCUST_ZERO_COPY": "0", "LOCUST_LEAN": "0"}, "single"),
    ({"LOCUST_GRAPH": "0"}, "single"),
    ({"LOCUST_GRAPH": "1"}, "single"),
    ({"LOCUST_PIECE_MB": "4"}, "single"),
    ({"LOCUST_MERGE_MAX_RECORDS": "100"}, "merge"),
    ({"LOCUST_CACHE_DIR": "", "LOCUST_PART_CACHE": "1"}, "cli"),
    ({"LOCUST_PART_CACHE": "0"}, "cli"),
    ({"LOCUST_FAST_EXIT": "0"}, "cli"),
    ({"LOCUST_PART_TUNE": "0", "LOCUST_PART_DEFAULT": "byte"}, "single"),
    ({"LOCUST_VPLAN": "0", "LOCUST_DEVPLAN": "0"}, "single"),
    ({"LOCUST_VPLAN_MIN_KB": "64", "LOCUST_SPLIT_MIN": "256"}, "single"),
    ({"LOCUST_PART_TUNE": "0", "LOCUST_PLAN_TRIGGER": "0"}, "single"),
    ({"LOCUST_SMALL_PASS_KB": "0"}, "single"),
    ({"LOCUST_DEV_CACHE": "0"}, "stream"),
    ({"LOCUST_HUGE_PIN": "0"}, "stream"),
    ({"LOCUST_DEV_CACHE_GB": "1", "LOCUST_CHUNK_MB": "1"}, "stream"),
    ({"LOCUST_ORD_TRACE": "1", "LOCUST_MAP_TRACE": "1", "LOCUST_ROCTX": "0",
      "LOCUST_LOG": "debug"}, "single"),
    ({"LOCUST_EXCHANGE": "0"}, "dist"),
    ({"LOCUST_EXCH_ASYNC": "0", "LOCUST_DIST_LOCAL": "0"}, "dist"),
    ({"LOCUST_EXCH_TRACE": "1", "LOCUST_OUT_WAIT_S": "60", "LOCUST_NUMA": "0",
      "LOCUST_SLOT_GRAPH": "0", "LOCUST_EXCH_SLOT": "64"}, "dist"),
]


def test_every_switch_has_a_case():
    """A switch added to csrc/ must get a case here (or a dedicated test that sets it)."""
    used = set()
    for d, _, files in os.walk(os.path.join(ROOT, "csrc")):
        for f in files:
            if f.endswith((".cpp", ".hpp", ".hip")):
                used |= set(re.findall(r'getenv\("(LOCUST_[A-Z0-9_]+)"',
                                       open(os.path.join(d, f), errors="replace").read()))
    covered = {k for env, _ in CASES for k in env} | {
        "LOCUST_FAULT",        # test_dist*.py, test_scale_ready.py
        "LOCUST_LINE_CACHE",   # test_line_index.py
        "LOCUST_T0"}           # tools/cli_cold.py (timestamps only)
    assert used and not sorted(used - covered)


@pytest.mark.gpu
@pytest.mark.parametrize("env,kind", CASES, ids=[",".join(f"{k[7:]}={v}" for k, v in e.items())
                                                  for e, _ in CASES])
def test_switch(env, kind):
    full = dict(os.environ)
    full.update(env)
    r = subprocess.run([sys.executable, WORKER, kind], env=full, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "switch worker ok" in r.stdout
