"""bench.py's one-line JSON contract (the driver parses it): metric and config from
BASELINE.json, value == ms_per_step, the 1-GPU headline on whole Hamlet."""
import json
import os
import subprocess
import sys

import pytest

import locust_amd as lc

pytestmark = pytest.mark.gpu


def _run(*args):
    p = subprocess.run([sys.executable, "bench.py", *args], cwd=lc.REPO_ROOT,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout  # exactly one line on stdout
    return json.loads(lines[0])


def test_bench_single_gpu_line():
    base = json.load(open(os.path.join(lc.REPO_ROOT, "BASELINE.json")))
    d = _run("--steps", "20", "--warmup", "3", "--no-extra")
    assert d["metric"] == base["metric"]
    assert d["n_gpus"] == 1 and d["steps"] == 20 and d["warmup"] == 3
    assert d["value"] == d["ms_per_step"] and 0 < d["value"] < 5
    assert d["higher_is_better"] is False and d["scaling"] == "weak"
    assert d["tokens"] == 32940 and d["unique"] == 5608
    assert abs(d["vs_baseline"] - d["value"] / 77.393) < 1e-4
    assert d["config"]["parallelism"] == "dp1" and d["config"]["global_batch"] == 4463


def test_bench_synth_cold_start_line():
    d = _run("--config", "synth1m", "--steps", "3", "--warmup", "1")
    assert d["unique"] == 202645 and d["scaling"] == "strong"
    cs = d["cold_start"]
    assert cs["first_job_ms"] > 0 and cs["third_job_ms"] > 0
