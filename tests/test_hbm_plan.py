"""HBM budget planning (SURVEY.md §5.7 "HBM budget accounting per GPU").

The reference sizes its device buffers by compile-time constants (main.cu:18-20, three
cudaMallocs at :393,402,451).  Here plan_device_pass prices an engine's arena before it
exists (the constructor's own sizing, DevicePipeline::shape_arena) and plans the pass
against its share of free HBM.  These checks need no GPU: the planner is host code."""
import pytest

import locust_amd as lc

GiB = 1 << 30
MiB = 1 << 20
HBM = 288 * GiB  # an MI355X


def plan(max_bytes, chunk_mb=0, free=HBM, share=1, sort="dict", lines=None, cap_records=0,
         map_path=None):
    cfg = lc.make_config("gpu", sort=sort, map_path=map_path)
    cfg.chunk_bytes = chunk_mb * MiB
    cfg.hbm_share = share
    return lc._C.plan_device_pass(cfg, max_bytes, lines if lines is not None else max_bytes,
                                  cap_records, free)


def test_streamed_256mib_pass_fits_6gb():
    """A 256 MiB streamed dictionary pass: 34.8 GB of arena in round 5, now <= 6 GB -- the
    token buffers hold one 32 MiB map window, the sort buffers the distinct keys."""
    p = plan(10 * GiB, chunk_mb=256)
    assert p["streaming"] and p["chunk_bytes"] == 256 * MiB
    assert p["map_window"] == 32 * MiB and p["pass_bytes"] == 32 * MiB
    assert p["cap"] == 16 * MiB + 1 and p["rcap"] == p["ucap"] == 16 * MiB
    assert p["device_bytes"] <= 6000 * MiB, p["device_bytes"] / MiB  # (round 5: 34,780 MiB)
    # the chunk size no longer scales the token buffers: only the two text chunks grow
    q = plan(10 * GiB, chunk_mb=1024)
    assert q["device_bytes"] - p["device_bytes"] == 2 * (1024 - 256) * MiB


def test_eight_ranks_on_one_gpu_stay_under_a_quarter_of_hbm():
    """10 GiB over 8 loopback ranks on one GPU: 1.25 GiB shards streamed in 256 MiB
    chunks; all eight engines together < 25 % of HBM."""
    share = 8
    p = plan(10 * GiB // 8, chunk_mb=256, share=share)
    assert p["streaming"] and 8 * p["device_bytes"] < 0.25 * HBM
    assert p["budget_bytes"] == int(HBM * 0.9) // 8


def test_one_pass_engine_sizes_distinct_keys_not_tokens():
    """A dictionary one-pass engine keeps every-token buffers only for the map output; the
    radix engine of the same pass holds every token in its sort buffers too."""
    d = plan(64 * MiB)
    r = plan(64 * MiB, sort="radix")
    assert not d["streaming"] and d["cap"] == 32 * MiB + 1
    assert d["rcap"] == 16 * MiB and r["rcap"] == r["cap"]
    assert d["device_bytes"] < r["device_bytes"]
    small = plan(200_000)  # Hamlet-sized: nothing changes (rcap == cap)
    assert small["rcap"] == small["cap"] == 100_001


def test_oversize_pass_is_planned_as_a_stream():
    """Past 2^30 tokens (the round-5 abort) or past the engine's HBM share, a one-pass
    dictionary input becomes a stream of 256 MiB chunks instead."""
    p = plan(4 * GiB)  # 2^31 worst-case tokens in one pass
    assert p["streaming"] and p["chunk_bytes"] == 256 * MiB and "2^30" in p["why"]
    q = plan(1 * GiB, free=16 * GiB)  # fits the token bound, not the HBM share
    assert q["streaming"] and "HBM" in q["why"] and q["device_bytes"] <= q["budget_bytes"]
    assert not plan(1 * GiB)["streaming"]  # the whole GPU: one pass


def test_oversize_chunk_is_refused_at_planning_time():
    with pytest.raises(Exception, match="--chunk-mb"):
        plan(400 * GiB, chunk_mb=200_000)
    with pytest.raises(Exception, match="HBM"):
        plan(10 * GiB, chunk_mb=4096, free=8 * GiB)
    # a chunk that covers the whole input asks for one pass of it: refused, not streamed
    with pytest.raises(Exception, match="smaller --chunk-mb"):
        plan(10 * GiB, chunk_mb=400_000)
    # a radix engine cannot stream: refused with the 2^30 bound, not silently wrong
    with pytest.raises(Exception, match="2\\^30"):
        plan(4 * GiB, sort="radix")


def test_receiver_engines_keep_every_record():
    p = plan(1, lines=1, cap_records=3_000_000)
    assert p["cap"] == p["rcap"] == 3_000_000 and not p["streaming"]


@pytest.mark.gpu
def test_cli_json_reports_the_hbm_plan(tmp_path):
    """`--json` carries the engine's device bytes, the GPU's free / total HBM and the pass
    shape -- one engine, a streamed engine, and every rank of a loopback run."""
    import json
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "build", "MapReduce")
    hamlet = os.path.join(root, "data", "hamlet.txt")

    def run(*args):
        j = tmp_path / "r.json"
        p = subprocess.run([cli, *map(str, args), "--json", str(j), "--quiet"], capture_output=True,
                           timeout=300)
        assert p.returncode == 0, p.stderr.decode()[-2000:]
        return json.loads(j.read_text())

    one = run(hamlet)
    assert 0 < one["hbm_device_bytes"] < 4 * GiB
    assert 200 * GiB < one["hbm_total_bytes"] and 0 < one["hbm_free_bytes"] <= one["hbm_total_bytes"]
    assert one["device_streaming"] is False
    g = tmp_path / "g.txt"
    subprocess.run([cli, "--gen", str(g), "--gen-bytes", str(6 << 20), "--seed", "2"], check=True,
                   capture_output=True, timeout=120)
    st = run(g, "--chunk-mb", 1)
    assert st["device_streaming"] is True and st["device_chunk_bytes"] == MiB
    assert 0 < st["device_map_window"] <= 32 * MiB
    ranks = run(g, "--gpus", 2, "--comm", "loopback")
    assert len(ranks["ranks"]) == 2
    assert ranks["hbm_device_bytes"] == sum(r["hbm_device_bytes"] for r in ranks["ranks"]) > 0
    assert all(r["hbm_total_bytes"] == ranks["hbm_total_bytes"] for r in ranks["ranks"])
    assert 0 < ranks["hbm_used_bytes_max"] <= ranks["hbm_total_bytes"]
