"""A fresh engine's first job does no one-time work (it regressed to
0.185 ms when the partition-map retune and the process's first roctx range ran inside it).

The CPU tests pin the structure that keeps one-time work out of the job: every kernel
file's code object is loaded at engine construction, the engine's construction initialises
roctx, starts the retune worker and makes its stream's first launch, and the retune after
a job is handed to the worker instead of running inline.  The GPU test bounds the first
job itself."""
import os
import re
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _src(*p):
    return open(os.path.join(ROOT, *p), errors="replace").read()


def _body(src: str, signature: str) -> str:
    """The brace-balanced body of the function whose definition starts with `signature`."""
    i = src.index(signature)
    j = src.index("{", i)
    depth = 0
    for k in range(j, len(src)):
        depth += {"{": 1, "}": -1}.get(src[k], 0)
        if depth == 0:
            return src[j:k + 1]
    raise AssertionError("unbalanced " + signature)


def test_every_kernel_module_is_warmed():
    warm = _body(_src("csrc", "include", "locust", "kernels.hpp"), "inline void warm_kernel_modules()")
    kdir = os.path.join(ROOT, "csrc", "kernels")
    for f in sorted(os.listdir(kdir)):
        if not f.endswith(".hip"):
            continue
        s = _src("csrc", "kernels", f)
        if "__global__" not in s:
            continue
        name = f[:-4]
        if name == "selftest":  # the string library's device self-test: never in a job
            continue
        assert re.search(r"void warm_module_%s\(\)" % name, s), f"{f}: no warm_module_{name}()"
        assert f"warm_module_{name}();" in warm, f"warm_kernel_modules() misses {name}"


def test_engine_construction_does_the_one_time_work():
    s = _src("csrc", "engine", "pipeline.hip")
    warm = _body(s, "void DevicePipeline::warm_modules_once(int device)")
    assert "warm_kernel_modules();" in warm and "TraceRange" in warm  # roctx initialised
    ctor = _body(s, "DevicePipeline::DevicePipeline(const JobConfig& c")
    assert "warm_modules_once(" in ctor
    assert "retune_worker.start();" in ctor  # the thread exists before the first job
    assert "launch_signal_host(" in ctor  # the stream's first kernel launch


def test_retune_never_runs_inside_a_job():
    s = _src("csrc", "engine", "pipeline.hip")
    mr = _body(s, "void DevicePipeline::maybe_retune(const EntryList& e)")
    assert "retune_worker.submit(" in mr
    # the map is built on the worker: no inline pass over the output in the job
    outside = mr.replace(mr[mr.index("retune_worker.submit("):], "")
    assert "part_map_from" not in outside and "part_map_groups" not in outside
    poll = _body(s, "void DevicePipeline::poll_retune()")
    assert "idle()" in poll and "wait_idle" not in poll  # adopting never blocks a job


@pytest.mark.gpu
def test_fresh_engine_first_job_is_cheap(hamlet):
    """A fresh engine's first Hamlet job within 2x (+ 50 us) of its steady jobs (round 4:
    0.185 vs 0.039 ms; round 5 bench cold_start 0.070-0.076 ms)."""
    import locust_amd as lc

    warm = lc._C.GpuEngine(lc.make_config("gpu", reduce_path="lds"), len(hamlet), 5000)
    warm.load(hamlet)
    warm.run_loaded()  # process-level first use (runtime queues, code objects)
    firsts, steadies = [], []
    for _ in range(3):
        eng = lc._C.GpuEngine(lc.make_config("gpu", reduce_path="lds"), len(hamlet), 5000)
        eng.load(hamlet)
        t = []
        for _ in range(6):
            t0 = time.perf_counter()
            eng.run_loaded()
            t.append(time.perf_counter() - t0)
        firsts.append(t[0])
        steadies.append(min(t[1:]))
        del eng
    first, steady = min(firsts), min(steadies)
    assert first < 2 * steady + 50e-6, (firsts, steadies)


def test_plan_runs_only_when_the_map_saw_crowding():
    """The in-job plan: the map raises OrderedExtra::plan_flag from a
    tile's partition counts (kPlanTrigger), the ordered kernel loads the flag with its
    ticket and plans only when it is up, and the self-clean re-zeroes it for the next job.
    Whole Hamlet peaks at 27 tokens of one partition per 1 KiB tile under the starting map,
    below the trigger (profiles/r5/partmap/hamlet_default_map_partitions.txt)."""
    mt = _src("csrc", "kernels", "map_tile.hpp")
    trig = int(re.search(r"constexpr u32 kPlanTrigger = (\d+);", mt).group(1))
    assert 27 < trig <= 64
    assert "atomicOr(plan_flag, 1u)" in mt
    d = _src("csrc", "kernels", "dict.hip")
    assert "__hip_atomic_load(ex.plan_flag" in d
    assert "vplan = flag != 0;" in d
    assert "if (ex.plan_flag) *ex.plan_flag = 0;" in d
    p = _src("csrc", "engine", "pipeline.hip")
    assert "ex.plan_flag = d_plan_flag" in p


def test_engine_runs_a_warm_up_job_without_side_effects():
    """GpuWordCount's constructor runs one two-byte lean job (warm_first_job): the map and
    the ordered build are enqueued once on the engine's stream before its first real job
    (cold probe: the first job's enqueue 20 -> 7-10 us).  The warm-up job must not retune
    the partition map from its one-key output nor print traces."""
    g = _src("csrc", "engine", "gpu_wordcount.hip")
    ctor = _body(g, "GpuWordCount::GpuWordCount(const JobConfig& cfg, u64 max_text_bytes, u64 max_lines)")
    assert "warm_first_job();" in ctor
    s = _src("csrc", "engine", "pipeline.hip")
    warm = _body(s, "void DevicePipeline::warm_first_job()")
    assert "lean_job(in)" in warm and "warming = true;" in warm and "run(in)" in warm
    for fn in ("void DevicePipeline::maybe_retune(const EntryList& e)",
               "void DevicePipeline::force_retune(const EntryList& e)",
               "void DevicePipeline::print_ord_trace()", "void DevicePipeline::print_map_trace()"):
        body = _body(s, fn)
        assert "warming" in body.split("\n", 3)[1] + body.split("\n", 3)[2], fn


@pytest.mark.gpu
def test_warm_up_job_with_letter_delimiters(hamlet):
    """The construction warm-up job picks a token byte outside the job's delimiter set: an
    engine whose delimiters include 'a' builds, and its jobs match the oracle."""
    import locust_amd as lc
    from locust_amd.utils import oracle

    delims = " ,.-;:'()\"\ta"
    cfg = lc.make_config("gpu", delimiters=delims)
    eng = lc._C.GpuEngine(cfg, len(hamlet), hamlet.count(b"\n") + 1)
    want = oracle.wordcount(hamlet, delims=delims.encode())[0]
    for _ in range(2):
        assert eng.run(hamlet).entries() == want
