#!/usr/bin/env python3
"""Headline benchmark: WordCount Map/Process/Reduce on MI355X (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--config hamlet4500|hamlet700|synth1m|synth10g]

One "step" is one complete WordCount job: H2D of the text, Map (tokenize/emit), Process
(compaction + radix sort), Reduce (boundary mark + head compaction + adjacent difference)
and D2H of the sorted (key, count) results (val = the prefix of the counts, rebuilt on read) -- the reference's timed stages
(main.cu:405-468) plus the transfers it leaves untimed.  The reference numbers are on a
GTX 1060 (README.md:72-88): 4,500-line whole-Hamlet LDS-reduce total 77.393 ms, 700-line
total 29.405 ms.

Ranks.  N = 1: one process, one GPU.  N > 1: one process per GPU, RANK / WORLD_SIZE /
LOCAL_RANK / MASTER_ADDR / MASTER_PORT from the env -- either set by
``torch.distributed.run`` or, when ``--gpus N`` is given without a launcher, by this script
itself: the parent starts N child rank processes (never an exec, before any GPU call of
its own), relays rank 0's JSON line and fails if any rank fails.  A rank that cannot get a
GPU of its own fails the run: a job never silently reports fewer GPUs than asked for.

Headline (``value``): whole Hamlet, weak scaling -- every rank maps its own copy of the
text, the ranks merge their combined (key, count) records on rank 0 (the gather strategy:
one all-gather of device-written slots, one root merge).  The ``synth1m`` extra, at every
N including 1, is BASELINE config 4 as strong scaling: 1M synthetic lines in total, 1/N per
rank, range-partitioned by sample-sort splitters and exchanged over xGMI (one fixed-slot
``ncclAllToAll`` in steady state), every rank writing its key range into the shared host
output over its own PCIe link, so N = 1, 2, 4, 8 form one curve.  Steps are timed between
barriers with the device synchronised on both sides; the MAX over ranks is reported.

This process never imports torch: the engine drives HIP/RCCL directly (torch's bundled
HIP runtime must not be loaded next to the system one).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "WordCount ms (Map/Process/Reduce) at 700 & 4500 lines; 1/2/4/8-GPU scaling"
BASELINE_MS = {"hamlet4500": 77.393, "hamlet700": 29.405}  # README.md:74-76, 86-88 (GPU/LDS)
BASELINE_STAGES = {
    "hamlet4500": {"map_ms": 0.040, "process_ms": 73.015, "reduce_ms": 4.338},
    "hamlet700": {"map_ms": 0.047, "process_ms": 27.646, "reduce_ms": 1.712},
}
# Synthetic BASELINE configs (BASELINE.json configs 4 and 5).  The reference publishes no
# number at these sizes; its file-size chart (README.md:98) gives ~54 MB/s at 1 GB
# (18,390 ms), used here to derive a comparison point for the same byte count.
SYNTH = {
    "synth1m": {"lines": 1_000_000, "bytes": 0},
    "synth10g": {"lines": 0, "bytes": 10_000_000_000},
}
REF_CHART_MB_PER_S = 1e9 / 18.390 / 1e6  # ~54.4 MB/s
CHUNK_BYTES = 256 << 20  # one device pass; larger shards stream


def chunk_bytes_for(nbytes: int) -> int:
    """Device pass size: inputs up to 256 MiB are ONE pass (the engine uploads them in
    line-aligned pieces, each mapped as it lands, and aggregates on the two-kernel ordered
    build); larger ones stream in 256 MiB chunks (PCIe-bound)."""
    return CHUNK_BYTES


def load_text(config: str) -> bytes:
    from locust_amd.utils import oracle

    with open(os.path.join(ROOT, "data", "hamlet.txt"), "rb") as f:
        hamlet = f.read()
    if config == "hamlet700":
        return oracle.window(hamlet, 0, 700)
    return hamlet


def synth_shard(config: str, rank: int, world: int, lines: int | None = None,
                nbytes: int | None = None):
    """This rank's part of the synthetic text, generated straight into pinned memory
    (strong scaling: the total is fixed, each of the N ranks owns 1/N of it).  `lines` /
    `nbytes` scale a config down (tests: --synth-lines, --synth-bytes)."""
    import locust_amd as lc

    spec = dict(SYNTH[config])
    if lines:
        spec = {"lines": lines, "bytes": 0}
    elif nbytes and not spec["lines"]:
        spec = {"lines": 0, "bytes": nbytes}
    if spec["lines"]:
        total_blocks = -(-spec["lines"] // 1024)
        b0, b1 = rank * total_blocks // world, (rank + 1) * total_blocks // world
        nl = min(spec["lines"], b1 * 1024) - b0 * 1024
        return lc._C.HostText.generate(lines=max(nl, 0), seed=1, first_block=b0)
    per = spec["bytes"] // world
    first = rank * -(-per // (1024 * 30))  # blocks are ~44 KB: shards never overlap
    return lc._C.HostText.generate(bytes=per, seed=1, first_block=first)


def _nlines(text: bytes) -> int:
    return text.count(b"\n") + (0 if text.endswith(b"\n") else 1)


def bench_single(text, steps: int, warmup: int, sort: str = "dict", graph: int = -1):
    """Whole-job time of `steps` back-to-back jobs, plus the median per-stage split from a
    short run with per-stage device events (graph=0).  The timed jobs carry no stage
    timestamps: small ones are lean direct launches with a polled completion word, and
    events would cost them more than a stage takes; timed_* are their own medians."""
    ms, gst, res = _time_single(text, steps, warmup, sort, graph)
    _, stages, _ = _time_single(text, min(steps, 30), min(warmup, 5), sort, 0)
    stages["timed_gpu_ms"] = gst["gpu_ms"]
    stages["timed_wall_ms"] = gst["wall_ms"]
    return ms, stages, res


def ref_semantics(text: bytes, steps: int = 50, warmup: int = 5):
    """Median Map / Process / Reduce with host timers where the reference took them
    (main.cu:405-468): the same semantics as its published GTX 1060 numbers."""
    import locust_amd as lc

    cfg = lc.make_config("gpu", reduce_path="lds", graph=0, ref_timers=True)
    eng = lc._C.GpuEngine(cfg, len(text), _nlines(text))
    eng.load(text)
    for _ in range(warmup):
        eng.run_loaded()
    acc = {"ref_map_ms": [], "ref_process_ms": [], "ref_reduce_ms": []}
    for _ in range(steps):
        t = eng.run_loaded().times()
        for k in acc:
            acc[k].append(t[k])
    med = {k[4:]: round(statistics.median(v), 4) for k, v in acc.items()}
    med["total_ms"] = round(sum(med.values()), 4)
    return med


BASELINE_CPU = {"map_ms": 2.333, "process_ms": 23.699, "reduce_ms": 1.100}  # README.md:74-76


def cpu_path(text: bytes, steps: int = 20, warmup: int = 3) -> dict:
    """BASELINE config 1: the CPU reference pipeline (single thread: tokenize, std::sort,
    linear reduce -- the reference's GPU_IMPLEMENTATION 0 build, main.cu:489-527), median
    stage times of `steps` runs against the reference's CPU column (700 lines)."""
    import locust_amd as lc

    cfg = lc.make_config("cpu")
    for _ in range(warmup):
        lc._C.cpu_run(cfg, text)
    acc = {"map_ms": [], "process_ms": [], "reduce_ms": [], "wall_ms": []}
    for _ in range(steps):
        t = lc._C.cpu_run(cfg, text).times()
        for k in acc:
            acc[k].append(t[k])
    return {k: round(statistics.median(v), 4) for k, v in acc.items()}


def cold_first_run(text) -> dict:
    """A fresh engine's first job (allocation excluded, first launches included): the
    regime of the reference's numbers, which include Thrust's first-call overhead -- and of
    every `./MapReduce <file>` invocation, which runs one job per process."""
    import locust_amd as lc

    if isinstance(text, bytes):
        cfg = lc.make_config("gpu", reduce_path="lds")
        eng = lc._C.GpuEngine(cfg, len(text), _nlines(text))
        eng.load(text)
        run = eng.run_loaded
    else:  # HostText: the synthetic configs (a cold partition map on a large vocabulary)
        cfg = lc.make_config("gpu", reduce_path="lds", chunk_bytes=chunk_bytes_for(text.size))
        eng = lc._C.GpuEngine(cfg, max(text.size, 1), max(text.size, 1))
        run = lambda: eng.run_text(text)  # noqa: E731
    t = [time.perf_counter()]
    for _ in range(3):
        run()
        t.append(time.perf_counter())
    return {"first_job_ms": round((t[1] - t[0]) * 1e3, 4), "second_job_ms": round((t[2] - t[1]) * 1e3, 4),
            "third_job_ms": round((t[3] - t[2]) * 1e3, 4)}


def _time_single(text, steps: int, warmup: int, sort: str, graph: int):
    import locust_amd as lc

    size = len(text) if isinstance(text, bytes) else text.size
    cfg = lc.make_config("gpu", reduce_path="lds", sort=sort, chunk_bytes=chunk_bytes_for(size),
                         graph=graph)
    if isinstance(text, bytes):
        eng = lc._C.GpuEngine(cfg, len(text), _nlines(text))
        eng.load(text)
        run = eng.run_loaded
    else:  # HostText (pinned; streamed when larger than one pass)
        eng = lc._C.GpuEngine(cfg, max(text.size, 1), max(text.size, 1))
        run = lambda: eng.run_text(text)  # noqa: E731
    for _ in range(warmup):
        res = run()
    # the end of the warmup: the partition map's retune from the first job's output runs on
    # the engine's worker thread; take it now rather than a few timed jobs in (a short
    # warmup -- the driver's is 5 jobs -- can end before the worker does)
    if warmup:
        eng.partition_map()
    # The timed loop is the jobs alone (each returns its complete result object); the
    # per-stage bookkeeping is a separate pass so the harness is not inside the timing.
    t0 = time.perf_counter()
    for _ in range(steps):
        res = run()
    t1 = time.perf_counter()
    ms = (t1 - t0) * 1e3 / steps
    stage = {"map_ms": [], "process_ms": [], "reduce_ms": [], "h2d_ms": [], "d2h_ms": [],
             "gpu_ms": [], "wall_ms": []}
    for _ in range(min(steps, 50)):
        t = run().times()
        for k in stage:
            stage[k].append(t[k])
    med = {k: statistics.median(v) for k, v in stage.items()}
    return ms, med, res


def untuned(text: bytes, steps: int, warmup: int) -> dict:
    """The headline job with the partition map's between-job retuning switched off
    (LOCUST_PART_TUNE=0): every job balances its partitions from its own map statistics
    only, like the one job of a `./MapReduce <file>` process."""
    old = os.environ.get("LOCUST_PART_TUNE")
    os.environ["LOCUST_PART_TUNE"] = "0"
    try:
        ms, _st, _res = _time_single(text, steps, warmup, "dict", -1)
    finally:
        if old is None:
            os.environ.pop("LOCUST_PART_TUNE", None)
        else:
            os.environ["LOCUST_PART_TUNE"] = old
    return {"ms_per_step": round(ms, 4)}


# ---------------------------------------------------------------------------------------
# multi-rank
# ---------------------------------------------------------------------------------------
def dist_rank(text, world: int, rank: int, local_rank: int, comm: str, backend: str):
    """This process's DistRank (communicator + engine for `text`), bootstrapped through
    rank 0's listening socket (inherited from a launcher, or bound here)."""
    import locust_amd as lc
    from locust_amd.parallel import connect_rank

    # comm="tcp" rehearses the multi-process path with several ranks on one GPU (RCCL
    # refuses two ranks per device); the benchmark itself uses RCCL.
    device = local_rank if comm == "rccl" else 0
    job = lc.make_config(backend, device=device, reduce_path="lds", combine=True,
                         chunk_bytes=chunk_bytes_for(len(text) if isinstance(text, bytes)
                                                     else text.size))
    dcfg = lc.make_dist_config(world, job)
    nbytes, nlines = _shape(text)
    # RCCL prints its version banner on stdout during init; keep stdout for the one JSON
    # line the driver parses by pointing fd 1 at stderr while the communicator comes up.
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dr = connect_rank(dcfg, rank, world, comm, nbytes, nlines, 120.0)
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    _load(dr, text)
    return dr


def _shape(text):
    if isinstance(text, bytes):
        return max(len(text), 1), max(_nlines(text), 1)
    return max(text.size, 1), max(text.size, 1)


def _load(dr, text) -> None:
    if isinstance(text, bytes):
        dr.load(text, 0)  # the shard sits in the engine's pinned buffer, like a loaded file
    else:
        dr.load_text(text, 0)


def time_dist(dr, steps: int, warmup: int, strategy: str = "auto"):
    import locust_amd as lc

    dr.set_strategy(getattr(lc._C.DistStrategy, strategy))
    res = None
    stamp(f"{strategy}:warmup")
    for _ in range(warmup):  # holds each result like the timed loop (steady buffer pool)
        res, _info = dr.run_loaded()
    stamp(f"{strategy}:timed")
    parts = {"map_ms": [], "shuffle_ms": [], "reduce_ms": [], "gather_ms": [],
             "sent_bytes": [], "recv_bytes": []}
    infos = []
    dr.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        res, info = dr.run_loaded()
        infos.append(info)
    dr.barrier()
    t1 = time.perf_counter()
    for info in infos:
        for k in parts:
            parts[k].append(info[k])
    mine = (t1 - t0) * 1e3 / steps
    ms = dr.allreduce_max(mine)
    med = {k: statistics.median(v) for k, v in parts.items()}
    _LAST_INFOS[:] = infos  # the timed jobs' per-rank records, for scale_diag
    return ms, med, res, info["strategy"]


_LAST_INFOS: list = []


# ---------------------------------------------------------------------------------------
# progress stamps and the watchdog: a run that hangs still ends with
# ONE JSON line, inside the budget, saying where every rank was
# ---------------------------------------------------------------------------------------
_PARTIAL: dict = {}  # what rank 0 has measured so far (scale_diag, ...) for a failure line
DEFAULT_BUDGET_S = 480.0  # below the driver's timeout for one N of the scaling run


def progress_dir() -> str:
    """Where the ranks of this run stamp their progress: LOCUST_PROGRESS_DIR (set by the
    self-spawning parent), else a directory named after the rendezvous (MASTER_PORT and
    torchrun's run id), so every rank of one run -- and only of it -- shares it."""
    d = os.environ.get("LOCUST_PROGRESS_DIR")
    if not d:
        tag = f"{os.environ.get('MASTER_PORT', 'local')}_{os.environ.get('TORCHELASTIC_RUN_ID', '')}"
        d = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"locust_bench_progress_{tag}")
    os.makedirs(d, exist_ok=True)
    return d


_STAGE = ["start", 0.0]  # this rank's last Python stage and when it was entered


def _native_stage():
    try:
        import locust_amd as lc

        return list(lc._C.native_stage())
    except Exception:  # noqa: BLE001 -- no extension yet (or built without it)
        return None


def stamp(stage: str | None = None) -> None:
    """This rank's last stage and when it got there, the distributed job stage its native
    code last entered, and a heartbeat time (atomic replace of rank<r>.json).  stage=None:
    a heartbeat only (the watchdog thread, every second)."""
    rank = int(os.environ.get("RANK", "0"))
    if stage is not None:
        _STAGE[:] = [stage, time.time()]
    try:
        d = progress_dir()
        tmp = os.path.join(d, f".rank{rank}.{os.getpid()}")
        with open(tmp, "w") as f:
            json.dump({"rank": rank, "stage": _STAGE[0], "t": _STAGE[1], "beat": time.time(),
                       "native": _native_stage() if "locust_amd" in sys.modules else None,
                       "pid": os.getpid()}, f)
        os.replace(tmp, os.path.join(d, f"rank{rank}.json"))
    except OSError:
        pass  # diagnostics only


def read_progress(world: int, d: str | None = None) -> dict:
    d = d or progress_dir()
    now = time.time()
    out = {}
    for r in range(world):
        try:
            with open(os.path.join(d, f"rank{r}.json")) as f:
                x = json.load(f)
            out[str(r)] = {"stage": x["stage"], "age_s": round(now - x["t"], 1),
                           # the native job stage it last entered and how many so far
                           "native_stage": (x.get("native") or [None])[0],
                           "native_stages": (x.get("native") or [None, None])[1],
                           # seconds since its watchdog thread last wrote: a live process
                           # (stuck) beats every second, a dead one stops
                           "heartbeat_age_s": round(now - x.get("beat", x["t"]), 1)}
        except (OSError, ValueError, KeyError):
            out[str(r)] = {"stage": None, "age_s": None}
    return out


def failure_line(world: int, reason: str, d: str | None = None) -> str:
    """The one JSON line of a failed run: no value, the reason, every rank's last stage
    and whatever rank 0 had measured (its scale_diag, when it got that far)."""
    line = {"metric": METRIC, "value": None, "unit": "ms", "n_gpus": world,
            "higher_is_better": False, "status": "failed", "reason": reason,
            "progress": read_progress(world, d)}
    line.update({k: v for k, v in _PARTIAL.items() if k not in line})
    return json.dumps(line)


def start_watchdog(budget_s: float, rank: int, world: int) -> None:
    """On expiry rank 0 prints the failure line and every rank exits 124 (rank 0 first: its
    line must be out before the launcher tears the job down).  os._exit, never an exec."""
    import threading

    if budget_s <= 0:
        return
    deadline = time.time() + budget_s + (0 if rank == 0 else 20)

    def run():
        while time.time() < deadline:
            time.sleep(1.0)
            stamp()  # heartbeat (and the native stage the job is in)
        if rank == 0:
            try:
                print(failure_line(world, f"watchdog: the {budget_s:.0f} s budget expired"),
                      flush=True)
            except Exception:  # noqa: BLE001 -- the exit below must happen regardless
                pass
        print(f"bench: rank {rank}: watchdog budget expired at stage "
              f"{read_progress(world).get(str(rank), {}).get('stage')}", file=sys.stderr,
              flush=True)
        os._exit(124)

    threading.Thread(target=run, daemon=True, name="bench-watchdog").start()


# ---------------------------------------------------------------------------------------
# N > 1: a self-diagnosing line
# ---------------------------------------------------------------------------------------
def nccl_debug_setup() -> str | None:
    """RCCL's INFO log into per-process files (never stdout, which carries the JSON line),
    so every rank can read which transport each of its peer pairs uses.  Must run before
    the communicator exists (RCCL reads the variables at init).  A user's NCCL_DEBUG_FILE
    wins (the log then goes where they said, and the transports are not parsed)."""
    if "NCCL_DEBUG_FILE" in os.environ:
        return None
    import tempfile

    d = os.path.join(tempfile.gettempdir(),
                     f"locust_nccl_{os.environ.get('MASTER_PORT', '0')}_{os.getuid()}")
    os.makedirs(d, exist_ok=True)
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT,GRAPH,P2P,SHM,NET")
    os.environ["NCCL_DEBUG_FILE"] = os.path.join(d, "nccl.%h.%p.log")
    return d


def nccl_transports(d: str | None, rank: int) -> dict:
    """{peer rank: sorted transports} of this process's channels, from its RCCL INFO log
    ("Channel 00/0 : 0[0] -> 1[1] via P2P/IPC")."""
    import glob
    import re

    if not d:
        return {}
    pat = re.compile(r"Channel \d+/\d+ ?: +(\d+)\[[^\]]*\] -> (\d+)\[[^\]]*\] via (\S.*?)\s*$")
    out: dict = {}
    for f in glob.glob(os.path.join(d, f"nccl.*.{os.getpid()}.log")):
        with open(f, errors="replace") as fh:
            for ln in fh:
                m = pat.search(ln)
                if m and int(m.group(1)) == rank:
                    out.setdefault(m.group(2), set()).add(m.group(3))
    return {k: sorted(v) for k, v in sorted(out.items(), key=lambda kv: int(kv[0]))}


def _rss_breakdown() -> dict:
    """Resident memory now, by kind (/proc/self/status, kB): anonymous, file-backed (device
    memory the GPU driver maps into the process counts here), shared."""
    out = {}
    try:
        with open("/proc/self/status") as f:
            for ln in f:
                k, _, v = ln.partition(":")
                if k in ("VmRSS", "RssAnon", "RssFile", "RssShmem"):
                    out[k] = int(v.split()[0])
    except OSError:
        pass
    return out


def scale_diag(dr, args, local_rank: int, nccl_dir: str | None, infos=None) -> dict:
    """Every rank's view of the last timed jobs, gathered to all ranks: per-rank stage
    medians (map / exchange / merge / emit), bytes sent to and received from each peer,
    its GPU's direct-access row and RCCL's transport per peer, and its peak RSS.  The
    summary gives the min / max over ranks of each stage."""
    import resource
    import socket

    infos = infos if infos is not None else list(_LAST_INFOS)
    names = {"map": "map_ms", "exchange": "shuffle_ms", "merge": "reduce_ms", "emit": "gather_ms"}
    device = local_rank if args.comm == "rccl" else 0
    mine = {
        "rank": dr.rank, "host": socket.gethostname(), "pid": os.getpid(),
        "device": device if args.backend == "gpu" else None,
        "stages_ms": {k: round(statistics.median(i[v] for i in infos), 4) if infos else None
                      for k, v in names.items()},
        "sent_to": infos[-1]["sent_to"] if infos else [],
        "recv_from": infos[-1]["recv_from"] if infos else [],
        "peak_rss_kb": resource.getrusage(resource.RUSAGE_SELF).ru_maxrss,
        "rss_now_kb": _rss_breakdown(),
        "pinned_bytes": infos[-1].get("pinned_bytes", 0) if infos else 0,
        # the HBM plan's outcome: this rank's engine device memory, its GPU's free / total
        # memory when the engine was built (plan_device_pass, csrc/include/locust/engine.hpp)
        "hbm_device_bytes": infos[-1].get("hbm_device_bytes", 0) if infos else 0,
        "hbm_free_bytes": infos[-1].get("hbm_free_bytes", 0) if infos else 0,
        "hbm_total_bytes": infos[-1].get("hbm_total_bytes", 0) if infos else 0,
        "comm": dr.comm_name,
        "transport": nccl_transports(nccl_dir, dr.rank) if args.comm == "rccl" else
                     {str(p): [args.comm] for p in range(dr.size) if p != dr.rank},
    }
    if args.backend == "gpu":
        import locust_amd as lc

        mine["peer_access_row"] = list(lc._C.peer_access_row(device))
    ranks = [json.loads(b) for b in dr.allgather_bytes(json.dumps(mine).encode())]
    for r in ranks:  # the access row in rank terms: can rank r's GPU reach rank q's directly
        row = r.pop("peer_access_row", None)
        r["peer_access"] = ([None if q["device"] == r["device"] else row[q["device"]]
                             for q in ranks] if row is not None else None)
    summary = {}
    for k in names:
        v = [r["stages_ms"][k] for r in ranks if r["stages_ms"][k] is not None]
        summary[k] = [min(v), max(v)] if v else None
    return {"stages_ms_min_max": summary, "ranks": ranks,
            "nccl_debug_dir": nccl_dir, "peak_rss_kb_max": max(r["peak_rss_kb"] for r in ranks),
            "hbm_device_bytes_max": max(r["hbm_device_bytes"] for r in ranks)}


def synth_point(args, rank: int, world: int, dr=None) -> dict:
    """BASELINE config 4 (1M synthetic lines) as one point of the strong-scaling curve:
    the total is fixed, this rank owns 1/N of it.  N = 1: the single-GPU engine (a
    one-rank job is the local pipeline); N > 1: a second engine on the ranks'
    communicator, exchanged with the sample-sort all-to-all."""
    t_gen = time.perf_counter()
    text = synth_shard("synth1m", rank, world, args.synth_lines)
    gen_s = time.perf_counter() - t_gen
    steps, warmup = min(args.steps, 20), min(args.warmup, 3)
    lines = args.synth_lines or SYNTH["synth1m"]["lines"]
    if dr is None:
        ms, stages, res = bench_single(text, steps, warmup)
        strategy, total_bytes = "local", text.size
    else:
        nbytes, nlines = _shape(text)
        dr.use_engine(dr.add_engine(nbytes, nlines))
        _load(dr, text)
        ms, stages, res, strategy = time_dist(dr, steps, warmup, "auto")
        synth_infos = list(_LAST_INFOS)
        sizes = [0.0] * world
        total_bytes = int(sum(_allgather_float(dr, float(text.size), sizes)))
        dr.use_engine(0)
    point = {"lines": lines, "n_gpus": world, "ms_per_step": round(ms, 4),
            "GB_per_s": round(total_bytes / (ms * 1e-3) / 1e9, 3), "bytes": total_bytes,
            "strategy": strategy, "tokens": res.num_tokens if rank == 0 else None,
            "unique": res.num_unique if rank == 0 else None, "gen_s": round(gen_s, 2),
            "output_bytes_per_key": (round(res.wire_bytes / max(res.num_unique, 1), 2)
                                     if rank == 0 else None),
            "stages_ms": {k: round(v, 4) for k, v in stages.items()}}
    if dr is not None:
        d = scale_diag(dr, args, int(os.environ.get("LOCAL_RANK", "0")), None, synth_infos)
        point["diag"] = {"stages_ms_min_max": d["stages_ms_min_max"],
                         "sent_to": [r["sent_to"] for r in d["ranks"]],
                         "recv_from": [r["recv_from"] for r in d["ranks"]]}
    return point


def _allgather_float(dr, v: float, out: list) -> list:
    # allreduce_max is the only float collective the binding has: sum via N max-rounds
    # would be silly; every rank's shard size is the same to within one 1,024-line block,
    # so rank r's size is gathered by masking: max over ranks of (v if r == me else 0).
    for r in range(len(out)):
        out[r] = dr.allreduce_max(v if r == dr.rank else 0.0)
    return out


# ---------------------------------------------------------------------------------------
# self-spawned ranks (--gpus N without a launcher)
# ---------------------------------------------------------------------------------------
def spawn_ranks(n: int, argv: list[str], budget_s: float = DEFAULT_BUDGET_S) -> int:
    """Start N rank processes of this script and relay rank 0's JSON line.  The parent
    never touches the GPU (children, never an exec).  The first failing rank stops the
    run: the others are killed, ONE failure line (status "failed", every rank's last
    progress stamp, what rank 0 had measured) is printed and its exit code returned.  A
    parent watchdog ends a run that outlives the ranks' own budget the same way."""
    import signal
    import socket
    import subprocess
    import tempfile
    import threading

    pdir = tempfile.mkdtemp(prefix="locust_bench_progress_")
    deadline = time.time() + budget_s + 40 if budget_s > 0 else None
    reason = ""

    boot = socket.socket()  # the bootstrap listener, inherited by rank 0 (no port race)
    boot.bind(("127.0.0.1", 0))
    boot.listen(n)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        master_port = s.getsockname()[1]
    procs = []
    out0: list[bytes] = []
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                       LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=str(master_port), LOCUST_PORT=str(boot.getsockname()[1]),
                       LOCUST_PROGRESS_DIR=pdir)
            env.pop("LOCUST_LISTEN_FD", None)
            fds: tuple = ()
            if r == 0:
                env["LOCUST_LISTEN_FD"] = str(boot.fileno())
                fds = (boot.fileno(),)
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv],
                                          env=env, pass_fds=fds, start_new_session=True,
                                          stdout=subprocess.PIPE if r == 0 else sys.stderr))
    finally:
        boot.close()
    reader = threading.Thread(target=lambda: out0.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    failed = 0
    while True:
        alive = False
        for r, p in enumerate(procs):
            rc = p.poll()
            if rc is None:
                alive = True
            elif rc != 0 and not failed:
                failed = rc if rc > 0 else 128 - rc
                reason = f"rank {r} failed with exit code {rc}"
                print(f"bench: {reason}", file=sys.stderr)
        if failed or not alive:
            break
        if deadline and time.time() > deadline:
            failed, reason = 124, f"parent watchdog: the ranks outlived {budget_s + 40:.0f} s"
            print(f"bench: {reason}", file=sys.stderr)
            break
        time.sleep(0.05)
    for p in procs:
        if p.poll() is None:
            for sig in (signal.SIGTERM, signal.SIGKILL):
                try:
                    os.killpg(p.pid, sig)
                    p.wait(timeout=5)
                    break
                except (ProcessLookupError, subprocess.TimeoutExpired):
                    continue
        p.wait()
    reader.join(timeout=10)
    lines = [ln for ln in b"".join(out0).decode(errors="replace").splitlines() if ln.strip()]
    if failed:
        # rank 0's own failure line (its watchdog) if it printed one, else one made here
        mine = [ln for ln in lines if '"status": "failed"' in ln]
        print(mine[-1] if mine else failure_line(n, reason, pdir), flush=True)
        return failed
    if not lines:
        print("bench: rank 0 printed no result line", file=sys.stderr)
        print(failure_line(n, "rank 0 printed no result line", pdir), flush=True)
        return 1
    print(lines[-1], flush=True)
    return 0


def visible_gpus() -> int:
    import locust_amd as lc

    return lc._C.device_count()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="hamlet4500",
                    choices=sorted(BASELINE_MS) + sorted(SYNTH))
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the side measurements (700 lines, radix path, synth1m, ...)")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "tcp", "tcpdev"],
                    help="communicator for N>1 (tcp: rehearsal with ranks sharing one GPU)")
    ap.add_argument("--backend", default="gpu", choices=["gpu", "cpu"],
                    help="cpu: rehearse the rank/communicator plumbing with the CPU engine")
    ap.add_argument("--strategy", default="auto", choices=["auto", "shuffle", "gather"],
                    help="N>1: after-map strategy (auto: gather-to-root for small combined "
                         "outputs, sample-sort all-to-all shuffle otherwise)")
    ap.add_argument("--force-dist", action="store_true",
                    help="use the distributed path even for one rank")
    ap.add_argument("--synth-lines", type=int, default=0,
                    help="lines of the synth1m strong-scaling extra (default 1M; tests)")
    ap.add_argument("--synth-bytes", type=int, default=0,
                    help="total bytes of --config synth10g (default 10 GB; tests)")
    ap.add_argument("--budget-s", type=float,
                    default=float(os.environ.get("LOCUST_BENCH_BUDGET_S", DEFAULT_BUDGET_S)),
                    help="watchdog: a run still going after this many seconds ends with one "
                         "failure line (status 'failed', every rank's last stage); 0: off")
    args = ap.parse_args()
    if args.backend == "cpu" and args.comm == "rccl" and args.gpus > 1:
        ap.error("--backend cpu needs --comm tcp")

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus, sys.argv[1:], args.budget_s)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    stamp("start")
    start_watchdog(args.budget_s, rank, world)
    if args.backend == "gpu" and args.comm == "rccl":
        # this rank's process on its GPU's NUMA node before the first GPU call (the pinned
        # shard is first touched there; locust_amd/parallel/numa.py)
        from locust_amd.parallel.numa import bind_to_gpu

        bind_to_gpu(local_rank)
    if args.gpus != world:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a "
              f"different GPU count than asked for", file=sys.stderr)
        return 2
    n = world
    if args.backend == "gpu":
        have = visible_gpus()
        need = (local_rank + 1) if args.comm == "rccl" else 1
        if have < need:
            print(f"bench: rank {rank} needs GPU {need - 1} but {have} visible "
                  f"(--gpus {n} --comm {args.comm})", file=sys.stderr)
            return 3

    synth = args.config in SYNTH
    if synth:
        t_gen = time.perf_counter()
        text = synth_shard(args.config, rank, n, nbytes=args.synth_bytes)
        print(f"rank {rank}: generated {text.size} B / {text.lines} lines in "
              f"{time.perf_counter() - t_gen:.1f} s", file=sys.stderr)
        nbytes, nlines = text.size, text.lines
    else:
        text = load_text(args.config)
        nbytes, nlines = len(text), _nlines(text)
    extra: dict = {}
    strategy = None
    rccl_ranks = None
    cpu = args.backend == "cpu"
    if n == 1 and not args.force_dist and cpu:
        c = cpu_path(text, args.steps, args.warmup)
        ms, stages = c["wall_ms"], c
        import locust_amd as lc

        res = lc._C.cpu_run(lc.make_config("cpu"), text)
    elif n == 1 and not args.force_dist:
        stamp("single:headline")
        if synth and not args.no_extra:
            extra["cold_start"] = cold_first_run(text)  # before any warm engine exists
        ms, stages, res = bench_single(text, args.steps, args.warmup)
        _PARTIAL["partial"] = {"ms_per_step": round(ms, 4)}
        stamp("single:extras")
        if not args.no_extra and args.config == "hamlet4500":
            ms700, st700, _ = bench_single(load_text("hamlet700"), args.steps, args.warmup)
            extra["hamlet700"] = {"ms_per_step": round(ms700, 4), "vs_baseline":
                                  round(ms700 / BASELINE_MS["hamlet700"], 6),
                                  "stages_ms": {k: round(v, 4) for k, v in st700.items()}}
            extra["untuned"] = untuned(text, args.steps, args.warmup)
            # The reference's own algorithm on the device: sort every token (LSD radix),
            # boundary-mark + compact + adjacent-difference (reported, not the headline).
            msr, str_, _ = bench_single(text, args.steps, args.warmup, sort="radix")
            extra["radix_path"] = {"ms_per_step": round(msr, 4),
                                   "stages_ms": {k: round(v, 4) for k, v in str_.items()}}
            # Host timers placed like the reference's (launch-only map, B2/B4): the
            # like-for-like comparison with BASELINE.md's per-stage rows.
            extra["cold_start"] = {"hamlet4500": cold_first_run(text),
                                   "hamlet700": cold_first_run(load_text("hamlet700"))}
            extra["reference_semantics_ms"] = {
                "hamlet4500": ref_semantics(text), "hamlet700": ref_semantics(load_text("hamlet700")),
                "baseline": BASELINE_STAGES}
            c700 = cpu_path(load_text("hamlet700"))
            extra["cpu_path"] = {
                "note": "BASELINE config 1: CPU reference pipeline, one thread, no GPU",
                "hamlet700_ms": c700, "hamlet4500_ms": cpu_path(text),
                "baseline_hamlet700_ms": dict(BASELINE_CPU, total_ms=27.132),
                "vs_baseline_hamlet700": round(c700["wall_ms"] / 27.132, 4)}
            extra["synth1m"] = synth_point(args, rank, n)
    else:
        nccl_dir = nccl_debug_setup() if args.comm == "rccl" else None
        stamp("connect")
        dr = dist_rank(text, n, rank, local_rank, args.comm, args.backend)
        rccl_ranks = dr.comm_count if dr.comm_name == "rccl" else None
        stamp("headline")
        ms, stages, res, strategy = time_dist(dr, args.steps, args.warmup, args.strategy)
        _PARTIAL["partial"] = {"ms_per_step": round(ms, 4), "strategy": strategy}
        stamp("scale_diag")
        extra["scale_diag"] = scale_diag(dr, args, local_rank, nccl_dir)
        _PARTIAL["scale_diag"] = extra["scale_diag"]
        if not args.no_extra and args.strategy == "auto" and strategy != "shuffle":
            # The sample-sort all-to-all shuffle on the same job (the path large inputs
            # take), so every scaling run also records the all-to-all path.
            ks, kw = (args.steps, args.warmup) if not synth else (min(args.steps, 10),
                                                                  min(args.warmup, 3))
            stamp("extra:shuffle")
            try:  # a side measurement: its failure must not cost the headline line
                mss, sts, _, _ = time_dist(dr, ks, kw, "shuffle")
                extra["shuffle_path"] = {"ms_per_step": round(mss, 4),
                                         "stages_ms": {k: round(v, 4) for k, v in sts.items()}}
            except Exception as e:  # noqa: BLE001
                print(f"rank {rank}: shuffle extra failed: {e}", file=sys.stderr)
                extra["shuffle_path"] = {"error": str(e)[:300]}
        if not args.no_extra and not synth:
            stamp("extra:synth1m")
            extra["synth1m"] = synth_point(args, rank, n, dr)
    stamp("done")
    if rank != 0:
        return 0
    if synth:
        total_bytes = nbytes * n  # approximately: every rank's shard is the same size
        base = total_bytes / (REF_CHART_MB_PER_S * 1e6) * 1e3
        data = (f"synthetic Hamlet-shaped text (native generator, seed 1), "
                f"{'1M lines' if args.config == 'synth1m' else f'{total_bytes / 1e9:.3g} GB'} in total, "
                f"1/N per GPU generated into pinned host memory")
        model = (f"WordCount {args.config}: dictionary path, "
                 + ("one pass, line-aligned upload pieces of 10 MiB (LOCUST_PIECE_MB), two-kernel ordered build"
                    if nbytes <= CHUNK_BYTES else
                    f"streamed in {chunk_bytes_for(nbytes) >> 20} MiB chunks")
                 + ", full H2D->D2H job per step")
        scaling = "strong"
        extra["GB_per_s"] = round(total_bytes / (ms * 1e-3) / 1e9, 3)
        extra["baseline_note"] = ("no published number at this size; baseline_ms = this byte "
                                  "count at the reference's ~54 MB/s file-size-chart rate "
                                  "(README.md:98, 1 GB in 18,390 ms)")
        baseline_stages = None
    else:
        base = BASELINE_MS[args.config]
        data = ("hamlet.txt fixture (real text); N>1: every rank maps its own copy; "
                "synth1m extra: synthetic text (native generator, seed 1)")
        model = (f"WordCount {args.config} ({nlines} lines/GPU): byte-parallel map + "
                 "ordered-dictionary Process+Reduce (one kernel: LDS hash aggregate, in-LDS "
                 "sort of distinct keys, look-back val offsets), full H2D->D2H job per step"
                 + ("" if n == 1 else "; ranks merged on rank 0"))
        scaling = "weak"
        baseline_stages = BASELINE_STAGES[args.config]
    line = {
        "metric": METRIC,
        "value": round(ms, 4),
        "unit": "ms",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": False,
        "scaling": scaling,
        "vs_baseline": round(ms / base, 6),
        "dtype": "int (u8 text, u64 packed keys/counts)",
        "data": data,
        "config": {
            "model": model,
            "global_batch": nlines * n,
            "seq_len": nbytes,
            "parallelism": f"dp{n}" + ("" if strategy is None else
                                       f"+{args.comm}_" + {"gather": "gather_merge",
                                                           "shuffle": "alltoall_shuffle",
                                                           "local": "one_rank_local"}[strategy]),
        },
        "baseline_ms": round(base, 3),
        "baseline_stages_ms": baseline_stages,
        "stages_ms_median": {k: round(v, 4) for k, v in stages.items()},
        "tokens": res.num_tokens,
        "unique": res.num_unique,
        # bytes the device wrote into host memory per result key (compact records: a header
        # word + the key's non-zero words; 40 for the 40-B record paths)
        "output_bytes_per_key": round(res.wire_bytes / max(res.num_unique, 1), 2),
        "rccl_ranks": rccl_ranks,
    }
    if cpu:
        line["backend"] = "cpu (rehearsal of the rank plumbing; not a GPU number)"
    line.update(extra)
    print(json.dumps(line), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
