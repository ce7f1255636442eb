#!/usr/bin/env python3
"""Headline benchmark: WordCount Map/Process/Reduce on MI355X (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--config hamlet4500|hamlet700|synth1m|synth10g]

One "step" is one complete WordCount job: H2D of the text, Map (tokenize/emit), Process
(compaction + radix sort), Reduce (boundary mark + head compaction + adjacent difference)
and D2H of the sorted (key, val, count) results -- the reference's timed stages
(main.cu:405-468) plus the transfers it leaves untimed.  The reference numbers are on a
GTX 1060 (README.md:72-88): 4,500-line whole-Hamlet LDS-reduce total 77.393 ms, 700-line
total 29.405 ms.

N = 1: one process, one GPU.  N > 1 (launched by torch.distributed.run, one process per
GPU, RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/MASTER_PORT from the env): weak scaling --
every rank maps its own copy of the text, then the ranks range-partition and shuffle the
map output with one RCCL all-to-all-v over xGMI, reduce their key range and gather the
globally sorted result on rank 0.  Steps are timed between barriers with the device
synchronised on both sides; the MAX over ranks is reported.

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
    line-aligned 4 MiB pieces, each mapped as it lands, and aggregates on the two-kernel
    ordered build); larger ones stream in 256 MiB chunks (PCIe-bound)."""
    return CHUNK_BYTES


def load_text(config: str) -> bytes:
    from locust_amd.utils import oracle

    with open(os.path.join(ROOT, "data", "hamlet.txt"), "rb") as f:
        hamlet = f.read()
    if config == "hamlet700":
        return oracle.window(hamlet, 0, 700)
    return hamlet


def synth_shard(config: str, rank: int, world: int):
    """This rank's part of the synthetic text, generated straight into pinned memory
    (strong scaling: the total is fixed, each of the N ranks owns 1/N of it)."""
    import locust_amd as lc

    spec = SYNTH[config]
    if spec["lines"]:
        total_blocks = -(-spec["lines"] // 1024)
        b0, b1 = rank * total_blocks // world, (rank + 1) * total_blocks // world
        lines = min(spec["lines"], b1 * 1024) - b0 * 1024
        return lc._C.HostText.generate(lines=lines, seed=1, first_block=b0)
    per = spec["bytes"] // world
    first = rank * -(-per // (1024 * 30))  # blocks are ~44 KB: shards never overlap
    return lc._C.HostText.generate(bytes=per, seed=1, first_block=first)


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
    nlines = text.count(b"\n") + (0 if text.endswith(b"\n") else 1)
    eng = lc._C.GpuEngine(cfg, len(text), nlines)
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


def cold_first_run(text: bytes) -> dict:
    """A fresh engine's first job (allocation excluded, first launches/captures included):
    the regime of the reference's numbers, which include Thrust's first-call overhead."""
    import locust_amd as lc

    if isinstance(text, bytes):
        cfg = lc.make_config("gpu", reduce_path="lds")
        nlines = text.count(b"\n") + (0 if text.endswith(b"\n") else 1)
        eng = lc._C.GpuEngine(cfg, len(text), nlines)
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
        nlines = text.count(b"\n") + (0 if text.endswith(b"\n") else 1)
        eng = lc._C.GpuEngine(cfg, len(text), nlines)
        eng.load(text)
        run = eng.run_loaded
    else:  # HostText (pinned; streamed when larger than one pass)
        eng = lc._C.GpuEngine(cfg, max(text.size, 1), max(text.size, 1))
        run = lambda: eng.run_text(text)  # noqa: E731
    for _ in range(warmup):
        res = run()
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


def bench_dist(text: bytes, steps: int, warmup: int, rank: int, world: int, local_rank: int,
               comm: str = "rccl"):
    import locust_amd as lc

    # comm="tcp" rehearses the multi-process path with several ranks on one GPU (RCCL
    # refuses two ranks per device); the benchmark itself always uses RCCL.
    device = local_rank if comm == "rccl" else 0
    job = lc.make_config("gpu", device=device, reduce_path="lds", combine=True,
                         chunk_bytes=chunk_bytes_for(len(text) if isinstance(text, bytes)
                                                     else text.size))
    dcfg = lc.make_dist_config(world, job)
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    from locust_amd.parallel import bootstrap_port, release_bootstrap_port

    port = bootstrap_port(rank, world)
    if isinstance(text, bytes):
        nbytes, nlines = len(text), text.count(b"\n") + (0 if text.endswith(b"\n") else 1)
    else:
        nbytes = nlines = max(text.size, 1)
    # RCCL prints its version banner on stdout during init; keep stdout for the one JSON
    # line the driver parses by pointing fd 1 at stderr while the communicator comes up.
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dr = lc._C.DistRank(dcfg, rank, comm, host, port, nbytes, nlines, 120.0)
        release_bootstrap_port()  # every rank connected inside the constructor
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    if isinstance(text, bytes):
        dr.load(text, 0)  # the shard sits in the engine's pinned buffer, like a loaded file
    else:
        dr.load_text(text, 0)
    return dr


def time_dist(dr, steps: int, warmup: int, strategy: str = "auto"):
    import locust_amd as lc

    dr.set_strategy(getattr(lc._C.DistStrategy, strategy))
    res = None
    for _ in range(warmup):  # holds each result like the timed loop (steady buffer pool)
        res, _info = dr.run_loaded()
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
    return ms, med, res, info["strategy"]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="hamlet4500",
                    choices=sorted(BASELINE_MS) + sorted(SYNTH))
    ap.add_argument("--no-extra", action="store_true", help="skip the 700-line side measurement")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "tcp"],
                    help="communicator for N>1 (tcp: rehearsal with ranks sharing one GPU)")
    ap.add_argument("--strategy", default="auto", choices=["auto", "shuffle", "gather"],
                    help="N>1: after-map strategy (auto: gather-to-root for small combined "
                         "outputs, sample-sort all-to-all shuffle otherwise)")
    ap.add_argument("--force-dist", action="store_true",
                    help="use the distributed path even for one rank")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world != 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    n = max(world, 1)

    synth = args.config in SYNTH
    if synth:
        t_gen = time.perf_counter()
        text = synth_shard(args.config, rank, n)
        print(f"rank {rank}: generated {text.size} B / {text.lines} lines in "
              f"{time.perf_counter() - t_gen:.1f} s", file=sys.stderr)
        nbytes, nlines = text.size, text.lines
    else:
        text = load_text(args.config)
        nbytes, nlines = len(text), text.count(b"\n") + (0 if text.endswith(b"\n") else 1)
    extra = {}
    strategy = None
    if n == 1 and not args.force_dist:
        if synth and not args.no_extra:
            extra["cold_start"] = cold_first_run(text)  # before any warm engine exists
        ms, stages, res = bench_single(text, args.steps, args.warmup)
        if not args.no_extra and args.config == "hamlet4500":
            ms700, st700, _ = bench_single(load_text("hamlet700"), args.steps, args.warmup)
            extra["hamlet700"] = {"ms_per_step": round(ms700, 4), "vs_baseline":
                                  round(ms700 / BASELINE_MS["hamlet700"], 6),
                                  "stages_ms": {k: round(v, 4) for k, v in st700.items()}}
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
    else:
        dr = bench_dist(text, args.steps, args.warmup, rank, world, local_rank, args.comm)
        ms, stages, res, strategy = time_dist(dr, args.steps, args.warmup, args.strategy)
        if not args.no_extra and args.strategy == "auto" and strategy != "shuffle":
            # The sample-sort all-to-all shuffle on the same job (the path large inputs
            # take), so every scaling run also records the all-to-all path.
            ks, kw = (args.steps, args.warmup) if not synth else (min(args.steps, 10),
                                                                  min(args.warmup, 3))
            try:  # a side measurement: its failure must not cost the headline line
                mss, sts, _, _ = time_dist(dr, ks, kw, "shuffle")
                extra["shuffle_path"] = {"ms_per_step": round(mss, 4),
                                         "stages_ms": {k: round(v, 4) for k, v in sts.items()}}
            except Exception as e:  # noqa: BLE001
                print(f"rank {rank}: shuffle extra failed: {e}", file=sys.stderr)
                extra["shuffle_path"] = {"error": str(e)[:300]}
    if rank != 0:
        return 0
    if synth:
        total_bytes = nbytes * n  # approximately: every rank's shard is the same size
        base = total_bytes / (REF_CHART_MB_PER_S * 1e6) * 1e3
        data = (f"synthetic Hamlet-shaped text (native generator, seed 1), "
                f"{'1M lines' if args.config == 'synth1m' else '10 GB'} in total, "
                f"1/N per GPU generated into pinned host memory")
        model = (f"WordCount {args.config}: dictionary path, "
                 + ("one pass, line-aligned upload pieces of up to 12 MiB, two-kernel ordered build"
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
        data = "hamlet.txt fixture (real text); N>1: every rank maps its own copy"
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
                                                           "shuffle": "alltoallv_shuffle",
                                                           "local": "one_rank_local"}[strategy]),
        },
        "baseline_ms": round(base, 3),
        "baseline_stages_ms": baseline_stages,
        "stages_ms_median": {k: round(v, 4) for k, v in stages.items()},
        "tokens": res.num_tokens,
        "unique": res.num_unique,
    }
    line.update(extra)
    print(json.dumps(line), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
