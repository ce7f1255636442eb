"""One RCCL rank, synth1m, forced shuffle: the device exchange end to end (plan, pack,
all-to-all, merge, report, emit into the shared host output) next to the local job, per-job
times, host syncs and per-stage medians.  Run under rocprofv3 --kernel-trace --stats for
the kernel split.
    python tools/exch_prof.py [--jobs 30] [--lines 1000000]"""
import argparse
import os
import socket
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import locust_amd as lc  # noqa: E402


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=30)
    ap.add_argument("--lines", type=int, default=None)
    a = ap.parse_args()
    text = bench.synth_shard("synth1m", 0, 1, a.lines)
    job = lc.make_config("gpu", reduce_path="lds", combine=True,
                         chunk_bytes=bench.chunk_bytes_for(text.size))
    for strategy in ("shuffle", "gather"):
        dcfg = lc.make_dist_config(1, job, strategy=strategy)
        dr = lc._C.DistRank(dcfg, 0, "rccl", "127.0.0.1", free_port(), text.size, text.size, 60.0)
        dr.load_text(text, 0)
        times, syncs, info = [], [], None
        res = None
        for _ in range(a.jobs):
            t0 = time.perf_counter()
            res, info = dr.run_loaded()
            times.append((time.perf_counter() - t0) * 1e3)
            syncs.append(info["host_syncs"])
        print(f"{strategy}: first {times[0]:.3f} ms, second {times[1]:.3f} ms, median "
              f"{statistics.median(times[2:]):.4f} ms; syncs {syncs[:4]}; unique {res.num_unique}; "
              f"shuffle_ms {info['shuffle_ms']:.4f} reduce_ms {info['reduce_ms']:.4f} "
              f"output_bytes {info['output_bytes']}", flush=True)
        del dr
    # the same forced shuffle as a one-rank RCCL clique (ranks = threads of this process:
    # the shared output is one pinned allocation instead of a registered shm segment)
    raw = text.to_bytes()
    if raw:
        cfgs = [lc.make_dist_config(1, job, strategy="shuffle") for _ in range(a.jobs)]
        out = lc._C.run_multi_schedule(raw, cfgs, "rccl")
        tm = [i["total_ms"] for _, i in out]
        print(f"clique shuffle: first {tm[0]:.3f} ms, median {statistics.median(tm[2:]):.4f} ms; "
              f"syncs {[i['host_syncs'] for _, i in out][:4]}", flush=True)
    ms, stages, res = bench.bench_single(text, a.jobs, 3)
    print(f"local (one-rank auto): {ms:.4f} ms; unique {res.num_unique}", flush=True)


if __name__ == "__main__":
    main()
