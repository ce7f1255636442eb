"""Host memory (RSS) of streaming engines in one process, as `MapReduce <file> --gpus N`
builds them (one per rank): RSS after each engine's construction and after its first
streamed job on a generated file -- which part of a rank's footprint is the engine's own.

    python tools/rss_engines.py [--engines 8] [--mb 512] [--chunk-mb 256]
"""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import locust_amd as lc  # noqa: E402


def rss_kb():
    for ln in open("/proc/self/status"):
        if ln.startswith(("VmRSS", "VmHWM", "RssAnon", "RssShmem", "RssFile")):
            yield ln.split()[0].rstrip(":"), int(ln.split()[1])


def show(tag):
    d = dict(rss_kb())
    print(f"{tag:34s} rss {d['VmRSS']:9d} kB  hwm {d['VmHWM']:9d}  anon {d['RssAnon']:9d}  "
          f"shmem {d['RssShmem']:9d}  file {d['RssFile']:8d}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engines", type=int, default=8)
    ap.add_argument("--mb", type=int, default=512)
    ap.add_argument("--chunk-mb", type=int, default=256)
    a = ap.parse_args()
    show("start")
    lc._C.device_count()
    show("runtime up")
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "t.txt")
        with open(f, "wb") as fh:
            fh.write(lc._C.HostText.generate(bytes=a.mb << 20, seed=7, first_block=0).to_bytes())
        show("file written")
        cfg = lc.make_config("gpu", reduce_path="lds", chunk_bytes=a.chunk_mb << 20)
        engs = []
        for k in range(a.engines):
            e = lc._C.GpuEngine(cfg, (a.mb << 20) * 2, (a.mb << 20) * 2)
            engs.append(e)
            show(f"engine {k} built")
            r = e.run_file(f)
            show(f"engine {k} first job ({r.num_unique} keys)")
            del r
    return 0


if __name__ == "__main__":
    sys.exit(main())
