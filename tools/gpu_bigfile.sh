# A --gen-made large file through ./MapReduce (streamed: pinned read ring -> device chunks):
# peak host RSS, wall time and page-cache throughput, cold-ish (just written) and warm.
# Usage: bash tools/gpu_bigfile.sh TAG [GIB]
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-bigfile}
G=${2:-10}
mkdir -p $O
F=/tmp/locust_big_$$.txt
trap 'rm -f $F' EXIT
timeout -k 10 300 ./build/MapReduce --gen $F --gen-bytes $((G<<30)) --seed 7 > $O/gen.txt
for run in 1 2; do
  /usr/bin/time -v timeout -k 10 300 ./build/MapReduce $F --quiet --json $O/run$run.json \
    > $O/run$run.out 2> $O/run$run.time
  python3 - "$O/run$run.json" "$O/run$run.time" "$G" <<'PY'
import json, re, sys
d = json.load(open(sys.argv[1]))
t = open(sys.argv[2]).read()
wall = re.search(r"Elapsed \(wall clock\) time.*: (.*)", t).group(1)
maxrss = int(re.search(r"Maximum resident set size \(kbytes\): (\d+)", t).group(1))
gib = float(sys.argv[3])
print(f"{gib:.0f} GiB file: job wall {d['wall_ms_median']:.1f} ms "
      f"({gib * 1.073741824 / (d['wall_ms_median'] / 1e3):.1f} GB/s), process wall {wall}, "
      f"VmHWM {d['max_rss_kb']} kB, time -v max RSS {maxrss} kB, chunks {d['chunks']}, "
      f"tokens {d['tokens']}, unique {d['unique']}")
PY
done
