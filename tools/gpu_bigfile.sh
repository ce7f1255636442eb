# A --gen-made large file through ./MapReduce (streamed: pinned read ring -> device chunks):
# peak host RSS (the CLI's VmHWM), wall time and page-cache throughput, twice (the second
# run reads a warm page cache).  Usage: bash tools/gpu_bigfile.sh TAG [GIB]
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-bigfile}
G=${2:-10}
mkdir -p $O
F=/tmp/locust_big_$$.txt
trap 'rm -f $F' EXIT
timeout -k 10 300 ./build/MapReduce --gen $F --gen-bytes $((G<<30)) --seed 7 > $O/gen.txt
for run in 1 2; do
  t0=$(date +%s.%N)
  timeout -k 10 300 ./build/MapReduce $F --quiet --json $O/run$run.json > $O/run$run.out
  t1=$(date +%s.%N)
  python3 - "$O/run$run.json" "$G" "$t0" "$t1" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
gib, t0, t1 = float(sys.argv[2]), float(sys.argv[3]), float(sys.argv[4])
b = gib * (1 << 30)
print(f"{gib:.0f} GiB file: job {d['wall_ms_median']:.1f} ms ({b / d['wall_ms_median'] / 1e6:.1f} GB/s), "
      f"process {t1 - t0:.2f} s ({b / (t1 - t0) / 1e9:.1f} GB/s), peak RSS {d['max_rss_kb']} kB, "
      f"chunks {d['chunks']}, tokens {d['tokens']}, unique {d['unique']}")
PY
done
