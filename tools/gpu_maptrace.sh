# Map kernel per-tile timeline (LOCUST_MAP_TRACE=1) on whole Hamlet: the last job's tiles,
# summarised.  Usage: bash tools/gpu_maptrace.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-mt}
mkdir -p $O
LOCUST_MAP_TRACE=1 LOCUST_GRAPH=0 timeout -k 10 120 ./build/MapReduce data/hamlet.txt --warmup 3 --iters 1 --quiet > /dev/null 2> $O/maptrace.txt
python3 - $O/maptrace.txt <<'PY'
import re, statistics, sys
lines = [l for l in open(sys.argv[1]) if l.startswith("map tile=")]
n = len(set(int(re.search(r"tile=\s*(\d+)", l).group(1)) for l in lines))
last = lines[-n:]
rows = [{k: float(v) for k, v in re.findall(r"(\w+)=\s*([\d.]+)", l)} for l in last]
for k in ("entry", "acquired", "staged", "masks", "prefix", "done"):
    v = [r[k] for r in rows]
    print(f"{k:9s} min={min(v):6.2f} median={statistics.median(v):6.2f} max={max(v):6.2f} us")
PY
