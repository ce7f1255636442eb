# Host memory (max RSS) of CLI runs: small file, a direct pinned read, a streamed file.
# Usage: bash tools/gpu_rss.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-rss}
mkdir -p $O
F=/tmp/locust_rss_$$.txt
timeout -k 10 60 ./build/MapReduce --gen $F --gen-bytes $((320<<20)) --seed 5
for args in "data/hamlet.txt" "data/hamlet.txt --backend cpu" "$F --chunk-mb 512" "$F --chunk-mb 64" "$F --chunk-mb 128"; do
  timeout -k 10 120 ./build/MapReduce $args --quiet --json $O/r.json > /dev/null
  python3 -c "import json; d=json.load(open('$O/r.json')); print('$args', d.get('max_rss_kb'), d.get('chunks'), d.get('wall_ms_median'))"
done
LOCUST_LOG=debug timeout -k 10 120 ./build/MapReduce $F --chunk-mb 64 --quiet > /dev/null 2> $O/log.txt || true
tail -5 $O/log.txt
rm -f $F
