# Where a multi-rank file job's host memory goes: RSS (anon / file / shmem) stamps per rank
# at LOCUST_LOG=debug, 8 loopback ranks on the one GPU.  Usage: bash tools/gpu_rss8.sh TAG [GIB]
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-rss8}
mkdir -p $O
export TMPDIR=/tmp
CLI=$GRAFT_REPO_ROOT/build/MapReduce
F=/tmp/locust_rss_$$.txt
timeout -k 10 200 $CLI --gen $F --gen-bytes $((${2:-4}<<30)) --seed 7 > /dev/null
LOCUST_LOG=debug timeout -k 10 300 $CLI $F --gpus 8 --comm loopback --quiet --json $O/rss8.json > /dev/null 2> $O/rss8.err || true
rm -f $F
grep -E "rss|shared output|engine \(" $O/rss8.err | grep -v "bytes \[" | head -60
python3 -c "import json;d=json.load(open('$O/rss8.json'));print('peak_rss_kb', d.get('peak_rss_kb'))"
