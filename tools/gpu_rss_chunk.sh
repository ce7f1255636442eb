# 8 loopback ranks on one GPU: host RSS vs the engines' chunk size (device arenas of
# 8 x ~34 GB at 256 MiB chunks fill most of the GPU's 288 GB).  Usage: bash tools/gpu_rss_chunk.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-rssc}
mkdir -p $O
CLI=$GRAFT_REPO_ROOT/build/MapReduce
F=/tmp/locust_rssc_$$.txt
timeout -k 10 200 $CLI --gen $F --gen-bytes $((4<<30)) --seed 7 > /dev/null
for c in 64 256 32; do
  LOCUST_LOG=debug timeout -k 10 300 $CLI $F --gpus 8 --comm loopback --chunk-mb $c --quiet --json $O/c$c.json > /dev/null 2> $O/c$c.err || true
  echo "== chunk $c MiB"; grep -E "engine \(|rank 0: engine built|r0\] map done|after the job" $O/c$c.err | sed 's/malloc in use.*//' | head -4
  python3 -c "import json;d=json.load(open('$O/c$c.json'));print('peak_rss_kb', d.get('peak_rss_kb'), 'wall_ms', d.get('wall_ms'))"
done
rm -f $F
