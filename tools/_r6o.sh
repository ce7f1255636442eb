cd $GRAFT_REPO_ROOT
O=gpurun_out/r6o5
mkdir -p $O
D=/tmp/locust_r6o_$$
mkdir -p $D
trap 'rm -rf $D' EXIT
timeout -k 10 120 ./build/MapReduce --gen $D/a.txt --gen-bytes $((320<<20)) --seed 5 > /dev/null
python3 - > $O/nodes.txt <<'PY'
import os
from locust_amd.parallel.numa import gpu_numa_node, node_cpus
allowed = os.sched_getaffinity(0)
g = gpu_numa_node(0)
print("gpu_node", g)
for n in sorted(int(x[4:]) for x in os.listdir("/sys/devices/system/node") if x.startswith("node") and x[4:].isdigit()):
    mine = sorted(set(node_cpus(n)) & allowed)
    print("node", n, ",".join(map(str, mine)))
PY
cat $O/nodes.txt
G=$(awk '/gpu_node/{print $2}' $O/nodes.txt)
while read tag n cpus; do
  [ "$tag" = node ] || continue
  [ -n "$cpus" ] || continue
  for i in 1 2 3; do
    LOCUST_CACHE_DIR=$D/c$n$i LOCUST_LOG=info taskset -c $cpus timeout -k 10 60 ./build/MapReduce $D/a.txt --chunk-mb 64 --json $O/n$n.$i.json > /dev/null 2> $O/n$n.$i.err
    python3 -c "import json; d=json.load(open('$O/n$n.$i.json')); s=d['startup']; print('node $n (gpu node $G) run $i max_rss_kb', d['max_rss_kb'], 'first_job_ms', round(s['first_job_ms'],1))"
  done
done < $O/nodes.txt
exit 0
