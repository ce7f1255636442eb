set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6k
mkdir -p $O
D=/tmp/locust_r6k_$$
mkdir -p $D
trap 'rm -rf $D' EXIT
timeout -k 10 120 ./build/MapReduce --gen $D/a.txt --gen-bytes $((1280<<20)) --seed 7 > /dev/null
for i in 1 2; do
LOCUST_LOG=debug timeout -k 10 60 ./build/MapReduce $D/a.txt --json $O/single$i.json > /dev/null 2> $O/single$i.err
LOCUST_LOG=debug timeout -k 10 60 ./build/MapReduce $D/a.txt 0 0 0 1 --byte-range 0: --spill-dir $D --spill-format binary --json $O/map$i.json > /dev/null 2> $O/map$i.err
done
for f in single1 map1 single2 map2; do
  echo "== $f"; grep -v "pinned .*MiB" $O/$f.err | head -30
  python3 -c "import json; d=json.load(open('$O/$f.json')); print({k: (round(v,2) if isinstance(v,float) else v) for k,v in (d.get('startup') or d).items() if k.endswith('_ms')})"
done
