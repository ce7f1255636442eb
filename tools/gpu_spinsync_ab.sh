# A/B of the host wait after each job: LOCUST_SPIN_SYNC=1 (hipStreamQuery poll) vs 0
# (hipStreamSynchronize), default bench, alternating in one call.  Usage: bash tools/gpu_spinsync_ab.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-spinab}
mkdir -p $O
for i in 1 2 3; do
  for v in 1 0; do
    LOCUST_SPIN_SYNC=$v timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-extra > $O/s${v}_$i.json 2> $O/s${v}_$i.err
    python -c "import json;d=json.loads(open('$O/s${v}_$i.json').read().strip().splitlines()[-1]);print('spin=$v', d['value'])"
  done
done
