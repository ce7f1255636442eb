# A/B of the one-graph gather-slot job (LOCUST_SLOT_GRAPH=1) against separate launches (0)
# on the one-rank RCCL bench, alternating in one call.  Usage: bash tools/gpu_slotgraph_ab.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-sgab}
mkdir -p $O
for i in 1 2 3; do
  for v in 1 0; do
    LOCUST_SLOT_GRAPH=$v timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 296$i$v bench.py --gpus 1 --steps 300 --warmup 20 --force-dist --no-extra > $O/g${v}_$i.json 2> $O/g${v}_$i.err
    python -c "import json;d=json.loads(open('$O/g${v}_$i.json').read().strip().splitlines()[-1]);print('slot_graph=$v', d['value'])"
  done
done
