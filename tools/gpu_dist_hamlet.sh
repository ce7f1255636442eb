# Distributed hamlet4500 with one RCCL rank: auto (local), forced gather, forced shuffle.
# Usage: bash tools/gpu_dist_hamlet.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-dh}
mkdir -p $O
for s in auto gather shuffle; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2964${#s} bench.py --gpus 1 --steps 500 --warmup 20 --force-dist --no-extra --strategy $s > $O/rccl1_$s.json 2> $O/rccl1_$s.err || { tail -20 $O/rccl1_$s.err; exit 1; }
  echo "$s $(python3 -c "import json;d=json.load(open('$O/rccl1_$s.json'));print(d['value'], d['config']['parallelism'])")"
done
