# Gather strategy as at world > 1 (slot graph off), one RCCL rank: direct launches (lean)
# vs replayed graphs for the shard engine's sequences.  Usage: bash tools/gpu_gather_lean_ab.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-gl}
mkdir -p $O
for i in 1 2; do for v in 1 0; do
  LOCUST_SLOT_GRAPH=0 LOCUST_LEAN=$v timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2967$v bench.py --gpus 1 --steps 1000 --warmup 50 --force-dist --no-extra --strategy gather > $O/g_$v.$i.json 2> $O/g_$v.$i.err || { tail -20 $O/g_$v.$i.err; exit 1; }
  echo "lean=$v gather $(python3 -c "import json;d=json.load(open('$O/g_$v.$i.json'));print(d['value'])")"
  LOCUST_LEAN=$v timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2968$v bench.py --gpus 1 --steps 500 --warmup 20 --force-dist --no-extra --strategy shuffle > $O/s_$v.$i.json 2> $O/s_$v.$i.err || { tail -20 $O/s_$v.$i.err; exit 1; }
  echo "lean=$v shuffle $(python3 -c "import json;d=json.load(open('$O/s_$v.$i.json'));print(d['value'])")"
done; done
