# Rehearse the multi-process benchmark path on one GPU (tcp staging), and RCCL with 1 rank.
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-dist}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 100 --warmup 10 --force-dist > gpurun_out/$TAG/rccl1.json 2> gpurun_out/$TAG/rccl1.err || { tail -30 gpurun_out/$TAG/rccl1.err; exit 1; }
cat gpurun_out/$TAG/rccl1.json
for n in 2 4; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2962$n bench.py --gpus $n --steps 30 --warmup 3 --comm tcp > gpurun_out/$TAG/tcp$n.json 2> gpurun_out/$TAG/tcp$n.err || { tail -30 gpurun_out/$TAG/tcp$n.err; exit 1; }
cat gpurun_out/$TAG/tcp$n.json
done
# the self-spawned form (no launcher: bench.py starts its own rank processes) with the
# device data plane staged over TCP (tcpdev: the device exchange and shared output run
# exactly as over RCCL)
timeout -k 10 300 python bench.py --gpus 2 --steps 30 --warmup 3 --comm tcpdev > gpurun_out/$TAG/tcpdev2.json 2> gpurun_out/$TAG/tcpdev2.err || { tail -30 gpurun_out/$TAG/tcpdev2.err; exit 1; }
cat gpurun_out/$TAG/tcpdev2.json
