# Distributed synthetic configs rehearsed on one GPU: RCCL with one rank, TCP with 2 ranks.
# Usage: bash tools/gpu_dist_synth.sh TAG
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-dsynth}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29631 bench.py --config synth1m --gpus 1 --steps 10 --warmup 3 --force-dist > gpurun_out/$TAG/rccl1_synth1m.json 2> gpurun_out/$TAG/rccl1_synth1m.err || { tail -30 gpurun_out/$TAG/rccl1_synth1m.err; exit 1; }
cat gpurun_out/$TAG/rccl1_synth1m.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29632 bench.py --config synth1m --gpus 2 --steps 10 --warmup 3 --comm tcp > gpurun_out/$TAG/tcp2_synth1m.json 2> gpurun_out/$TAG/tcp2_synth1m.err || { tail -30 gpurun_out/$TAG/tcp2_synth1m.err; exit 1; }
cat gpurun_out/$TAG/tcp2_synth1m.json
