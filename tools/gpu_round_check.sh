# Round-end rehearsal in one call: GPU tests, smoke(), the default bench, the one-rank RCCL
# bench (slot job as one graph) and its kernel/API profile.  Usage: bash tools/gpu_round_check.sh TAG
set -e
cd $GRAFT_REPO_ROOT
T=${1:-rc}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -60 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -30 $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29711 bench.py --gpus 1 --steps 300 --warmup 20 > $O/dist1.json 2> $O/dist1.err || { tail -30 $O/dist1.err; exit 1; }
tail -1 $O/dist1.json
bash tools/gpu_distprof.sh $T/distprof
