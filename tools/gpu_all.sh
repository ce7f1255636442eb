# GPU tests + bench + rocprof in one gpurun call.  Usage: bash tools/gpu_all.sh TAG
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-run}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/$TAG/pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/$TAG/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/$TAG/pytest_gpu.txt
bash tools/gpu_bench.sh $TAG
