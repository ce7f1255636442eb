# GPU tests then the distributed rehearsal.  Usage: bash tools/gpu_test_dist.sh TAG
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-run}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/$TAG/pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/$TAG/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/$TAG/pytest_gpu.txt
bash tools/gpu_dist.sh $TAG
