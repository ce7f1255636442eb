# Dist/merge GPU tests, then the distributed rehearsal (RCCL 1 rank, TCP 2/4 ranks).
set -e
cd $GRAFT_REPO_ROOT
T=${1:-merge}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_kernels.py tests/test_dist.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.txt 2>&1 || { tail -60 gpurun_out/$T/pytest.txt; exit 1; }
tail -2 gpurun_out/$T/pytest.txt
bash tools/gpu_dist.sh $T
