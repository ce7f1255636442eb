# All GPU tests, the single-GPU host A/B and the distributed rehearsal.  Usage: bash tools/gpu_quick.sh TAG
set -e
cd $GRAFT_REPO_ROOT
T=${1:-quick}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.txt 2>&1 || { tail -60 gpurun_out/$T/pytest.txt; exit 1; }
tail -2 gpurun_out/$T/pytest.txt
timeout -k 10 300 python tools/host_ab.py --rounds 3
bash tools/gpu_dist.sh $T
