# Device exchange + shared output checks on one GPU (loopback ranks, one RCCL rank).
# Usage: bash tools/gpu_exch.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-exch}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dist.py tests/test_stream.py tests/test_cli_gpu.py \
  -x -v --timeout 200 --timeout-method thread -m gpu > $O/pytest.txt 2>&1
