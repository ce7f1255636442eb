# Run selected GPU tests: bash tools/gpu_one.sh TAG "pytest -k expression"
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-one}
mkdir -p $O
timeout -k 10 600 python -m pytest tests -x -q -m gpu -k "$2" > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
