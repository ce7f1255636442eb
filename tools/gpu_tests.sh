# All GPU tests, then the default bench.  Usage: bash tools/gpu_tests.sh TAG [pytest args...]
set -e
cd $GRAFT_REPO_ROOT
T=${1:-t}
shift || true
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread "$@" > $O/pytest_gpu.txt 2>&1 || { tail -80 $O/pytest_gpu.txt; exit 1; }
tail -3 $O/pytest_gpu.txt
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
