# Ordered-kernel phase trace + headline bench + GPU tests.  Usage: bash tools/gpu_ordab.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-oab}
mkdir -p $O
LOCUST_ORD_TRACE=1 LOCUST_GRAPH=0 timeout -k 10 120 ./build/MapReduce data/hamlet.txt --warmup 3 --iters 1 --quiet > $O/out.txt 2> $O/trace.txt
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
