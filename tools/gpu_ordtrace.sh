# Ordered-kernel phase trace on whole Hamlet.  Usage: bash tools/gpu_ordtrace.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ot}
mkdir -p $O
LOCUST_ORD_TRACE=1 LOCUST_GRAPH=0 timeout -k 10 120 ./build/MapReduce data/hamlet.txt --warmup 3 --iters 1 --quiet > $O/out.txt 2> $O/trace.txt
tail -60 $O/trace.txt
timeout -k 10 300 python bench.py --no-extra > $O/bench.json 2> $O/bench.err
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['value'], d['stages_ms_median'])"
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
