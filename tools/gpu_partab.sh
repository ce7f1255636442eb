# Ordered-kernel phase traces with the first-byte map (LOCUST_PART_TUNE=0) and the
# balanced map, the headline bench both ways, then the GPU tests.
# Usage: bash tools/gpu_partab.sh TAG [pytest -k expr]
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pab}
mkdir -p $O
for tune in 0 1; do
  LOCUST_PART_TUNE=$tune LOCUST_ORD_TRACE=1 LOCUST_GRAPH=0 timeout -k 10 120 ./build/MapReduce data/hamlet.txt --warmup 3 --iters 1 --quiet > $O/out_$tune.txt 2> $O/trace_$tune.txt
  grep "ord span" $O/trace_$tune.txt | tail -1
  LOCUST_PART_TUNE=$tune timeout -k 10 300 python bench.py --no-extra > $O/bench_$tune.json 2> $O/bench_$tune.err
  python -c "import json;d=json.load(open('$O/bench_$tune.json'));print('tune=$tune bench', d['value'], d['stages_ms_median'])"
done
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${2:+-k "$2"} > $O/pytest_gpu.txt 2>&1 || { tail -60 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
