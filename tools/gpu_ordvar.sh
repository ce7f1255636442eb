# Ordered-kernel phase traces (balanced map) for LOCUST_ORD_VARIANT values, plus a kernel
# timeline.  Usage: bash tools/gpu_ordvar.sh TAG V1 [V2 ...]
set -e
cd $GRAFT_REPO_ROOT
T=${1:-ov}
shift
O=gpurun_out/$T
mkdir -p $O
for v in "$@"; do
  LOCUST_ORD_VARIANT=$v LOCUST_ORD_TRACE=1 LOCUST_GRAPH=0 timeout -k 10 120 ./build/MapReduce data/hamlet.txt --warmup 3 --iters 1 --quiet > /dev/null 2> $O/trace_v$v.txt
  echo "== variant $v"; python3 tools/ordtrace_span.py $O/trace_v$v.txt 4
  LOCUST_ORD_VARIANT=$v timeout -k 10 300 python bench.py --no-extra > $O/bench_v$v.json 2> $O/bench_v$v.err
  python3 -c "import json;d=json.load(open('$O/bench_v$v.json'));print('variant $v bench', d['value'], d['stages_ms_median']['graph_gpu_ms'])"
done
