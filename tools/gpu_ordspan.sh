# Ordered-kernel critical path on whole Hamlet (LOCUST_ORD_TRACE) + kernel timeline of the
# headline job (graph replay).  Usage: bash tools/gpu_ordspan.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-os}
mkdir -p $O
LOCUST_ORD_TRACE=1 LOCUST_GRAPH=0 timeout -k 10 120 ./build/MapReduce data/hamlet.txt --warmup 5 --iters 1 --quiet > /dev/null 2> $O/trace.txt
python3 tools/ordtrace_span.py $O/trace.txt 8
bash tools/gpu_kprof.sh $1/kp > /dev/null
tail -12 $O/kp/k4500.timeline.txt
