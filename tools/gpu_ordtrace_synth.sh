# Ordered-kernel phase trace on synth1m (the large-vocabulary ordered build over the
# per-piece partials).  Usage: bash tools/gpu_ordtrace_synth.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ots}
mkdir -p $O
./build/MapReduce --gen /tmp/synth1m.txt --gen-lines 1000000 --seed 1 > /dev/null
LOCUST_ORD_TRACE=1 LOCUST_GRAPH=0 timeout -k 10 120 ./build/MapReduce /tmp/synth1m.txt --warmup 3 --iters 1 --quiet > $O/out.txt 2> $O/trace.txt
tail -5 $O/trace.txt
