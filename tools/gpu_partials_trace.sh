# Per-workgroup timeline of the large pass's partials kernel (LOCUST_ORD_TRACE) on a 1M-line
# synthetic job.  Usage: bash tools/gpu_partials_trace.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ptrace}
mkdir -p $O
build/MapReduce --gen /tmp/synth1m.txt --gen-lines 1000000 --seed 1 > /dev/null
LOCUST_GRAPH=0 LOCUST_ORD_TRACE=1 timeout -k 10 120 build/MapReduce /tmp/synth1m.txt --warmup 2 --iters 1 --quiet > /dev/null 2> $O/trace.txt
grep "partials span" $O/trace.txt
grep "partials b=" $O/trace.txt | tail -1024 > $O/last.txt
sort -t= -k7 -n $O/last.txt | tail -12
awk '{print $5}' $O/last.txt | sort | uniq -c | sort -rn | head -3
