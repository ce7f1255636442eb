# Per-partition phase trace of the partitioned sort (LOCUST_ORD_TRACE) on whole Hamlet, radix path.
# Usage: bash tools/gpu_psort_trace.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pstrace}
mkdir -p $O
LOCUST_GRAPH=0 LOCUST_ORD_TRACE=1 timeout -k 10 120 build/MapReduce data/hamlet.txt --sort radix --warmup 4 --iters 2 --quiet > /dev/null 2> $O/trace.txt
grep "psort span" $O/trace.txt | tail -3
grep "psort p=" $O/trace.txt | tail -256 | sort -t= -k7 -n | tail -25
