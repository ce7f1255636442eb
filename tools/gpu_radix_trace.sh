# Reference-algorithm path (--sort radix): per-partition phase stamps of the fused
# sort + reduce kernel, warm (LOCUST_ORD_TRACE=1), and kernel stats.  Usage: bash tools/gpu_radix_trace.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-radix}
mkdir -p $O
LOCUST_ORD_TRACE=1 timeout -k 10 120 ./build/MapReduce data/hamlet.txt --sort radix --warmup 5 --iters 1 --quiet > /dev/null 2> $O/trace.txt
grep "span" $O/trace.txt | tail -1
sort -t= -k7 -n $O/trace.txt | grep "^psort p" | awk '{print}' | sort -k9 -t'|' | tail -8
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kradix -o run --output-format csv -- $GRAFT_REPO_ROOT/build/MapReduce $GRAFT_REPO_ROOT/data/hamlet.txt --sort radix --warmup 5 --iters 25 --quiet > /dev/null
cd $GRAFT_REPO_ROOT
python3 tools/kstats.py $O/kradix/run_kernel_stats.csv | tee $O/kradix.summary.txt
