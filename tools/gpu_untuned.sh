# Headline job with and without the between-job partition retune: kernel stats and the
# ordered kernel's phase trace of each.  Usage: bash tools/gpu_untuned.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-untuned}
mkdir -p $O
export TMPDIR=/tmp
CLI=$GRAFT_REPO_ROOT/build/MapReduce
H=$GRAFT_REPO_ROOT/data/hamlet.txt
for t in 1 0; do
  (cd /tmp && LOCUST_PART_TUNE=$t timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/k$t -o run --output-format csv -- $CLI $H --warmup 5 --iters 20 --quiet > /dev/null)
  echo "== PART_TUNE=$t"; python3 tools/kstats.py $O/k$t/run_kernel_stats.csv > $O/k$t.summary.txt; cat $O/k$t.summary.txt
  LOCUST_PART_TUNE=$t LOCUST_ORD_TRACE=1 LOCUST_GRAPH=0 timeout -k 10 120 $CLI $H --warmup 3 --iters 1 --quiet > /dev/null 2> $O/trace$t.txt
  grep "^ord span" $O/trace$t.txt
done
