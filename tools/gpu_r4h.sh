# Launch fixed costs vs LDS / block / grid, per-workgroup release costs, and the ordered
# kernel's self-clean tail.  Usage: bash tools/gpu_r4h.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4h}
mkdir -p $O
export TMPDIR=/tmp
CLI=$GRAFT_REPO_ROOT/build/MapReduce
H=$GRAFT_REPO_ROOT/data/hamlet.txt
timeout -k 10 60 ./build/lds_launch | tee $O/lds_launch.txt
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/k_lds -o run --output-format csv -- $GRAFT_REPO_ROOT/build/lds_launch > /dev/null
python3 $GRAFT_REPO_ROOT/tools/kstats.py $O/k_lds/run_kernel_stats.csv | head -14
cd $GRAFT_REPO_ROOT
for f in 0 1; do
  LOCUST_FUSE=0 LOCUST_EXP_FENCE=$f LOCUST_ORD_TRACE=1 timeout -k 10 60 $CLI $H --warmup 5 --iters 3 --quiet > /dev/null 2> $O/ordtrace_two$f.txt
  echo "== two, fence exp $f"; grep -E "span|tail" $O/ordtrace_two$f.txt | tail -2
  LOCUST_FUSE=1 LOCUST_EXP_FENCE=$f LOCUST_ORD_TRACE=1 timeout -k 10 60 $CLI $H --warmup 5 --iters 3 --quiet > /dev/null 2> $O/ordtrace_fused$f.txt
  echo "== fused, fence exp $f"; grep -E "span|tail|fused:" $O/ordtrace_fused$f.txt | tail -3
done
