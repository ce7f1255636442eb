# LDS counters of the headline kernels (CLI on whole Hamlet), current build and ab/prev.
# Usage: bash tools/gpu_pmc_map.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmcmap}
mkdir -p $O
cd /tmp
for v in now prev; do
  if [ $v = prev ]; then CLI=$GRAFT_REPO_ROOT/ab/prev/build/MapReduce; else CLI=$GRAFT_REPO_ROOT/build/MapReduce; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES -d $O/pmc_$v -o run --output-format csv -- $CLI $GRAFT_REPO_ROOT/data/hamlet.txt --warmup 2 --iters 5 --quiet > /dev/null
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/k_$v -o run --output-format csv -- $CLI $GRAFT_REPO_ROOT/data/hamlet.txt --warmup 5 --iters 40 --quiet > /dev/null
  echo "== $v"; python3 $GRAFT_REPO_ROOT/tools/kstats.py $O/k_$v/run_kernel_stats.csv | head -2
done
cd $GRAFT_REPO_ROOT
python3 tools/pmc_summary.py $O/pmc_summary_now.txt $O/pmc_now > /dev/null 2>&1 || true
python3 tools/pmc_summary.py $O/pmc_summary_prev.txt $O/pmc_prev > /dev/null 2>&1 || true
grep -A2 "map_fast_kernel<1, 1024>" $O/pmc_summary_now.txt $O/pmc_summary_prev.txt || true
