# GPU tests, then the untuned headline's kernel stats with the small-pass plan on / off
# (where the plan's cost sits: map occupancy masks or the ordered kernel's preamble).
# Usage: bash tools/gpu_vplan_kstats.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-vpk}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
export TMPDIR=/tmp
CLI=$GRAFT_REPO_ROOT/build/MapReduce
H=$GRAFT_REPO_ROOT/data/hamlet.txt
for v in 1 0; do
  (cd /tmp && LOCUST_PART_TUNE=0 LOCUST_VPLAN=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/vp$v -o run --output-format csv -- $CLI $H --warmup 5 --iters 40 --quiet > /dev/null)
  echo "== VPLAN=$v"; python3 tools/kstats.py $O/vp$v/run_kernel_stats.csv | tee $O/vp$v.summary.txt | head -2
done
