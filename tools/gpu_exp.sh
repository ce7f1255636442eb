# ad-hoc experiment: DVFS sensitivity of the short kernels
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-exp}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for it in 20 2000; do
  timeout -k 10 300 ./build/MapReduce data/hamlet.txt --warmup $it --iters $it --quiet --json gpurun_out/$TAG/cli_$it.json > /dev/null
  cat gpurun_out/$TAG/cli_$it.json
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- $GRAFT_REPO_ROOT/build/MapReduce $GRAFT_REPO_ROOT/data/hamlet.txt --warmup 3000 --iters 3000 --quiet > /dev/null
cd $GRAFT_REPO_ROOT && python3 tools/kstats.py gpurun_out/$TAG/prof/run_kernel_stats.csv
