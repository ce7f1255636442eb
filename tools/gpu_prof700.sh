set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-p700}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- $GRAFT_REPO_ROOT/build/MapReduce $GRAFT_REPO_ROOT/data/hamlet.txt 0 700 --warmup 5 --iters 20 --quiet > /dev/null
cd $GRAFT_REPO_ROOT && python3 tools/kstats.py gpurun_out/$TAG/prof/run_kernel_stats.csv
