# GPU bench + profile (run under gpurun).  Usage: bash tools/gpu_bench.sh [tag]
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r1}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
cat gpurun_out/$TAG/bench.json
timeout -k 10 300 ./build/MapReduce data/hamlet.txt --warmup 20 --iters 50 --quiet --json gpurun_out/$TAG/cli4500.json > gpurun_out/$TAG/cli4500.txt
cat gpurun_out/$TAG/cli4500.txt gpurun_out/$TAG/cli4500.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- $GRAFT_REPO_ROOT/build/MapReduce $GRAFT_REPO_ROOT/data/hamlet.txt --warmup 5 --iters 20 --quiet > /dev/null
cd $GRAFT_REPO_ROOT
python3 tools/kstats.py gpurun_out/$TAG/prof/run_kernel_stats.csv
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof700 -o run --output-format csv -- $GRAFT_REPO_ROOT/build/MapReduce $GRAFT_REPO_ROOT/data/hamlet.txt 0 700 --warmup 5 --iters 20 --quiet > /dev/null
cd $GRAFT_REPO_ROOT && python3 tools/kstats.py gpurun_out/$TAG/prof700/run_kernel_stats.csv
