# Kernel trace of the headline job (whole Hamlet, graph replay) + per-kernel timeline and
# stats.  Usage: bash tools/gpu_kprof.sh TAG [extra CLI args]
set -e
cd $GRAFT_REPO_ROOT
T=${1:-kp}
shift || true
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k4500 -o run --output-format csv -- $GRAFT_REPO_ROOT/build/MapReduce $GRAFT_REPO_ROOT/data/hamlet.txt --warmup 10 --iters 40 --quiet "$@" > /dev/null
cd $GRAFT_REPO_ROOT
python3 tools/kstats.py $O/k4500/run_kernel_stats.csv | tee $O/k4500.summary.txt
python3 tools/ktimeline.py $O/k4500/run_kernel_trace.csv 8 | tee $O/k4500.timeline.txt
