# Kernel + memory-copy trace of steady synth1m jobs (tools/steps.py, 8 jobs): where the
# job's time goes between the upload pieces, the map / partials kernels and the ordered
# build.  Usage: bash tools/gpu_copytrace.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-copytrace}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/steps.py 1000000 8 > $O/steps.txt 2>&1
ls $O/trace
