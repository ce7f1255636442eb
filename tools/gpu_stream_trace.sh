# Kernel trace of streamed in-memory jobs, engine after engine (tools/stream_probe.py).
# Usage: bash tools/gpu_stream_trace.sh TAG [probe args...]
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-stream}
shift || true
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof -o st -- python3 tools/stream_probe.py "$@" > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep "^engine\|^generated" $O/probe.log
find $O/prof -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
find $O/prof -name "*memory_copy_trace.csv" -exec cp {} $O/memcpy_trace.csv \;
rm -rf $O/prof
