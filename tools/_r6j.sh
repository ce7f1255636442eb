set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6j
mkdir -p $O
D=/tmp/locust_r6j_$$
mkdir -p $D
trap 'rm -rf $D' EXIT
timeout -k 10 120 ./build/MapReduce --gen $D/a.txt --gen-bytes $((1280<<20)) --seed 7 > /dev/null
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof -o m -- $GRAFT_REPO_ROOT/build/MapReduce $D/a.txt 0 0 0 1 --byte-range 0: --spill-dir $D --spill-format binary --json $O/map.json > $O/map.out 2>&1
cd $GRAFT_REPO_ROOT
K=$(find $O/prof -name "*kernel_trace.csv" | head -1)
C=$(find $O/prof -name "*memory_copy_trace.csv" | head -1)
head -2 $C > $O/copy_head.txt
python3 tools/stream_windows.py $K $C --first 8 | tee $O/windows.txt
python3 -c "import json; d=json.load(open('$O/map.json')); print({k: round(d[k],1) for k in ('job_ms','setup_ms','run_ms','map_ms')})"
# single stage over the same file for comparison
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof1 -o s -- $GRAFT_REPO_ROOT/build/MapReduce $D/a.txt --json $O/single.json > /dev/null 2>&1
cd $GRAFT_REPO_ROOT
K=$(find $O/prof1 -name "*kernel_trace.csv" | head -1)
C=$(find $O/prof1 -name "*memory_copy_trace.csv" | head -1)
python3 tools/stream_windows.py $K $C --first 8 | tee $O/windows_single.txt
rm -rf $O/prof $O/prof1
