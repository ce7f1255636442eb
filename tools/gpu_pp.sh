# Piecewise large-pass check: correctness over repeated runs, the synth1m bench and a
# kernel timeline, plus one traced run (map tiles + partials + ordered phases).
# Usage: bash tools/gpu_pp.sh TAG
set -e
cd $GRAFT_REPO_ROOT
T=${1:-pp}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
PYTHONPATH=. timeout -k 10 200 python tools/dbg_large.py 1000000 > $O/dbg.txt 2>&1 || { tail -30 $O/dbg.txt; exit 1; }
cat $O/dbg.txt
timeout -k 10 300 python bench.py --config synth1m --steps 20 --warmup 3 > $O/synth1m.json 2> $O/synth1m.err || { tail -30 $O/synth1m.err; exit 1; }
cat $O/synth1m.json
CLI=$GRAFT_REPO_ROOT/build/MapReduce
$CLI --gen /tmp/synth1m.txt --gen-lines 1000000 --seed 1 > /dev/null
LOCUST_ORD_TRACE=1 LOCUST_MAP_TRACE=1 timeout -k 10 120 $CLI /tmp/synth1m.txt --warmup 2 --iters 1 --quiet > /dev/null 2> $O/trace.txt || { tail -30 $O/trace.txt; exit 1; }
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ksynth -o run --output-format csv -- $CLI /tmp/synth1m.txt --warmup 3 --iters 5 --quiet > /dev/null
cd $GRAFT_REPO_ROOT
python3 tools/kstats.py $O/ksynth/run_kernel_stats.csv | tee $O/ksynth.summary.txt
python3 tools/ktimeline.py $O/ksynth/run_kernel_trace.csv 40 > $O/ksynth.timeline.txt
