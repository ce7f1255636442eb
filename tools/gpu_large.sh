# Large-pass cycle: the large-ordered GPU tests, the synth1m bench and a kernel trace of a
# 1M-line synthetic job through the CLI.  Usage: bash tools/gpu_large.sh TAG [pytest -k expr]
set -e
cd $GRAFT_REPO_ROOT
T=${1:-large}
K=${2:-"large_ordered"}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "$K" --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 300 python bench.py --config synth1m --steps 20 --warmup 3 > $O/synth1m.json 2> $O/synth1m.err || { tail -30 $O/synth1m.err; exit 1; }
cat $O/synth1m.json
CLI=$GRAFT_REPO_ROOT/build/MapReduce
$CLI --gen /tmp/synth1m.txt --gen-lines 1000000 --seed 1 > /dev/null
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ksynth -o run --output-format csv -- $CLI /tmp/synth1m.txt --warmup 3 --iters 5 --quiet > /dev/null
cd $GRAFT_REPO_ROOT
python3 tools/kstats.py $O/ksynth/run_kernel_stats.csv | tee $O/ksynth.summary.txt
python3 tools/ktimeline.py $O/ksynth/run_kernel_trace.csv 40 > $O/ksynth.timeline.txt
