# Tests + benches (headline and synthetic configs) + profiles in one call.
# Usage: bash tools/gpu_full.sh TAG
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-full}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.txt 2>&1 || { tail -60 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --config synth1m --steps 20 --warmup 3 > $O/synth1m.json 2> $O/synth1m.err || { tail -30 $O/synth1m.err; exit 1; }
cat $O/synth1m.json
timeout -k 10 600 python bench.py --config synth10g --steps 3 --warmup 1 > $O/synth10g.json 2> $O/synth10g.err || { tail -30 $O/synth10g.err; exit 1; }
cat $O/synth10g.json
bash tools/gpu_profile.sh $TAG/prof
