# One build->measure cycle: GPU tests, headline bench, kernel profile of the 4,500-line job.
# Usage: bash tools/gpu_cycle.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-cycle}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.txt 2>&1 || { tail -60 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['value'], d['stages_ms_median'], '700:', d['hamlet700']['ms_per_step'], 'radix:', d['radix_path']['ms_per_step'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- $GRAFT_REPO_ROOT/build/MapReduce $GRAFT_REPO_ROOT/data/hamlet.txt --warmup 5 --iters 20 --quiet > /dev/null
cd $GRAFT_REPO_ROOT && python3 tools/kstats.py $O/prof/run_kernel_stats.csv
if [ -n "$AB_ENV" ]; then
  env $AB_ENV timeout -k 10 300 python bench.py > $O/bench_ab.json 2> $O/bench_ab.err || { tail -30 $O/bench_ab.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_ab.json'));print('A/B $AB_ENV', d['value'], d['stages_ms_median'], '700:', d['hamlet700']['ms_per_step'])"
fi
