# Round-end check: the whole GPU test suite, the bench line, __graft_entry__.smoke(), and
# kernel-stat summaries of the bench's configs.  Usage: bash tools/gpu_full.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-full}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -30 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('headline',d['value'],'ms',d['ms_per_step'],'untuned',d.get('untuned'),'700',d['hamlet700']['ms_per_step'],'synth1m',d['synth1m']['ms_per_step'],d['synth1m']['GB_per_s'])"
