# Round-4 check: GPU tests of the touched areas, benches, cold CLI breakdown, 10 GiB ranks.
# Usage: bash tools/gpu_r4.sh TAG [pytest files...]
set -e
cd $GRAFT_REPO_ROOT
T=${1:-r4}
shift || true
O=gpurun_out/$T
mkdir -p $O
FILES=${@:-tests/test_gpu_engine.py tests/test_file_shards.py tests/test_scale_ready.py tests/test_cli_gpu.py tests/test_dist.py}
timeout -k 10 600 python -u -m pytest $FILES -x -v -s -m gpu --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('headline',d['value'],'untuned',d['untuned'],'700',d['hamlet700']['ms_per_step'],'synth1m',d['synth1m']['ms_per_step'],d['synth1m']['GB_per_s'])"
timeout -k 10 200 python tools/cli_cold.py --out $O/cold.txt
