set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_small_pass.py tests/test_stage_split.py tests/test_stream.py tests/test_strings.py tests/test_switches.py tests/test_tile_order.py -v -m gpu --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('headline',d['value'],'untuned',d.get('untuned'),'700',d['hamlet700']['ms_per_step'],'radix',d['radix_path']['ms_per_step'],'synth1m',d['synth1m']['ms_per_step'],'cold',d['cold_start'])"
timeout -k 10 120 python tools/cli_cold.py --runs 7 --out $O/cli_cold_fast.txt
LOCUST_FAST_EXIT=0 timeout -k 10 120 python tools/cli_cold.py --runs 7 --out $O/cli_cold_full_exit.txt
timeout -k 10 300 bash tools/gpu_profile.sh r6e/prof > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -40 $O/profile.log
