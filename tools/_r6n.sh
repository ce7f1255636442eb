set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6n
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_stream.py tests/test_switches.py tests/test_gpu_engine.py tests/test_cli_gpu.py tests/test_hbm_plan.py tests/test_stage_split.py tests/test_small_pass.py tests/test_file_shards.py tests/test_large_ordered.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('headline',d['value'],'untuned',d.get('untuned'),'700',d['hamlet700']['ms_per_step'],'synth1m',d['synth1m']['ms_per_step'],d['synth1m']['GB_per_s'],'cold',d['cold_start'])"
timeout -k 10 600 bash tools/gpu_stage10g.sh r6n/s10 10 8 3 bytes > $O/stage.txt 2>&1 || { tail -30 $O/stage.txt; exit 1; }
cat $O/s10/summary.txt
D=/tmp/locust_r6n_$$
mkdir -p $D
trap 'rm -rf $D' EXIT
timeout -k 10 120 ./build/MapReduce --gen $D/a.txt --gen-bytes $((1280<<20)) --seed 7 > /dev/null
for i in 1 2; do
LOCUST_LOG=debug timeout -k 10 60 ./build/MapReduce $D/a.txt 0 0 0 1 --byte-range 0: --spill-dir $D --spill-format binary --json $O/map$i.json > /dev/null 2> $O/map$i.err
grep -E "engine \(|stream setup" $O/map$i.err
python3 -c "import json; d=json.load(open('$O/map$i.json')); print({k: round(d[k],1) for k in ('job_ms','runtime_init_ms','setup_ms','run_ms','map_ms')})"
done
