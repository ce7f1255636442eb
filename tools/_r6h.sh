set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_stream.py tests/test_hbm_plan.py tests/test_stage_split.py tests/test_file_shards.py tests/test_cli_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 600 bash tools/gpu_stage10g.sh r6h/s10 10 8 3 bytes > $O/stage.txt 2>&1 || { tail -30 $O/stage.txt; exit 1; }
cat gpurun_out/r6h/s10/summary.txt
D=/tmp/locust_r6h_$$
mkdir -p $D
trap 'rm -rf $D' EXIT
timeout -k 10 120 ./build/MapReduce --gen $D/a.txt --gen-bytes $((1400<<20)) --seed 7 > /dev/null
for i in 0 1 2; do
LOCUST_LOG=debug timeout -k 10 120 ./build/MapReduce $D/a.txt 0 0 0 1 --byte-range 0: --spill-dir $D --spill-format binary --json $O/map_dbg$i.json > $O/map_dbg.out 2> $O/map_dbg$i.err
grep -E "engine \(|stream setup" $O/map_dbg$i.err || true
python3 -c "import json; d=json.load(open('$O/map_dbg$i.json')); print({k: round(d[k],1) for k in ('job_ms','runtime_init_ms','setup_ms','run_ms','spill_write_ms','map_ms')})"
done
