set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 600 bash tools/gpu_stage10g.sh r6g/s10 10 8 3 bytes > $O/stage.txt 2>&1
cat gpurun_out/r6g/s10/summary.txt
D=/tmp/locust_r6g_$$
mkdir -p $D
trap 'rm -rf $D' EXIT
timeout -k 10 120 ./build/MapReduce --gen $D/a.txt --gen-bytes $((1400<<20)) --seed 7 > /dev/null
LOCUST_LOG=debug timeout -k 10 120 ./build/MapReduce $D/a.txt 0 0 0 1 --byte-range 0: --spill-dir $D --spill-format binary --json $O/map_dbg.json > $O/map_dbg.out 2> $O/map_dbg.err
grep -E "engine \(|stream setup|teardown" $O/map_dbg.err || true
python3 -c "import json; d=json.load(open('$O/map_dbg.json')); print({k: d[k] for k in ('job_ms','runtime_init_ms','window_ms','setup_ms','run_ms','spill_write_ms','map_ms')})"
timeout -k 10 300 python tools/exit_probe.py --runs 7 --out $O/exit_probe.txt
timeout -k 10 120 python tools/cli_cold.py --runs 5 --out $O/cli_cold.txt > /dev/null
grep -E "process_ms|exit_ms|runtime_init|engine_ms|first_job" $O/cli_cold.txt
