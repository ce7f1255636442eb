# Kernel timeline of the shuffle strategy (device exchange) on one
# RCCL rank.  Usage: bash tools/gpu_distprof_shuffle.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-dpg}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
LOCUST_SLOT_GRAPH=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29653 timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d $O/s1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --force-dist --no-extra --strategy shuffle --steps 100 --warmup 10 > $O/s1.json 2> $O/s1.err
cd $GRAFT_REPO_ROOT
python3 tools/kstats.py $O/s1/run_kernel_stats.csv | tee $O/s1.kernels.txt
python3 tools/ktimeline.py $O/s1/run_kernel_trace.csv 16 > $O/s1.timeline.txt
python3 - $O/s1/run_hip_api_stats.csv <<'PY' | tee $O/s1.api.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:20]:
    print(f"{r['Name'][:40]:40s} calls={r['Calls']:>7} avg_us={float(r['AverageNs'])/1e3:9.2f} total_ms={float(r['TotalDurationNs'])/1e6:9.2f}")
PY
