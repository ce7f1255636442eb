# Kernel timeline of the gather strategy as it runs at world > 1 (slot graph off), on one
# RCCL rank.  Usage: bash tools/gpu_distprof_gather.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-dpg}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
LOCUST_SLOT_GRAPH=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29652 timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d $O/g1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --force-dist --no-extra --strategy gather --steps 200 --warmup 20 > $O/g1.json 2> $O/g1.err
cd $GRAFT_REPO_ROOT
python3 tools/kstats.py $O/g1/run_kernel_stats.csv | tee $O/g1.kernels.txt
python3 tools/ktimeline.py $O/g1/run_kernel_trace.csv 16 > $O/g1.timeline.txt
python3 - $O/g1/run_hip_api_stats.csv <<'PY' | tee $O/g1.api.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:20]:
    print(f"{r['Name'][:40]:40s} calls={r['Calls']:>7} avg_us={float(r['AverageNs'])/1e3:9.2f} total_ms={float(r['TotalDurationNs'])/1e6:9.2f}")
PY
