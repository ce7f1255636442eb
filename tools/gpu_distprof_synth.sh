# Kernel timeline of the distributed synth1m job with one RCCL rank (no --pmc).
# Usage: bash tools/gpu_distprof_synth.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-dps}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
MASTER_ADDR=127.0.0.1 MASTER_PORT=29651 timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d $O/d1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config synth1m --force-dist --no-extra --steps 10 --warmup 3 > $O/d1.json 2> $O/d1.err
cd $GRAFT_REPO_ROOT
cat $O/d1.json
python3 tools/kstats.py $O/d1/run_kernel_stats.csv | tee $O/d1.kernels.txt
python3 tools/kjobs.py $O/d1/run_kernel_trace.csv 1 > $O/d1.job.txt
python3 - $O/d1/run_hip_api_stats.csv <<'PY' | tee $O/d1.api.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f"{r['Name'][:40]:40s} calls={r['Calls']:>7} avg_us={float(r['AverageNs'])/1e3:9.2f} total_ms={float(r['TotalDurationNs'])/1e6:9.2f}")
PY
