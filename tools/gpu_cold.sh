# Cold first jobs: engine-by-engine timings and a kernel trace of a fresh process.
# Usage: bash tools/gpu_cold.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-cold}
mkdir -p $O
timeout -k 10 120 python tools/cold_probe.py --config synth1m --engines 3 2>&1 | tail -3 | cut -c1-120
HIP_ENABLE_DEFERRED_LOADING=0 timeout -k 10 120 python tools/cold_probe.py --config synth1m --engines 2 2>&1 | tail -2 | cut -c1-120
LOCUST_DEVPLAN=0 timeout -k 10 120 python tools/cold_probe.py --config synth1m --engines 2 2>&1 | tail -2 | cut -c1-120
timeout -k 10 120 python tools/cold_probe.py --config hamlet4500 --engines 2 2>&1 | tail -2 | cut -c1-120
HIP_ENABLE_DEFERRED_LOADING=0 timeout -k 10 120 python tools/cold_probe.py --config hamlet4500 --engines 2 2>&1 | tail -2 | cut -c1-120
timeout -k 10 60 ./build/MapReduce data/hamlet.txt --json $O/cli_hamlet.json --quiet > /dev/null && cat $O/cli_hamlet.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o cold -- python3 tools/cold_probe.py --config synth1m --engines 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
