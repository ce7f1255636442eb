# A fresh engine's first large job in a warm process: host log + kernel/copy timeline.
# Usage: bash tools/gpu_cold2.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-cold2}
mkdir -p $O
LOCUST_LOG=debug timeout -k 10 120 python tools/cold_probe.py --config synth1m --engines 2 > $O/log.txt 2>&1 || { tail -20 $O/log.txt; exit 1; }
grep -v "^\[locust DEBUG\] output buffer" $O/log.txt | tail -40 | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d $O/prof -o cold -- python3 tools/cold_probe.py --config synth1m --engines 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
