# Round-4 host-side checks: the 10 GiB file at --gpus 8 (RSS), the runtime's own RSS by
# mapping, the inter-GPU probe, and the cold CLI breakdown with allocation logging.
# Usage: bash tools/gpu_r4d.sh TAG
set -e
cd $GRAFT_REPO_ROOT
T=${1:-r4d}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 120 ./build/rss_probe > $O/rss_probe.txt 2>&1 || { tail -20 $O/rss_probe.txt; exit 1; }
grep -v "^\s*\[" $O/rss_probe.txt | head -20
timeout -k 10 200 ./build/xgmi_probe 256 > $O/xgmi_probe.txt 2>&1 || { tail -20 $O/xgmi_probe.txt; exit 1; }
tail -8 $O/xgmi_probe.txt
timeout -k 10 120 python tools/cli_cold.py --out $O/cold.txt
LOCUST_LOG=debug timeout -k 10 60 ./build/MapReduce data/hamlet.txt --iters 3 --quiet > /dev/null 2> $O/cli_debug.txt || true
grep -n "output buffer\|retune" $O/cli_debug.txt | head
bash tools/gpu_bigfile_ranks.sh $T/big 10 8 loopback
