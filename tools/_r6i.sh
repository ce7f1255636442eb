set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6i
mkdir -p $O
D=/tmp/locust_r6i_$$
mkdir -p $D
trap 'rm -rf $D' EXIT
timeout -k 10 120 ./build/MapReduce --gen $D/a.txt --gen-bytes $((4<<30)) --seed 7 > /dev/null
timeout -k 10 300 ./build/read_probe $D/a.txt 0 4 8 12 16 > $O/read_probe.txt 2>&1
cat $O/read_probe.txt
rm -f $D/a.txt
timeout -k 10 600 bash tools/gpu_stage10g.sh r6i/s10 10 8 3 bytes > $O/stage.txt 2>&1 || { tail -30 $O/stage.txt; exit 1; }
cat gpurun_out/r6i/s10/summary.txt
