# Geometric upload tail A/B on synth1m (two processes each way) and the device-arena
# cycle micro.  Usage: bash tools/gpu_tail_arena.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-tail}
mkdir -p $O
for v in 1 0 1 0; do
  echo "LOCUST_PIECE_TAIL=$v" >> $O/tail_ab.txt
  LOCUST_PIECE_TAIL=$v PYTHONPATH=. timeout -k 10 120 python -u tools/steps.py 1000000 60 >> $O/tail_ab.txt 2>&1
done
timeout -k 10 120 ./build/arena_cycle 6 4 4 0 > $O/arena_cycle.txt 2>&1
timeout -k 10 120 ./build/arena_cycle 6 4 4 1 >> $O/arena_cycle.txt 2>&1
