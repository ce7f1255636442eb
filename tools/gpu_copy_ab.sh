# Piece-copy variants on synth1m, one process per variant (in-process A/B of stream
# layouts is invalid: engines share the process's 4 HW queues), two rounds alternating.
# Usage: bash tools/gpu_copy_ab.sh TAG "VAR=v,VAR=v" ...
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-copyab}
shift
mkdir -p $O
for round in 1 2; do
  for v in "$@"; do
    echo "== $v (round $round)" >> $O/copy_ab.txt
    env $(echo "$v" | tr ',' ' ') PYTHONPATH=. timeout -k 10 120 python -u tools/steps.py 1000000 60 2>&1 | grep -E "^mean" >> $O/copy_ab.txt
  done
done
cat $O/copy_ab.txt
