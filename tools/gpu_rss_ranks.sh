# Anonymous / shmem growth of a file job by rank count (LOCUST_LOG=debug stamps), one GPU.
# Usage: bash tools/gpu_rss_ranks.sh TAG [GIB]
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-rssr}
mkdir -p $O
CLI=$GRAFT_REPO_ROOT/build/MapReduce
F=/tmp/locust_rssr_$$.txt
timeout -k 10 200 $CLI --gen $F --gen-bytes $((${2:-2}<<30)) --seed 7 > /dev/null
for g in 1 2 4 8; do
  LOCUST_LOG=debug timeout -k 10 300 $CLI $F --gpus $g --comm loopback --quiet > /dev/null 2> $O/g$g.err || true
  echo "== --gpus $g"; grep -E "engine built|shard ready|map done|after the job|with the streaming" $O/g$g.err | grep -E "rank 0|r0\]|INFO" | sed 's/malloc in use.*//'
done
GPU_MAX_HW_QUEUES=2 LOCUST_LOG=debug timeout -k 10 300 $CLI $F --gpus 8 --comm loopback --quiet > /dev/null 2> $O/g8q2.err || true
echo "== --gpus 8, GPU_MAX_HW_QUEUES=2"; grep -E "engine built|map done|after the job" $O/g8q2.err | grep -E "rank 0|r0\]|INFO" | sed 's/malloc in use.*//'
rm -f $F
