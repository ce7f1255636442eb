set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6f
mkdir -p $O
for q in 1 2; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python tools/cli_cold.py --runs 5 --out $O/cli_cold_hwq$q.txt > /dev/null
  grep -E "process_ms|exit_ms|runtime_init|engine_ms" $O/cli_cold_hwq$q.txt | head -5
done
timeout -k 10 900 python tools/partmap_heldout.py --out $O/partmap_heldout.md --rounds 3
cat $O/partmap_heldout.md
