set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_full.sh r6l
timeout -k 10 600 bash tools/gpu_profile.sh r6l/prof > gpurun_out/r6l/prof.log 2>&1 || { tail -20 gpurun_out/r6l/prof.log; exit 1; }
grep -E "map_fast|dict_ordered" gpurun_out/r6l/prof/k4500.summary.txt || true
grep -A2 "map_fast_kernel" gpurun_out/r6l/prof/pmc_summary.txt | tail -1 || true
timeout -k 10 600 bash tools/gpu_hbm.sh r6l/hbm 10 8 > gpurun_out/r6l/hbm.log 2>&1 || { tail -20 gpurun_out/r6l/hbm.log; exit 1; }
cat gpurun_out/r6l/hbm/summary.txt
timeout -k 10 120 python tools/cli_cold.py --runs 7 --out gpurun_out/r6l/cli_cold.txt > /dev/null
head -14 gpurun_out/r6l/cli_cold.txt
