set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_full.sh r6p
timeout -k 10 600 bash tools/gpu_stage10g.sh r6p/s10 10 8 3 bytes > gpurun_out/r6p/stage.txt 2>&1 || { tail -30 gpurun_out/r6p/stage.txt; exit 1; }
cat gpurun_out/r6p/s10/summary.txt
timeout -k 10 120 python tools/cli_cold.py --runs 7 --out gpurun_out/r6p/cli_cold.txt > /dev/null
head -12 gpurun_out/r6p/cli_cold.txt
