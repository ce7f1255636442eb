# Shared output regions + pinned-allocation log: distributed GPU tests, then the 8-rank
# RSS breakdown.  Usage: bash tools/gpu_r4j.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4j}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dist.py tests/test_dist_procs.py tests/test_file_shards.py tests/test_scale_ready.py tests/test_cli_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash tools/gpu_rss8.sh ${1:-r4j} 4
grep -E "pinned" $O/rss8.err | sort | uniq -c | sort -rn | head -20
