# Multi-rank file path after the RSS changes: GPU tests of the file ranks and CLI, the
# 8-rank RSS breakdown (4 GiB) and the 10 GiB file at --gpus 8.  Usage: bash tools/gpu_r4k.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4k}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_file_shards.py tests/test_cli_gpu.py tests/test_scale_ready.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash tools/gpu_rss8.sh ${1:-r4k} 4 | grep -E "INFO|peak_rss|map done" | grep -E "INFO|peak|r0\]"
bash tools/gpu_bigfile_ranks.sh ${1:-r4k}/big10 10 8
