set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
make -q -j8 >/dev/null 2>&1 || echo "make not up to date (rebuilding)"
timeout -k 10 300 ./build/MapReduce data/hamlet.txt 0 700 > gpurun_out/gpu700.txt 2> gpurun_out/gpu700.err && echo cli700 ok
head -8 gpurun_out/gpu700.txt
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.txt 2>&1; echo pytest rc=$?
tail -30 gpurun_out/pytest_gpu.txt
