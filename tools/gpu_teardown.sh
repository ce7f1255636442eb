# Streamed-copy slowdown after another device user's teardown: the copy micro per teardown
# step, then the synth10g per-job probe.  Usage: bash tools/gpu_teardown.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-teardown}
mkdir -p $O
for s in none stream mapped devfree all; do
  timeout -k 10 120 ./build/copy_teardown $s 4 >> $O/copy_teardown.txt 2>&1
done
PYTHONPATH=. timeout -k 10 400 python -u tools/s10g_probe.py 10 4 > $O/s10g_probe.txt 2>&1
