# Kernel statistics of synth1m jobs (tools/steps.py) per LOCUST_ORD_VARIANT value, one
# rocprofv3 run each.  Usage: bash tools/gpu_variant_kstats.sh TAG V...
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-vk}
shift
mkdir -p $O
export TMPDIR=/tmp
for v in "$@"; do
  (cd /tmp && LOCUST_ORD_VARIANT=$v PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/v$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/steps.py 1000000 30 > $O/v$v.steps.txt 2>&1)
  echo "== variant $v: $(grep '^mean' $O/v$v.steps.txt)"
  python3 tools/kstats.py $O/v$v/run_kernel_stats.csv | head -4
done
