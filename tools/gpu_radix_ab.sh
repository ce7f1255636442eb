# Radix path A/B: LOCUST_PSORT_VARIANT / LOCUST_RADIX_FUSED settings, kernel stats each.
# Usage: bash tools/gpu_radix_ab.sh TAG "ENV=v ..." ...
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-radixab}
shift
mkdir -p $O
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  cd /tmp
  env $v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/v$i -o run --output-format csv -- $GRAFT_REPO_ROOT/build/MapReduce $GRAFT_REPO_ROOT/data/hamlet.txt --sort radix --warmup 5 --iters 40 --quiet > /dev/null 2>&1
  cd $GRAFT_REPO_ROOT
  echo "== $v"
  python3 tools/kstats.py $O/v$i/run_kernel_stats.csv | head -3
  env $v timeout -k 10 120 ./build/MapReduce data/hamlet.txt --sort radix --warmup 20 --iters 200 --quiet --json $O/v$i.json > /dev/null
  python3 -c "import json;d=json.load(open('$O/v$i.json'));print('job median ms', d['wall_ms_median'])"
done
