# Root-merge kernel profiles in isolation (tools/merge_prof.py): 8 runs of a full Hamlet
# each, and 8 runs of a 1/8 chunk each.  Summaries: gpurun_out/$T/*.txt
set -e
cd $GRAFT_REPO_ROOT
T=${1:-mergeprof}
R=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $R
cd /tmp && export TMPDIR=/tmp
for shape in full chunk; do
  flag=""; [ $shape = chunk ] && flag="--chunk"
  timeout -k 10 120 rocprofv3 --kernel-trace -d $R/$shape -o p -- \
    python3 $GRAFT_REPO_ROOT/tools/merge_prof.py 8 30 $flag > $R/$shape.log 2>&1
  python3 $GRAFT_REPO_ROOT/tools/kstats.py $R/$shape > $R/$shape.txt
  echo "== $shape"; tail -1 $R/$shape.log; grep merge $R/$shape.txt
done
