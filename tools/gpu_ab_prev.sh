# Separate-process A/B of the current build against a control worktree (ab/prev, built
# in-tree), same box, alternating: the bench's headline and its 700-line config.
# Usage: bash tools/gpu_ab_prev.sh TAG [ROUNDS]
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-abprev}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_switches.py tests/test_dist.py tests/test_compact.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in $(seq 1 ${2:-3}); do
  for v in prev now; do
    if [ $v = prev ]; then B=ab/prev/bench.py; else B=bench.py; fi
    timeout -k 10 200 python $B --steps 400 --warmup 50 --no-extra > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { tail -20 $O/b_${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b_${v}_$i.json'));print('$v', d['value'], d.get('hamlet700',{}).get('ms_per_step'))"
  done
done
