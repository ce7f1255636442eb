# synth1m A/B (separate processes, alternating) of the current build against the control
# worktree ab/prev, plus the ordered kernel's phase trace on synth1m and GPU tests.
# Usage: bash tools/gpu_ab_synth.sh TAG [ROUNDS]
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-absynth}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_compact.py tests/test_dist.py tests/test_switches.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash tools/gpu_ordtrace_synth.sh ${1:-absynth}/ots > /dev/null
grep "ord span" $O/ots/trace.txt | tail -1
for i in $(seq 1 ${2:-3}); do
  for v in prev now; do
    if [ $v = prev ]; then B=ab/prev/bench.py; else B=bench.py; fi
    timeout -k 10 200 python $B --config synth1m --steps 100 --warmup 10 --no-extra > $O/s_${v}_$i.json 2> $O/s_${v}_$i.err || { tail -20 $O/s_${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/s_${v}_$i.json'));print('$v', d['value'], d['ms_per_step'])"
  done
done
