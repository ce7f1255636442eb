# The whole GPU suite, then separate-process A/B (alternating) against ab/prev on the
# headline and synth1m.  Usage: bash tools/gpu_ab_both.sh TAG [ROUNDS]
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-aball}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in $(seq 1 ${2:-3}); do
  for v in prev now; do
    if [ $v = prev ]; then B=ab/prev/bench.py; else B=bench.py; fi
    timeout -k 10 200 python $B --steps 400 --warmup 50 --no-extra > $O/h_${v}_$i.json 2> $O/h_${v}_$i.err || { tail -20 $O/h_${v}_$i.err; exit 1; }
    timeout -k 10 200 python $B --config synth1m --steps 100 --warmup 10 --no-extra > $O/s_${v}_$i.json 2> $O/s_${v}_$i.err || { tail -20 $O/s_${v}_$i.err; exit 1; }
    python3 -c "import json;h=json.load(open('$O/h_${v}_$i.json'));s=json.load(open('$O/s_${v}_$i.json'));print('$v headline', h['value'], 'B/key', h.get('output_bytes_per_key'), 'synth1m', s['ms_per_step'], 'B/key', s.get('output_bytes_per_key'))"
  done
done
