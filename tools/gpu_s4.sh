# Round-3 session-4 check: GPU tests, the synth10g per-engine probe, the synth10g and
# default bench lines.  Usage: bash tools/gpu_s4.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-s4}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
PYTHONPATH=. timeout -k 10 400 python -u tools/s10g_probe.py 10 3 > $O/s10g_probe.txt 2>&1
cat $O/s10g_probe.txt
timeout -k 10 600 python bench.py --config synth10g --steps 3 --warmup 1 > $O/synth10g.json 2> $O/synth10g.err || { tail -30 $O/synth10g.err; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "
import json
for f in ['synth10g', 'bench']:
    d = json.load(open('$O/' + f + '.json')); print(f, d['value'], d.get('GB_per_s'), d.get('synth1m', {}).get('ms_per_step'))
"
