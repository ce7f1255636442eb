# zero-copy A/B + GPU tests.  Usage: bash tools/gpu_zc.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-zc}
mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.txt 2>&1 || { tail -60 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
for z in 0 1; do
LOCUST_ZERO_COPY=$z timeout -k 10 300 python bench.py > $O/bench_zc$z.json 2> $O/bench_zc$z.err || { tail -30 $O/bench_zc$z.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_zc$z.json'));print('zc=$z', d['value'], d['stages_ms_median'], d['hamlet700']['ms_per_step'])"
done
timeout -k 10 300 python bench.py --config synth1m --steps 20 --warmup 3 > $O/synth1m.json 2> $O/synth1m.err || { tail -30 $O/synth1m.err; exit 1; }
python -c "import json;d=json.load(open('$O/synth1m.json'));print('synth1m', d['value'], d['stages_ms_median'], d['GB_per_s'])"
