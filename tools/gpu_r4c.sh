# Round-4 fused map + ordered launch: tests, A/Bs in one process (fused vs two launches,
# compact vs 40-B output), the one-rank shuffle, the default bench and kernel profiles.
# Usage: bash tools/gpu_r4c.sh TAG
set -e
cd $GRAFT_REPO_ROOT
T=${1:-r4c}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_switches.py tests/test_dist.py \
  tests/test_cli_gpu.py tests/test_compact.py -x -v --timeout 200 --timeout-method thread -m gpu \
  > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for c in hamlet4500 hamlet700; do
  timeout -k 10 200 python tools/env_ab.py "LOCUST_FUSE=1" "LOCUST_FUSE=0" "LOCUST_FUSE=1,LOCUST_COMPACT_OUT=0" \
    --config $c > $O/ab_$c.txt 2>&1 || { tail -20 $O/ab_$c.txt; exit 1; }
  tail -3 $O/ab_$c.txt
done
timeout -k 10 200 python tools/exch_prof.py --jobs 30 > $O/exch_prof.txt 2>&1 || { tail -20 $O/exch_prof.txt; exit 1; }
tail -5 $O/exch_prof.txt
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('headline',d['value'],'untuned',d['untuned'],'700',d['hamlet700']['ms_per_step'],'synth1m',d['synth1m']['ms_per_step'],d['synth1m']['GB_per_s'])"
bash tools/gpu_profile.sh $T/prof > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep -A4 "== k4500\|== ksynth\|== kexch" $O/prof.log | head -30
