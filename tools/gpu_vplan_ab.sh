# A/B of the ordered kernel's in-job workgroup plan (LOCUST_VPLAN) with and without the
# between-job partition retuning (LOCUST_PART_TUNE), plus an untuned phase trace.
# Usage: bash tools/gpu_vplan_ab.sh TAG
set -e
timeout -k 10 600 python -u -m pytest tests/test_large_ordered.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${1:-vplan}_pytest.txt 2>&1 || { tail -40 gpurun_out/${1:-vplan}_pytest.txt; exit 1; }
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-vplan}
mkdir -p $O
V="LOCUST_VPLAN=1 LOCUST_VPLAN=0 LOCUST_VPLAN=1,LOCUST_PART_TUNE=0 LOCUST_VPLAN=0,LOCUST_PART_TUNE=0"
timeout -k 10 300 python tools/env_ab.py $V --rounds 5 > $O/ab_hamlet4500.txt 2>&1 || { tail -30 $O/ab_hamlet4500.txt; exit 1; }
cat $O/ab_hamlet4500.txt
timeout -k 10 300 python tools/env_ab.py $V --rounds 5 --config hamlet700 > $O/ab_hamlet700.txt 2>&1 || { tail -30 $O/ab_hamlet700.txt; exit 1; }
cat $O/ab_hamlet700.txt
for vp in 1 0; do
  LOCUST_VPLAN=$vp LOCUST_PART_TUNE=0 LOCUST_ORD_TRACE=1 timeout -k 10 120 python -c "
import bench, locust_amd as lc
t = bench.load_text('hamlet4500')
e = lc._C.GpuEngine(lc.make_config('gpu', reduce_path='lds'), len(t), bench._nlines(t))
e.load(t)
for _ in range(6): e.run_loaded()
" > $O/ordtrace_untuned_vplan$vp.txt 2>&1 || { tail -30 $O/ordtrace_untuned_vplan$vp.txt; exit 1; }
  grep "ord span" $O/ordtrace_untuned_vplan$vp.txt | tail -3
done
timeout -k 10 300 python tools/env_ab.py LOCUST_VPLAN=1 LOCUST_VPLAN=0 --rounds 3 --steps 40 --config synth1m > $O/ab_synth1m.txt 2>&1 || { tail -30 $O/ab_synth1m.txt; exit 1; }
cat $O/ab_synth1m.txt
timeout -k 10 300 python tools/env_ab.py LOCUST_DEVPLAN=1 LOCUST_DEVPLAN=0 "LOCUST_DEVPLAN=0,LOCUST_PART_TUNE=0" --rounds 3 --steps 40 --config synth1m > $O/ab_devplan_synth1m.txt 2>&1 || { tail -30 $O/ab_devplan_synth1m.txt; exit 1; }
cat $O/ab_devplan_synth1m.txt
for dp in 1 0; do
  LOCUST_DEVPLAN=$dp timeout -k 10 120 python -c "
import bench, json
t = bench.synth_shard('synth1m', 0, 1)
print('devplan=$dp cold', json.dumps(bench.cold_first_run(t)))
" 2>&1 | tail -1
done
