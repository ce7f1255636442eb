# Fused map + ordered launch vs two launches on whole Hamlet: kernel stats, the ordered
# kernel's phase trace (with the fused launch's tile stamps), and the in-process A/B.
# Usage: bash tools/gpu_r4f.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4f}
mkdir -p $O
export TMPDIR=/tmp
CLI=$GRAFT_REPO_ROOT/build/MapReduce
H=$GRAFT_REPO_ROOT/data/hamlet.txt
timeout -k 10 300 python -u -m pytest tests/test_switches.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
LOCUST_FUSE=1 timeout -k 10 60 $CLI $H > $O/out_fused.txt
LOCUST_FUSE=0 timeout -k 10 60 $CLI $H > $O/out_two.txt
cmp $O/out_fused.txt $O/out_two.txt && echo "fused output identical"
LOCUST_FUSE=1 LOCUST_ORD_TRACE=1 timeout -k 10 60 $CLI $H --warmup 5 --iters 3 --quiet > /dev/null 2> $O/ordtrace_fused.txt
grep -E "span|fused" $O/ordtrace_fused.txt | tail -2
grep "ord p=" $O/ordtrace_fused.txt | tail -6
LOCUST_FUSE=0 LOCUST_ORD_TRACE=1 timeout -k 10 60 $CLI $H --warmup 5 --iters 3 --quiet > /dev/null 2> $O/ordtrace_two.txt
grep -E "span" $O/ordtrace_two.txt | tail -1
cd /tmp
for v in "fused:LOCUST_FUSE=1" "two:LOCUST_FUSE=0"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/k_$n -o run --output-format csv -- $CLI $H --warmup 5 --iters 40 --quiet > /dev/null
  echo "== $n ($e)"; python3 $GRAFT_REPO_ROOT/tools/kstats.py $O/k_$n/run_kernel_stats.csv | head -3
done
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/env_ab.py "LOCUST_FUSE=1" "LOCUST_FUSE=0" --config hamlet4500 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
tail -2 $O/ab.txt
