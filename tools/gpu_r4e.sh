# Headline kernels, fused vs two launches, compact vs 40-B: kernel stats of the CLI on whole
# Hamlet under each setting, ordered-kernel phase traces, and the in-process A/B.
# Usage: bash tools/gpu_r4e.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_dist.py tests/test_switches.py \
  tests/test_compact.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
CLI=$GRAFT_REPO_ROOT/build/MapReduce
H=$GRAFT_REPO_ROOT/data/hamlet.txt
cd /tmp
for v in "fused:LOCUST_FUSE=1" "two:LOCUST_FUSE=0" "two40:LOCUST_FUSE=0 LOCUST_COMPACT_OUT=0" "fused40:LOCUST_FUSE=1 LOCUST_COMPACT_OUT=0"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/k_$n -o run --output-format csv -- $CLI $H --warmup 5 --iters 40 --quiet > /dev/null
  echo "== $n ($e)"; python3 $GRAFT_REPO_ROOT/tools/kstats.py $O/k_$n/run_kernel_stats.csv | head -3
done
cd $GRAFT_REPO_ROOT
LOCUST_FUSE=0 LOCUST_ORD_TRACE=1 timeout -k 10 60 $CLI $H --warmup 5 --iters 3 --quiet > /dev/null 2> $O/ordtrace_two.txt || true
tail -12 $O/ordtrace_two.txt
timeout -k 10 200 python tools/env_ab.py "LOCUST_FUSE=1" "LOCUST_FUSE=0" "LOCUST_FUSE=0,LOCUST_COMPACT_OUT=0" --config hamlet4500 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
tail -3 $O/ab.txt
# where a multi-rank file job's host memory goes: per-rank RSS stamps (LOCUST_LOG=debug)
F=/tmp/locust_rss_$$.txt
timeout -k 10 200 $CLI --gen $F --gen-bytes $((4<<30)) --seed 7 > /dev/null
LOCUST_LOG=debug timeout -k 10 300 $CLI $F --gpus 8 --comm loopback --quiet --json $O/rss8.json > /dev/null 2> $O/rss8.err || true
rm -f $F
grep -E "rss|engine \(" $O/rss8.err | head -40
# control: the round-3 closing build (a worktree under ab/r3, built in-tree), same box
if [ -x ab/r3/build/MapReduce ]; then
  cd /tmp
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/k_r3 -o run --output-format csv -- $GRAFT_REPO_ROOT/ab/r3/build/MapReduce $H --warmup 5 --iters 40 --quiet > /dev/null
  echo "== r3 control"; python3 $GRAFT_REPO_ROOT/tools/kstats.py $O/k_r3/run_kernel_stats.csv | head -3
  cd $GRAFT_REPO_ROOT
  timeout -k 10 200 python ab/r3/bench.py --steps 200 --warmup 20 --no-extra > $O/bench_r3.json 2> $O/bench_r3.err && python -c "import json;print('r3 control headline', json.load(open('$O/bench_r3.json'))['value'])"
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-extra > $O/bench_now.json 2> $O/bench_now.err && python -c "import json;print('now headline', json.load(open('$O/bench_now.json'))['value'])"
fi
