# Radix-path cycle: its GPU tests, the radix bench extra and a kernel trace of the CLI
# with --sort radix.  Usage: bash tools/gpu_radix.sh TAG [pytest -k expression]
set -e
cd $GRAFT_REPO_ROOT
T=${1:-radix}
K=${2:-"psort or gpu_engine or cli_gpu"}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "$K" --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 300 python - > $O/radix_bench.json <<'PY'
import json, bench
t = bench.load_text("hamlet4500")
out = {}
for sort in ("radix", "dict"):
    ms, st, res = bench.bench_single(t, 200, 20, sort=sort)
    out[sort] = {"ms_per_step": round(ms, 4), "stages_ms": {k: round(v, 4) for k, v in st.items()},
                 "unique": res.num_unique}
print(json.dumps(out))
PY
cat $O/radix_bench.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kradix -o run --output-format csv -- $GRAFT_REPO_ROOT/build/MapReduce $GRAFT_REPO_ROOT/data/hamlet.txt --sort radix --warmup 10 --iters 40 --quiet > /dev/null
cd $GRAFT_REPO_ROOT
python3 tools/kstats.py $O/kradix/run_kernel_stats.csv | tee $O/kradix.summary.txt
python3 tools/ktimeline.py $O/kradix/run_kernel_trace.csv 8 | tee $O/kradix.timeline.txt
