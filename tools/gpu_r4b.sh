# Round-4 fused shuffle tail + compact output: the exchange / shared-output tests, the switch
# sweep, compact-vs-40-B A/B in one process, and the one-RCCL-rank synth1m shuffle profile.
# Usage: bash tools/gpu_r4b.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dist.py tests/test_stream.py tests/test_dist_procs.py \
  tests/test_scale_ready.py tests/test_switches.py tests/test_compact.py -x -v --timeout 200 \
  --timeout-method thread -m gpu > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for c in hamlet4500 hamlet700 synth1m; do
  timeout -k 10 200 python tools/env_ab.py "LOCUST_COMPACT_OUT=1" "LOCUST_COMPACT_OUT=0" --config $c \
    > $O/ab_$c.txt 2>&1 || { tail -20 $O/ab_$c.txt; exit 1; }
  tail -4 $O/ab_$c.txt
done
timeout -k 10 200 python tools/exch_prof.py --jobs 30 > $O/exch_prof.txt 2>&1 || { tail -20 $O/exch_prof.txt; exit 1; }
tail -8 $O/exch_prof.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kexch -o kexch -- python3 tools/exch_prof.py --jobs 20 > $O/kexch.log 2>&1 || { tail -20 $O/kexch.log; exit 1; }
python3 tools/kstats.py $O/kexch > $O/kexch.summary.txt 2>&1 || true
head -12 $O/kexch.summary.txt
timeout -k 10 200 python tools/rss_engines.py --engines 8 --mb 512 > $O/rss_engines.txt 2>&1 || { tail -20 $O/rss_engines.txt; exit 1; }
cat $O/rss_engines.txt
