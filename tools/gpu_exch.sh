# One-RCCL-rank synth1m: forced shuffle vs gather vs local job times (tools/exch_prof.py),
# then kernel stats of the shuffle jobs.  Usage: bash tools/gpu_exch.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-exch}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/exch_prof.py --jobs 30 > $O/exch_prof.txt 2>&1 || { tail -20 $O/exch_prof.txt; exit 1; }
grep -E "shuffle|gather|local" $O/exch_prof.txt | tail -5
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kexch -o kexch --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/exch_prof.py --jobs 20 > $O/kexch.log 2>&1 || { tail -20 $O/kexch.log; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/kstats.py $O/kexch/kexch_kernel_stats.csv | head -12
