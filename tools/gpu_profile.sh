# Kernel-trace stats + PMC counters of the headline jobs.  Usage: bash tools/gpu_profile.sh TAG
# (counters in their own runs, never combined with sys/runtime tracing)
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-prof}
mkdir -p $O
export TMPDIR=/tmp
CLI=$GRAFT_REPO_ROOT/build/MapReduce
H=$GRAFT_REPO_ROOT/data/hamlet.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k4500 -o run --output-format csv -- $CLI $H --warmup 5 --iters 20 --quiet > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k700 -o run --output-format csv -- $CLI $H 0 700 --warmup 5 --iters 20 --quiet > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kradix -o run --output-format csv -- $CLI $H --sort radix --warmup 5 --iters 20 --quiet > /dev/null
$CLI --gen /tmp/synth1m.txt --gen-lines 1000000 --seed 1 > /dev/null && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ksynth -o run --output-format csv -- $CLI /tmp/synth1m.txt --warmup 2 --iters 5 --quiet > /dev/null || true
# stage 2 over 4 spills of synth1m line windows: the device merge of sorted runs
if [ -f /tmp/synth1m.txt ]; then
  for k in 0 1 2 3; do
    timeout -k 10 120 $CLI /tmp/synth1m.txt $((k*250000)) $(((k+1)*250000)) $k 1 --spill-dir /tmp --spill-format binary --quiet > /dev/null
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kstage2 -o run --output-format csv -- $CLI x 0 0 0 2 --inputs /tmp/out.0.kv,/tmp/out.1.kv,/tmp/out.2.kv,/tmp/out.3.kv --quiet --json $O/stage2.json > /dev/null || echo "stage-2 profile failed"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kexch -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/exch_prof.py --jobs 20 > $O/kexch.txt 2>&1 || echo "exchange profile failed"
P=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  P=$((P+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $O/pmc$P -o run --output-format csv -- $CLI $H --warmup 2 --iters 5 --quiet > /dev/null || echo "pmc set $P failed: $set"
done
cd $GRAFT_REPO_ROOT
for k in k4500 k700 kradix ksynth kstage2 kexch; do
  [ -f $O/$k/run_kernel_stats.csv ] && { echo "== $k"; python3 tools/kstats.py $O/$k/run_kernel_stats.csv | tee $O/$k.summary.txt; }
done
python3 tools/pmc_summary.py $O/pmc_summary.txt $O/pmc*
