# Large-partition sort in the ordered kernel: LDS radix (default) vs bucket + all-pairs
# ranks (LOCUST_ORD_VARIANT=16), synth1m jobs and the ordered kernel's span.
# Usage: bash tools/gpu_largesort_ab.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-lsab}
mkdir -p $O
CLI=$GRAFT_REPO_ROOT/build/MapReduce
$CLI --gen /tmp/synth1m.txt --gen-lines 1000000 --seed 1 > /dev/null
for i in 1 2; do for v in 0 16; do
  LOCUST_ORD_VARIANT=$v PYTHONPATH=. timeout -k 10 100 python tools/steps.py 1000000 40 > $O/st_$v.txt 2>&1
  echo "variant=$v $(tail -1 $O/st_$v.txt)"
done; done
for v in 0 16; do
  LOCUST_ORD_VARIANT=$v LOCUST_ORD_TRACE=1 timeout -k 10 120 $CLI /tmp/synth1m.txt --warmup 2 --iters 1 --quiet > /dev/null 2> $O/trace_$v.txt
  echo "variant=$v $(grep 'ord span' $O/trace_$v.txt | tail -1)"
done
