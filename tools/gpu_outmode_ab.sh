# Host output buffers: fine-grained (default, records written straight over PCIe) vs
# coarse-grained (LOCUST_OUT_NONCOHERENT=1: written through the L2, flushed by the
# system-scope release) -- whole Hamlet and 700 lines, lean jobs, then synth1m.
# Usage: bash tools/gpu_outmode_ab.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-outmode}
mkdir -p $O
for i in 1 2; do for nc in 0 1; do
  LOCUST_OUT_NONCOHERENT=$nc timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --no-extra > $O/h_$nc.json
  LOCUST_OUT_NONCOHERENT=$nc timeout -k 10 120 python bench.py --config synth1m --steps 40 --warmup 5 > $O/s_$nc.json
  echo "nc=$nc hamlet $(python3 -c "import json;print(json.load(open('$O/h_$nc.json'))['value'])") synth1m $(python3 -c "import json;print(json.load(open('$O/s_$nc.json'))['value'])")"
done; done
