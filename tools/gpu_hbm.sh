# HBM budget: a GIB GiB file over N loopback ranks on the ONE GPU
# (every rank streams its 1/N byte range in 256 MiB chunks, 32 MiB map windows) -- each
# rank's engine device memory (plan_device_pass), the GPU's memory in use after the job,
# and the result lines against the one-rank run.  Then a one-pass 256 MiB file through
# ./MapReduce (the single-engine arena) and an oversize --chunk-mb, which must be refused.
# Usage: bash tools/gpu_hbm.sh TAG [GIB] [N]
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-hbm}
G=${2:-10}
N=${3:-8}
mkdir -p $O
export TMPDIR=/tmp
CLI=$GRAFT_REPO_ROOT/build/MapReduce
D=/tmp/locust_hbm_$$
mkdir -p $D
trap 'rm -rf $D' EXIT
F=$D/big.txt
timeout -k 10 300 $CLI --gen $F --gen-bytes $((G<<30)) --seed 7 > /dev/null
timeout -k 10 300 $CLI $F --json $O/one.json | grep "^print key:" > $D/one.lines
timeout -k 10 300 $CLI $F --gpus $N --comm loopback --json $O/ranks.json | grep "^print key:" > $D/ranks.lines
cmp $D/one.lines $D/ranks.lines && echo "$N ranks == one rank ($(wc -l < $D/one.lines) lines)" | tee $O/summary.txt
python3 - $O <<'PY' | tee -a $O/summary.txt
import json, sys
o = sys.argv[1]
one = json.load(open(f"{o}/one.json"))
d = json.load(open(f"{o}/ranks.json"))
GiB = 1 << 30
print("one rank: engine %.2f GiB (chunk %d MiB, window %d MiB), GPU free before %.1f of %.1f GiB"
      % (one["hbm_device_bytes"] / GiB, one["device_chunk_bytes"] >> 20, one["device_map_window"] >> 20,
         one["hbm_free_bytes"] / GiB, one["hbm_total_bytes"] / GiB))
tot = d["hbm_total_bytes"]
for r in d["ranks"]:
    print("rank %d: engine %.2f GiB, input %d MiB streamed=%s" % (r["rank"], r["hbm_device_bytes"] / GiB,
          r["input_bytes"] >> 20, r["input_streamed"]))
print("%d ranks: engines %.2f GiB = %.1f %% of HBM; GPU memory in use after the job %.2f GiB = %.1f %%"
      % (len(d["ranks"]), d["hbm_device_bytes"] / GiB, 100 * d["hbm_device_bytes"] / tot,
         d["hbm_used_bytes_max"] / GiB, 100 * d["hbm_used_bytes_max"] / tot))
PY
head -c $((256<<20)) $F > $D/p256.txt
timeout -k 10 120 $CLI $D/p256.txt --quiet --json $O/p256.json > /dev/null
python3 -c "import json; d=json.load(open('$O/p256.json')); print('256 MiB one pass: engine %.2f GiB, streaming %s' % (d['hbm_device_bytes']/2**30, d['device_streaming']))" | tee -a $O/summary.txt
timeout -k 10 120 $CLI $F --chunk-mb 400000 --quiet > /dev/null 2> $O/oversize.err && { echo "oversize chunk was not refused"; exit 1; }
echo "oversize --chunk-mb refused: $(cat $O/oversize.err)" | tee -a $O/summary.txt
