# A --gen-made large file through ./MapReduce at --gpus 1 (run_direct) and --gpus N
# (per-rank byte ranges; loopback ranks share the box's GPU unless the node has N GPUs):
# identical result lines, per-rank bytes read and the process's peak RSS.
# Usage: bash tools/gpu_bigfile_ranks.sh TAG [GIB] [N] [COMM]
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-bigranks}
G=${2:-10}
N=${3:-8}
C=${4:-loopback}
mkdir -p $O
F=/tmp/locust_bigr_$$.txt
trap 'rm -f $F $F.1 $F.n' EXIT
timeout -k 10 300 ./build/MapReduce --gen $F --gen-bytes $((G<<30)) --seed 7 > $O/gen.txt
t0=$(date +%s.%N)
timeout -k 10 300 ./build/MapReduce $F --json $O/one.json > $F.1
t1=$(date +%s.%N)
LOCUST_LOG=info timeout -k 10 600 ./build/MapReduce $F --gpus $N --comm $C --json $O/ranks.json > $F.n 2> $O/ranks.err
t2=$(date +%s.%N)
grep '^print key' $F.1 > $F.1.k; grep '^print key' $F.n > $F.n.k
if cmp -s $F.1.k $F.n.k; then same=identical; else same=DIFFERENT; fi
rm -f $F.1.k $F.n.k
python3 - $O/one.json $O/ranks.json $G $t0 $t1 $t2 "$same" <<'PY' | tee $O/summary.txt
import json, sys
one, rk = json.load(open(sys.argv[1])), json.load(open(sys.argv[2]))
gib, t0, t1, t2, same = float(sys.argv[3]), *map(float, sys.argv[4:7]), sys.argv[7]
print(f"{gib:.0f} GiB file, --gpus 1: process {t1 - t0:.2f} s, peak RSS {one['max_rss_kb']} kB, "
      f"unique {one['unique']}")
print(f"--gpus {len(rk['ranks'])}: process {t2 - t1:.2f} s, job {rk['wall_ms']:.1f} ms, "
      f"peak RSS {rk['peak_rss_kb']} kB, unique {rk['unique']}, result lines {same}")
for r in rk["ranks"]:
    print(f"  rank {r['rank']}: read {r['input_bytes']} B streamed={r['input_streamed']} "
          f"peers_p2p={r['peer_p2p']} map {r['map_ms']:.1f} ms shuffle {r['shuffle_ms']:.1f} ms "
          f"syncs {r['host_syncs']}")
PY
