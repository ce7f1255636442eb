# RCCL env A/B on the one-rank distributed bench: API call counts + ms/job per setting.
# Usage: bash tools/gpu_rccl_env_ab.sh TAG "VAR=v VAR2=v" ["VAR=v" ...]
set -e
cd $GRAFT_REPO_ROOT
T=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
i=0
for setting in "" "$@"; do
  i=$((i+1))
  cd /tmp
  env_args=$setting
  ( export $env_args MASTER_ADDR=127.0.0.1 MASTER_PORT=2967$i; timeout -k 10 200 rocprofv3 --hip-trace --stats -d $O/r$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --force-dist --no-extra --steps 200 --warmup 20 > $O/r$i.json 2> $O/r$i.err )
  cd $GRAFT_REPO_ROOT
  python3 - "$O/r$i" "$setting" <<'PY'
import csv, json, sys
d = sys.argv[1]
rows = {r["Name"]: int(r["Calls"]) for r in csv.DictReader(open(d + "/run_hip_api_stats.csv"))}
j = json.loads(open(d + ".json").read().strip().splitlines()[-1])
print(repr(sys.argv[2]), "ms/job", j["value"], {k: rows.get(k, 0) for k in ("hipExtMallocWithFlags", "hipFree", "hipMemsetAsync", "hipMemcpyAsync")})
PY
done
