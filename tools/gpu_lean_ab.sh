# Lean direct-launch jobs vs graph replay on the headline configs (alternating runs).
# Usage: bash tools/gpu_lean_ab.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-lean}
mkdir -p $O
for i in 1 2; do
  for v in 1 0; do
    LOCUST_LEAN=$v timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --no-extra > $O/h4500_lean$v.$i.json
    echo "lean=$v h4500 $(python3 -c "import json;print(json.load(open('$O/h4500_lean$v.$i.json'))['value'])")"
    LOCUST_LEAN=$v timeout -k 10 120 python bench.py --config hamlet700 --steps 2000 --warmup 50 --no-extra > $O/h700_lean$v.$i.json
    echo "lean=$v h700 $(python3 -c "import json;print(json.load(open('$O/h700_lean$v.$i.json'))['value'])")"
  done
done
