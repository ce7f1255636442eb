# The starting partition map (letters split on the second byte) against the first-byte
# map: GPU tests, in-process A/B of the headline with the retune off and on, kernel stats
# and phase traces (tools/gpu_untuned.sh), the bench line.  Usage: bash tools/gpu_pmdefault.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pm}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
PYTHONPATH=. timeout -k 10 300 python -u tools/env_ab.py "LOCUST_PART_TUNE=0,LOCUST_PART_DEFAULT=byte" "LOCUST_PART_TUNE=0" "LOCUST_PART_DEFAULT=byte" "LOCUST_PART_TUNE=1" --steps 300 --rounds 4 > $O/env_ab.txt 2>&1
tail -5 $O/env_ab.txt
bash tools/gpu_untuned.sh ${1:-pm} > /dev/null
head -2 $O/k0.summary.txt
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
python3 -c "
import json; d = json.load(open('$O/bench.json')); print(d['value'], d['untuned'], d['cold_start'], d['synth1m']['ms_per_step'])"
