# GPU tests, then the small-pass plan threshold A/B (untuned headline; plan forced on vs the
# size threshold) and the bench line.  Usage: bash tools/gpu_plan_ab.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-plan}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
PYTHONPATH=. timeout -k 10 300 python -u tools/env_ab.py "LOCUST_PART_TUNE=0,LOCUST_VPLAN_MIN_KB=0" "LOCUST_PART_TUNE=0" "LOCUST_PART_TUNE=0,LOCUST_VPLAN_MIN_KB=0,LOCUST_PART_DEFAULT=byte" "LOCUST_PART_TUNE=1" --steps 300 --rounds 4 > $O/env_ab.txt 2>&1
tail -4 $O/env_ab.txt
PYTHONPATH=. timeout -k 10 300 python -u tools/env_ab.py "LOCUST_PART_TUNE=0,LOCUST_VPLAN_MIN_KB=0" "LOCUST_PART_TUNE=0" "LOCUST_PART_TUNE=1" --config hamlet700 --steps 300 --rounds 4 > $O/env_ab700.txt 2>&1
tail -3 $O/env_ab700.txt
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
python3 -c "
import json; d = json.load(open('$O/bench.json')); print(d['value'], d['untuned'], d['cold_start'], d['synth1m']['ms_per_step'], d['radix_path']['ms_per_step'])"
