set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_scale_ready.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/pytest_scale.txt 2>&1 || { tail -40 $O/pytest_scale.txt; exit 1; }
tail -2 $O/pytest_scale.txt
timeout -k 10 400 bash tools/gpu_stage10g.sh r6b/s10b 10 8 3 bytes
timeout -k 10 400 bash tools/gpu_stage10g.sh r6b/s10l 10 8 3 lines
# one map window's construction / first-job phases (debug log)
D=/tmp/locust_dbg_$$; mkdir -p $D
timeout -k 10 200 ./build/MapReduce --gen $D/f.txt --gen-bytes $((2<<30)) --seed 7 > /dev/null
S=$(stat -c %s $D/f.txt)
LOCUST_LOG=debug timeout -k 10 120 ./build/MapReduce $D/f.txt 0 0 0 1 --byte-range $((S/2)):$S --spill-dir $D --spill-format binary --json $O/dbg_map.json > /dev/null 2> $O/dbg_map.err
LOCUST_LOG=debug timeout -k 10 120 ./build/MapReduce $D/f.txt 0 0 1 1 --byte-range 0:$((S/2)) --spill-dir $D --spill-format binary --json $O/dbg_map2.json > /dev/null 2> $O/dbg_map2.err
rm -rf $D
grep -E "engine \(|ms" $O/dbg_map.err | head -30
cat $O/dbg_map.json
