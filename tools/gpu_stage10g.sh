# The reference's stage split at 10 GiB: a --gen-made file mapped as
# N line windows (N stage-1 processes, each reading only its window: combined, indexed
# spills), then one stage 2 over all spills and R key-range reducers; the result lines must
# equal the single-stage run's.  Prints every process's peak RSS, wall time and spill size.
# Usage: bash tools/gpu_stage10g.sh TAG [GIB] [WINDOWS] [REDUCERS]
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-stage10g}
G=${2:-10}
N=${3:-8}
R=${4:-3}
mkdir -p $O
D=/tmp/locust_stage_$$
F=$D/big.txt
mkdir -p $D
trap 'rm -rf $D' EXIT
timeout -k 10 300 ./build/MapReduce --gen $F --gen-bytes $((G<<30)) --seed 7 > $O/gen.txt
L=$(python3 -c "import locust_amd as l; print(l._C.find_line_window('$F', 0, -1)[2])")
echo "$G GiB, $L lines, $N windows, $R reducers" | tee $O/summary.txt
t0=$(date +%s.%N)
timeout -k 10 300 ./build/MapReduce $F --json $O/single.json > $D/single.out
t1=$(date +%s.%N)
grep "^print key:" $D/single.out > $D/single.lines
python3 -c "import json,sys; d=json.load(open('$O/single.json')); print('single stage: %.2f s process, peak RSS %d kB, unique %d' % ($t1-$t0, d['max_rss_kb'], d['unique']))" | tee -a $O/summary.txt
INPUTS=""
for k in $(seq 0 $((N-1))); do
  s=$((L*k/N)); e=$((L*(k+1)/N))
  t0=$(date +%s.%N)
  timeout -k 10 300 ./build/MapReduce $F $s $e $k 1 --spill-dir $D --spill-format binary --json $O/map$k.json > $O/map$k.out
  t1=$(date +%s.%N)
  python3 -c "import json; d=json.load(open('$O/map$k.json')); print('map %d [%d, %d): %.2f s process, job %.1f ms, streamed %s, spill %d B (%d records), peak RSS %d kB' % ($k, $s, $e, $t1-$t0, d['job_ms'], d['streamed'], d['spill_bytes'], d['spill_records'], d['peak_rss_kb']))" | tee -a $O/summary.txt
  INPUTS="$INPUTS${INPUTS:+,}$D/out.$k.kv"
done
t0=$(date +%s.%N)
timeout -k 10 300 ./build/MapReduce $F 0 0 0 2 --inputs $INPUTS --json $O/reduce.json > $D/reduce.out
t1=$(date +%s.%N)
grep "^print key:" $D/reduce.out > $D/reduce.lines
python3 -c "import json; d=json.load(open('$O/reduce.json')); print('reduce: %.2f s process, read %.1f ms, setup %.1f ms, merge %.1f ms, records %d, peak RSS %d kB' % ($t1-$t0, d['read_ms'], d['setup_ms'], d['merge_ms'], d['input_records'], d['peak_rss_kb']))" | tee -a $O/summary.txt
cmp $D/single.lines $D/reduce.lines && echo "stage split == single stage ($(wc -l < $D/single.lines) lines)" | tee -a $O/summary.txt
rm -f $D/ranges.lines
for r in $(seq 0 $((R-1))); do
  timeout -k 10 300 ./build/MapReduce $F 0 0 $r 2 --inputs $INPUTS --reducer $r/$R --result-file $D/res.$r --json $O/reducer$r.json > /dev/null
  cat $D/res.$r >> $D/ranges.lines
  python3 -c "import json; d=json.load(open('$O/reducer$r.json')); print('reducer $r/$R: records read %d, merged %d, val base %d, peak RSS %d kB' % (d['records_read'], d['input_records'], d['val_base'], d['peak_rss_kb']))" | tee -a $O/summary.txt
done
cmp $D/single.lines $D/ranges.lines && echo "$R key-range reducers == single stage" | tee -a $O/summary.txt
