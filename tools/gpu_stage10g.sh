# The reference's stage split at 10 GiB: a --gen-made file mapped as
# N windows (N stage-1 processes: combined, indexed spills), then one stage 2 over all
# spills and R key-range reducers; the result lines must equal the single-stage run's.
# MODE bytes (default): the launcher's way -- byte ranges size*k/N, moved to line starts by
# the CLI (--byte-range), no prefix scan.  MODE lines: the reference's line windows, found
# through the cached sparse line index (the line count pass builds it).
# Prints every process's peak RSS, wall time, spill size and the map job's split:
# window (finding its bytes) / setup (engine construction) / run (read + map + combine).
# Usage: bash tools/gpu_stage10g.sh TAG [GIB] [WINDOWS] [REDUCERS] [MODE]
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-stage10g}
G=${2:-10}
N=${3:-8}
R=${4:-3}
MODE=${5:-bytes}
mkdir -p $O
D=/tmp/locust_stage_$$
F=$D/big.txt
mkdir -p $D
export LOCUST_CACHE_DIR=$D/cache
trap 'rm -rf $D' EXIT
timeout -k 10 300 ./build/MapReduce --gen $F --gen-bytes $((G<<30)) --seed 7 > $O/gen.txt
S=$(stat -c %s $F)
if [ "$MODE" = lines ]; then
  t0=$(date +%s.%N)
  L=$(python3 -c "import locust_amd as l; print(l._C.find_line_window('$F', 0, -1)[2])")
  t1=$(date +%s.%N)
  echo "$G GiB, $L lines (counted in $(python3 -c "print('%.2f' % ($t1-$t0))") s), $N line windows, $R reducers" | tee $O/summary.txt
else
  echo "$G GiB ($S bytes), $N byte windows, $R reducers" | tee $O/summary.txt
fi
# the single stage three times (its engine setup alone varied 27-170 ms between runs):
# the comparison takes the median job
for i in 0 1 2; do
  t0=$(date +%s.%N)
  timeout -k 10 300 ./build/MapReduce $F --json $O/single$i.json > $D/single.out
  t1=$(date +%s.%N)
  python3 -c "import json,sys; d=json.load(open('$O/single$i.json')); s=d['startup']; print('single stage %d: %.2f s process, job %.1f ms (engine %.1f, read %.1f, first job %.1f), peak RSS %d kB, unique %d' % ($i, $t1-$t0, s['engine_ms']+s['read_ms']+s['first_job_ms'], s['engine_ms'], s['read_ms'], s['first_job_ms'], d['max_rss_kb'], d['unique']))" | tee -a $O/summary.txt
done
grep "^print key:" $D/single.out > $D/single.lines
INPUTS=""
for k in $(seq 0 $((N-1))); do
  if [ "$MODE" = lines ]; then
    s=$((L*k/N)); e=$((L*(k+1)/N)); W="$s $e"; RANGE=""
  else
    a=$((S*k/N)); b=$((S*(k+1)/N)); W="0 0"; RANGE="--byte-range $a:$b"
  fi
  t0=$(date +%s.%N)
  timeout -k 10 300 ./build/MapReduce $F $W $k 1 $RANGE --spill-dir $D --spill-format binary --json $O/map$k.json > $O/map$k.out
  t1=$(date +%s.%N)
  python3 -c "import json; d=json.load(open('$O/map$k.json')); print('map %d bytes [%d, %d): %.2f s process, job %.1f ms (window %.1f, setup %.1f, run %.1f), map %.1f ms, streamed %s, spill %d B (%d records), peak RSS %d kB' % ($k, d['byte_begin'], d['byte_end'], $t1-$t0, d['job_ms'], d['window_ms'], d['setup_ms'], d['run_ms'], d['map_ms'], d['streamed'], d['spill_bytes'], d['spill_records'], d['peak_rss_kb']))" | tee -a $O/summary.txt
  INPUTS="$INPUTS${INPUTS:+,}$D/out.$k.kv"
done
python3 - $O $N <<'PY' | tee -a $O/summary.txt
import json, statistics, sys
o, n = sys.argv[1], int(sys.argv[2])
jobs = [json.load(open(f"{o}/map{k}.json"))["job_ms"] for k in range(n)]
singles = []
for i in range(3):
    st = json.load(open(f"{o}/single{i}.json"))["startup"]
    singles.append(st["engine_ms"] + st["read_ms"] + st["first_job_ms"])  # a map's job_ms parts
single = statistics.median(singles)
med = statistics.median(jobs)
print("maps: median %.1f ms, spread %.2f..%.2f of median, sum %.1f ms; single-stage job median %.1f ms, sum/single %.2f"
      % (med, min(jobs) / med, max(jobs) / med, sum(jobs), single, sum(jobs) / single))
PY
t0=$(date +%s.%N)
timeout -k 10 300 ./build/MapReduce $F 0 0 0 2 --inputs $INPUTS --json $O/reduce.json > $D/reduce.out
t1=$(date +%s.%N)
grep "^print key:" $D/reduce.out > $D/reduce.lines
python3 -c "import json; d=json.load(open('$O/reduce.json')); print('reduce: %.2f s process, runtime init %.1f ms, read %.1f ms, setup %.1f ms, merge %.1f ms, records %d, peak RSS %d kB' % ($t1-$t0, d['runtime_init_ms'], d['read_ms'], d['setup_ms'], d['merge_ms'], d['input_records'], d['peak_rss_kb']))" | tee -a $O/summary.txt
cmp $D/single.lines $D/reduce.lines && echo "stage split == single stage ($(wc -l < $D/single.lines) lines)" | tee -a $O/summary.txt
rm -f $D/ranges.lines
for r in $(seq 0 $((R-1))); do
  timeout -k 10 300 ./build/MapReduce $F 0 0 $r 2 --inputs $INPUTS --reducer $r/$R --result-file $D/res.$r --json $O/reducer$r.json > /dev/null
  cat $D/res.$r >> $D/ranges.lines
  python3 -c "import json; d=json.load(open('$O/reducer$r.json')); print('reducer $r/$R: records read %d, merged %d, val base %d, read %.1f ms, setup %.1f ms, merge %.1f ms, peak RSS %d kB' % (d['records_read'], d['input_records'], d['val_base'], d['read_ms'], d['setup_ms'], d['merge_ms'], d['peak_rss_kb']))" | tee -a $O/summary.txt
done
cmp $D/single.lines $D/ranges.lines && echo "$R key-range reducers == single stage" | tee -a $O/summary.txt
