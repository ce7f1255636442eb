# Every bench config on one box: headline (with its side measurements), synth1m, synth10g.
# Usage: bash tools/gpu_bench_all.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-ball}
mkdir -p $O
timeout -k 10 300 python bench.py > $O/headline.json 2> $O/headline.err || { tail -20 $O/headline.err; exit 1; }
cut -c1-300 $O/headline.json
timeout -k 10 300 python bench.py --config synth1m --steps 50 --warmup 5 > $O/synth1m.json 2> $O/synth1m.err || { tail -20 $O/synth1m.err; exit 1; }
cut -c1-300 $O/synth1m.json
timeout -k 10 400 python bench.py --config synth10g --steps 3 --warmup 1 > $O/synth10g.json 2> $O/synth10g.err || { tail -20 $O/synth10g.err; exit 1; }
cut -c1-300 $O/synth10g.json
