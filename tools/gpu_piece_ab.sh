# synth1m vs the middle upload piece size (LOCUST_PIECE_MB), separate processes, alternating.
# Usage: bash tools/gpu_piece_ab.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-piece}
mkdir -p $O
for r in 1 2 3 4 5; do
  for mb in ${PIECES:-8 10 12 16}; do
    LOCUST_PIECE_MB=$mb timeout -k 10 200 python bench.py --config synth1m --steps 100 --warmup 10 --no-extra > $O/p${mb}_$r.json 2> $O/p${mb}_$r.err || { tail -20 $O/p${mb}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/p${mb}_$r.json'));print('piece $mb MiB round $r:', d['ms_per_step'])"
  done
done
