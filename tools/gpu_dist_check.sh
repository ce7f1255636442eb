# Distributed GPU tests + the synth1m rehearsals (RCCL 1 rank: local and forced exchange).
# Usage: bash tools/gpu_dist_check.sh TAG
set -e
cd $GRAFT_REPO_ROOT
T=${1:-dchk}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "dist or multi or large_ordered or stream" --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
bash tools/gpu_dist_synth.sh $T
