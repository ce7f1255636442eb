set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6j2
mkdir -p $O
D=/tmp/locust_r6j_$$
mkdir -p $D
trap 'rm -rf $D' EXIT
timeout -k 10 120 ./build/MapReduce --gen $D/a.txt --gen-bytes $((1280<<20)) --seed 7 > /dev/null
sync
prof() {  # TAG args...
  local tag=$1; shift
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/p_$tag -o t -- $GRAFT_REPO_ROOT/build/MapReduce "$@" > /dev/null 2>&1
  cd $GRAFT_REPO_ROOT
  K=$(find $O/p_$tag -name "*kernel_trace.csv" | head -1)
  C=$(find $O/p_$tag -name "*memory_copy_trace.csv" | head -1)
  cp $K $O/$tag.kernels.csv; cp $C $O/$tag.copies.csv; rm -rf $O/p_$tag
  echo "== $tag"
  python3 tools/stream_windows.py $O/$tag.kernels.csv $O/$tag.copies.csv --first 3
}
prof single1 $D/a.txt --json $O/single1.json
prof map1 $D/a.txt 0 0 0 1 --byte-range 0: --spill-dir $D --spill-format binary --json $O/map1.json
prof single2 $D/a.txt --json $O/single2.json
prof map2 $D/a.txt 0 0 0 1 --byte-range 0: --spill-dir $D --spill-format binary --json $O/map2.json
gzip -f $O/*.csv
