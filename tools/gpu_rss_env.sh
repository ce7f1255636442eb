# HIP runtime host RSS under runtime knobs (tools/rss_probe.hip), then the CLI's RSS.
# Usage: bash tools/gpu_rss_env.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-rss_env}
mkdir -p $O
for env in "" "HSA_KERNARG_POOL_SIZE=1048576" "ROC_AQL_QUEUE_SIZE=1024" "GPU_STAGING_BUFFER_SIZE=1" \
           "GPU_PINNED_XFER_SIZE=1 GPU_PINNED_MIN_XFER_SIZE=1" "GPU_XFER_BUFFER_SIZE=1" \
           "ROC_SIGNAL_POOL_SIZE=64" "GPU_MAX_HW_QUEUES=1" "HIP_INITIAL_DM_SIZE=0" \
           "GPU_BLIT_ENGINE_TYPE=1" "GPU_BLIT_ENGINE_TYPE=2"; do
  echo "== env: ${env:-default}" >> $O/probe.txt
  env $env timeout -k 10 60 ./build/rss_probe >> $O/probe.txt 2>&1
done
